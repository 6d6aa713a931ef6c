# Top-K edge tests, then the Syn-1M (bf16) rocprofv3 kernel stats for the non-decoder step breakdown.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s1m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -q --timeout 200 --timeout-method thread > $O/tk_edge.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload syn1m --steps 100 --warmup 10 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
