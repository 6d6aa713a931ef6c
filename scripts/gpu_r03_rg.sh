# Row-gradient apply with 16-B sc1 partials and a last-taker acquire (was an acq_rel ticket), GEMM split-K partials
# in fragment order with 16-B sc1 stores: their GPU tests, the Syn-1M and Syn-10M bench lines, a rocprofv3 kernel
# trace of the Syn-1M bench (graph-mode step timeline), the make-tune per-config wall time (All_Beauty stand-in).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_rg}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_dp.py > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log
timeout -k 10 400 python -u scripts/bench_tune.py --epochs 10 --configs 2 > $O/tune.jsonl 2> $O/tune.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload syn1m --steps 50 --warmup 10 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
