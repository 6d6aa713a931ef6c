# Syn-1M (configs[2]) bench lines (bf16, fp8) and the rocprofv3 kernel stats of the bf16 one.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/syn1m
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_bf16.log 2>&1
timeout -k 10 400 python -u bench.py --workload syn1m --precision fp8 --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_fp8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload syn1m --steps 100 --warmup 10 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
