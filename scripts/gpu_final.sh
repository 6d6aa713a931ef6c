# Round-end evidence: every GPU test, the default bench (with the CPU baseline), Syn-1M and Syn-10M lines in
# bf16 and fp8, and rocprofv3 kernel-trace stats of the default and Syn-1M fp8 benches.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --steps 200 --warmup 10 --probe-steps 5 --no-cpu-baseline > gpurun_out/final/bench_syn1m.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --precision fp8 --steps 200 --warmup 10 --probe-steps 5 --no-cpu-baseline > gpurun_out/final/bench_syn1m_fp8.log 2>&1
timeout -k 10 400 python -u bench.py --workload syn10m --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/final/bench_syn10m.log 2>&1
timeout -k 10 400 python -u bench.py --workload syn10m --precision fp8 --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/final/bench_syn10m_fp8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --probe-steps 5 > $R/gpurun_out/final/prof.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof_syn8 -o run -- python3 $R/bench.py --workload syn1m --precision fp8 --steps 30 --warmup 3 --no-cpu-baseline --probe-steps 2 > $R/gpurun_out/final/prof_syn8.log 2>&1
