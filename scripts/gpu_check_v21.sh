# Tree check after the GEMM tile and split-K changes: every GPU test, smoke(), the default bench and the Syn-1M fp8
# rocprofv3 kernel stats.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/v21
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v21/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v21/smoke.log 2>&1
timeout -k 10 200 python bench.py > gpurun_out/v21/bench.log 2>&1
timeout -k 10 200 python scripts/bench_gemm.py --batch 4096 --reps 50 > gpurun_out/v21/gemm4096.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/v21/p -o run -- python3 $R/bench.py --workload syn1m --precision fp8 --steps 40 --warmup 3 --no-cpu-baseline --probe-steps 2 > $R/gpurun_out/v21/p.log 2>&1
