# Round-end check of the final tree: every GPU test, the driver's smoke(), the default bench with the CPU
# baseline and its rocprofv3 kernel-trace stats, and the Syn-1M fp8 line.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final2/pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final2/bench.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --precision fp8 --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/final2/bench_syn1m_fp8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final2/prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu-baseline --probe-steps 5 > $R/gpurun_out/final2/prof.log 2>&1
