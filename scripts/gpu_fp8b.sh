# fp8 decoder parity tests + Syn-10M (d = 768) and Syn-1M fp8 benches
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1
timeout -k 10 400 python -u bench.py --workload syn10m --precision fp8 --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/bench_syn10m_fp8.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --precision fp8 --steps 40 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m_fp8.log 2>&1
