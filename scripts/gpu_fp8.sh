# fp8 decoder: parity tests, then Syn-1M bench with the fp8 sweep beside the bf16 one
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --precision fp8 --steps 40 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m_fp8.log 2>&1
