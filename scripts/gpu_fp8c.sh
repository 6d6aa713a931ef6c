# fp8 sweep iteration: parity tests, decoder microbench at d = 384 / 768, Syn-1M fp8 bench
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1
timeout -k 10 120 python scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 100000 --D 384 --reps 20 > gpurun_out/dec_fp8.log 2>&1
timeout -k 10 120 python scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 200000 --D 768 --reps 10 >> gpurun_out/dec_fp8.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --precision fp8 --steps 40 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m_fp8.log 2>&1
