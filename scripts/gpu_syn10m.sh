# Kernel + train-step parity tests, then the Syn-10M (d = 768) and Syn-1M benches on one GPU.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
timeout -k 10 600 python -u bench.py --workload syn10m --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/bench_syn10m.log 2>&1
timeout -k 10 400 python bench.py --workload syn1m --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m.log 2>&1
