set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -m gpu -x -s -v --timeout 240 --timeout-method thread > gpurun_out/pytest_dp.log 2>&1
