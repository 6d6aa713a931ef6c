# Grid-search (src/ml/tune.py) GPU tests.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tune.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_tune.log 2>&1
