# Train-step pins (bf16 / fp8 vs golden G2, validate loss vs G1, resume, lr change) with their measured
# deviations printed, then every GPU test on the new default decoder (barrier B after GEMM2's own half).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pins
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_api.py -v -s --timeout 200 --timeout-method thread > $O/pins.log 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
