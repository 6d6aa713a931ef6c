#!/bin/bash
# round 5, first run of the version-6 d = 768 bf16 sweep: parity, then v5 vs v6 in one process
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05a
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_kernels.py::test_decoder_bf16_d768_v6_tasks" "tests/test_gpu_kernels.py::test_decoder_bf16_d768" \
  "tests/test_gpu_kernels.py::test_decoder_train_fused_d768" "tests/test_gpu_api.py::test_adam_dense_matches_torch_cpu" > gpurun_out/r05a/pytest_v6.log 2>&1 || { tail -30 gpurun_out/r05a/pytest_v6.log; exit 1; }
tail -3 gpurun_out/r05a/pytest_v6.log
HVAE_LIB=build_var/libhvae_ab.so timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
  --reps 10 --rounds 2 --ab HVAE_DEC_V6=0 HVAE_DEC_V6=1 > gpurun_out/r05a/ab_v5_v6.jsonl 2>&1 || { tail -30 gpurun_out/r05a/ab_v5_v6.jsonl; exit 1; }
cat gpurun_out/r05a/ab_v5_v6.jsonl
