#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05d
timeout -k 10 120 python -u scripts/debug_dec6.py 96x32 96x320 4096x3200 4096x200000 2>&1 | tee gpurun_out/r05d/debug.log
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_kernels.py::test_decoder_bf16_d768_v6_tasks" 2>&1 | tee gpurun_out/r05d/pytest.log
HVAE_LIB=build_var/libhvae_ab.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
  --reps 10 --rounds 3 --ab HVAE_DEC_V6=0 HVAE_DEC_V6=1 2>&1 | tee gpurun_out/r05d/ab_v5_v6.jsonl
