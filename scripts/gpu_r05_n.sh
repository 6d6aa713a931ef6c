#!/bin/bash
# fp8 version-5 sweep: DEC5_EXPPOLY8 (of 8) exponential pairs per producer lane and tile on the packed polynomial
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05n
out=gpurun_out/r05n/dec5_f8_exppoly.jsonl
: > $out
HVAE_LIB=build_var/libhvae_d5f8ep8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -x -q \
  --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r05n/test.log || exit 1
for r in 1 2; do
  for v in prod d5f8ep2 d5f8ep4 d5f8ep8; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --dtype fp8 \
      --reps 10 2>gpurun_out/r05n/err_$v.log | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" | tee -a $out || exit 1
  done
done
