#!/bin/bash
# version-5 bf16 sweep: DEC5_EXPPOLY (of 4) exponential pairs per producer lane and tile on a packed-f32 polynomial
# exp2 (v_pk_fma_f32) instead of v_exp_f32, vs the product build; parity of the all-polynomial build first
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05m
out=gpurun_out/r05m/dec5_exppoly.jsonl
: > $out
HVAE_LIB=build_var/libhvae_d5ep4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "d768" -x -q \
  --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r05m/test.log || exit 1
for r in 1 2; do
  for v in prod d5ep1 d5ep2 d5ep4; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 \
      2>gpurun_out/r05m/err_$v.log | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" | tee -a $out || exit 1
  done
done
