#!/bin/bash
# version-6 sweep: LDS-DMA pieces moved into phase 2 (DEC6_DMAP = 4 / 6 / 12 of the 12) vs the product build (all in
# phase 1) and version 5 (A/B library); parity of the moved builds first
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05k
out=gpurun_out/r05k/dec6_dmap.jsonl
: > $out
for v in d6p6 d6p12; do
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "v6" -x -q \
    --timeout 120 --timeout-method thread 2>&1 | tee gpurun_out/r05k/test_$v.log || exit 1
done
for r in 1 2; do
  for v in prod d6p4 d6p6 d6p12 v5; do
    lib=build_var/libhvae_$v.so; env=""
    [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    [ $v = v5 ] && lib=build_var/libhvae_ab.so && env="HVAE_DEC_V6=0"
    env $env HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 \
      2>gpurun_out/r05k/err_$v.log | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" | tee -a $out || exit 1
  done
done
