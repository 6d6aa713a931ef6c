#!/bin/bash
# version-6 sweep after the operand-read re-schedule: parity first, then v5 / v6 product A/B and ablation arms
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05f
out=gpurun_out/r05f/dec6_ab.jsonl
: > $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "v6 or d768" -x -q --timeout 120 --timeout-method thread \
  2>&1 | tee gpurun_out/r05f/test.log || exit 1
for r in 1 2; do
  for v in 1 0; do
    HVAE_DEC_V6=$v timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 \
      2>gpurun_out/r05f/err_v$v.log | sed "s/\"arm\": \"\"/\"arm\": \"HVAE_DEC_V6=$v\"/" | tee -a $out || exit 1
  done
  for a in 1 8 16 24; do
    HVAE_LIB=build_var/libhvae_d6abl$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 \
      --D 768 --reps 10 2>gpurun_out/r05f/err_$a.log | sed "s/\"arm\": \"\"/\"arm\": \"DEC6_ABL=$a\"/" | tee -a $out || exit 1
  done
done
