#!/bin/bash
# version 5 vs version 6 bf16 d = 768 sweep, one process, interleaved rounds (A/B library), Syn-10M shard
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05j
HVAE_LIB=build_var/libhvae_ab.so timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
  --reps 10 --rounds 4 --ab HVAE_DEC_V6=0 HVAE_DEC_V6=1 2>gpurun_out/r05j/err.log | tee gpurun_out/r05j/ab_v5_v6.jsonl
