#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05c
timeout -k 10 120 python -u scripts/probe_dec6.py 4096 200000,1000000 2>&1 | tee gpurun_out/r05c/probe.log
HVAE_LIB=build_var/libhvae_ab.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
  --reps 10 --rounds 3 --ab HVAE_DEC_V6=0 HVAE_DEC_V6=1 2>&1 | tee gpurun_out/r05c/ab_v5_v6.jsonl
