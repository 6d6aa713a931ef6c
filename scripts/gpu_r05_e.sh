#!/bin/bash
# version-6 sweep anatomy: timing-ablation builds (DEC6_ABL, outputs invalid by construction), each arm its own
# process, two interleaved rounds, Syn-10M shard 4096 x 1M x 768
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05e
out=gpurun_out/r05e/dec6_ablation.jsonl
: > $out
for r in 1 2; do
  for a in 0 1 128 4 260 287; do
    HVAE_LIB=build_var/libhvae_d6abl$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 \
      --D 768 --reps 10 2>/dev/null | sed "s/\"arm\": \"\"/\"arm\": \"DEC6_ABL=$a\"/" | tee -a $out || exit 1
  done
done
