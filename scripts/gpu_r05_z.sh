#!/bin/bash
# decoder finalize (16-B form): CSR entries per load batch 16 (product) / 8 / 4 (variant builds), train form,
# Syn-1M and Syn-10M shapes
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05z
out=gpurun_out/r05z/fin_eb.jsonl
: > $out
for r in 1 2; do
  for v in prod fineb8 fineb4; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    for shp in "--N 100000 --D 384" "--N 1000000 --D 768"; do
      HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 $shp --train --probe decoder_finalize \
        --reps 10 2>>gpurun_out/r05z/err.log | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" | tee -a $out || exit 1
    done
  done
done
