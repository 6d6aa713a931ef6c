#!/bin/bash
# version-6 sweep: LDS-DMA pieces staggered by wave within a phase-1 step (DEC6_STAGGER 2 / 3) vs the product build;
# phase anatomy of the staggered builds
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05i
out=gpurun_out/r05i/dec6_stagger.jsonl
: > $out
for r in 1 2; do
  for v in prod d6st2 d6st3; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 \
      2>gpurun_out/r05i/err_$v.log | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" | tee -a $out || exit 1
  done
done
for v in d6tmst2 d6tmst3; do
  echo "== $v" | tee -a gpurun_out/r05i/phases.log
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 120 python -u scripts/probe_dec6_phases.py 2>gpurun_out/r05i/err_$v.log \
    | tee -a gpurun_out/r05i/phases.log || exit 1
done
