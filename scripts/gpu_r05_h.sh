#!/bin/bash
# version-6 sweep phase anatomy (s_memtime timing builds): full sweep, no LDS-DMA, no softmax
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05h
for v in d6tm d6tm1 d6tm4; do
  echo "== $v" | tee -a gpurun_out/r05h/phases.log
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 120 python -u scripts/probe_dec6_phases.py 2>gpurun_out/r05h/err_$v.log \
    | tee -a gpurun_out/r05h/phases.log || exit 1
done
