#!/bin/bash
# round 5: version 5 vs version 6 of the d = 768 bf16 sweep in one process (Syn-10M shard), then the default bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05b
export PYTHONDONTWRITEBYTECODE=1
HVAE_LIB=build_var/libhvae_ab.so timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 \
  --reps 10 --rounds 2 --ab HVAE_DEC_V6=0 HVAE_DEC_V6=1 > gpurun_out/r05b/ab_v5_v6.jsonl 2>&1 || { tail -30 gpurun_out/r05b/ab_v5_v6.jsonl; exit 1; }
cat gpurun_out/r05b/ab_v5_v6.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/r05b/bench_syn10m.json 2> gpurun_out/r05b/bench_syn10m.err || { tail -20 gpurun_out/r05b/bench_syn10m.err; exit 1; }
cat gpurun_out/r05b/bench_syn10m.json
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_api.py::test_adam_dense_matches_torch_cpu" > gpurun_out/r05b/pytest_adam.log 2>&1; tail -3 gpurun_out/r05b/pytest_adam.log
