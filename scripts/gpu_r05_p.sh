#!/bin/bash
# bench lines (bf16, fp8 at Syn-10M) after the probe's head-start hold: per-family launch_us vs the kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05p
for P in bf16 fp8; do
  timeout -k 10 300 python -u bench.py --precision $P --steps 100 --warmup 20 --no-cpu-baseline \
    > gpurun_out/r05p/bench_$P.json 2> gpurun_out/r05p/bench_$P.err || exit 1
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]);print(sys.argv[2],d['ms_per_step'],{k:v['avg_us'] for k,v in d['launch_us'].items()})" gpurun_out/r05p/bench_$P.json $P
done
