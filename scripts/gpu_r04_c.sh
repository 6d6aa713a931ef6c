#!/bin/bash
# round 4 pass c: bench lines after the hardware-sqrt Adam, the W = 8 rank-step emulation, decoder split A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c
mkdir -p $O
R=$GRAFT_REPO_ROOT
echo "bench syn10m"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log || exit 3
cut -c1-400 $O/bench_syn10m.json
echo "dp emul"
timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 1 8 --steps 20 --warmup 6 > $O/dp_emul.jsonl 2> $O/dp_emul.log || exit 4
cat $O/dp_emul.jsonl
echo "splits"
for round in 1 2; do
  HVAE_LIB=$R/build_var/libhvae_ab.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 \
    --ab HVAE_DEC_SPLITS=4 HVAE_DEC_SPLITS=8 HVAE_DEC_SPLITS=16 --rounds 1 >> $O/splits_ab.jsonl 2>> $O/splits_ab.log || exit 5
done
cat $O/splits_ab.jsonl
echo "bench syn1m"
timeout -k 10 300 python -u bench.py --workload syn1m --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log || exit 6
cut -c1-300 $O/bench_syn1m.json
echo "bench all_beauty"
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline > $O/bench_ab.json 2> $O/bench_ab.log || exit 7
cut -c1-300 $O/bench_ab.json
