# Version-5 anatomy at the Syn-10M shard: timing-ablation builds (DEC5_ABL bit mask, outputs invalid by
# construction), two interleaved rounds, each arm in its own process.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_abl5
mkdir -p $O
cd $R
for round in 1 2; do
  for a in 0 1 2 4 8 16 24 25 31 32 64; do
    HVAE_LIB=$R/build_var/libhvae_abl$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --ab DUMMY=abl$a --rounds 1 >> $O/abl.jsonl 2>> $O/abl.log
  done
done
