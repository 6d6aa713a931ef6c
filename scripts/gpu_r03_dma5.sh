# Version-5 LDS-DMA placement and register staging A/B at the Syn-10M shard (build_var/libhvae_<arm>.so), three
# interleaved rounds, one process per arm and round.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_dma5
mkdir -p $O
cd $R
for round in 1 2 3; do
  for a in ${ARMS:-abl0 pdma7 pdma13 cdma12 rst6 rst8 rst6c12}; do
    HVAE_LIB=$R/build_var/libhvae_$a.so timeout -k 10 60 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --ab DUMMY=$a --rounds 1 >> $O/ab.jsonl 2>> $O/ab.log
  done
done
