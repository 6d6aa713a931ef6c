# Version-5 anatomy at the Syn-10M shard (4096 x 1M x 768): timing-ablation builds (DEC5_ABL bit mask, outputs
# invalid by construction) and static-priority A/B builds, interleaved rounds, each arm in its own process.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_abl5}
mkdir -p $O
cd $R
for round in 1 2; do
  for a in ${ARMS:-abl0 abl1 abl3 abl7 abl31 abl96 prio1 prio2}; do
    HVAE_LIB=$R/build_var/libhvae_$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --ab DUMMY=$a --rounds 1 >> $O/abl.jsonl 2>> $O/abl.log
  done
done
