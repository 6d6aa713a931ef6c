# Version-5 decoder: LDS-DMA split between producer and consumer waves (DEC5_DMA_B pieces of 12 on the consumer),
# each variant against version 4 in the same process at the Syn-10M shard shape (4096 x 1,000,000 x 768).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5c
mkdir -p $O
cd $R
for V in dmab4 dmab5 dmab6 dmab7 dmab8 dmab6ah3; do
  HVAE_LIB=$R/build_var/libhvae_$V.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 2 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_$V.jsonl 2>&1
done
