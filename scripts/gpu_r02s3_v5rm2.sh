# Version 5 (conflict-free GEMM1 row map) against version 4 in one process at the Syn-10M shard, 4 interleaved
# rounds per arm pair: DEC5_DMA_B = 5, 6, 7 (consumer's share of the 12 LDS-DMA pieces).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5rm2
mkdir -p $O
cd $R
for V in dmab6 dmab5 dmab7 dmab6; do
  HVAE_LIB=$R/build_var/libhvae_$V.so timeout -k 10 240 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 4 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 >> $O/ab_$V.jsonl 2>&1
done
