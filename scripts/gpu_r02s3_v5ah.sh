# Version 5 GEMM1 read-ahead (DEC5_G1_AHEAD 1 / 3 variants against the default 2), each against version 4 in the
# same process at the Syn-10M shard.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5ah
mkdir -p $O
cd $R
timeout -k 10 240 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 3 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_ah2.jsonl 2>&1
for V in ah1 ah3; do
  HVAE_LIB=$R/build_var/libhvae_$V.so timeout -k 10 240 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 3 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_$V.jsonl 2>&1
done
