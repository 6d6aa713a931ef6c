# Version-5 decoder variants (build_var/libhvae_<v>.so from scripts/build_variant5.sh), each against version 4
# in the same process, at 4096 x 200,000 x 768.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5b
mkdir -p $O
cd $R
for V in ah4 dmab12 dmab6; do
  HVAE_LIB=$R/build_var/libhvae_$V.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 200000 --D 768 --reps 10 --rounds 2 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_$V.jsonl 2>&1
done
