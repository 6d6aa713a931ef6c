# Round 6, call P3: the forward chain with its column tiles rotated per block (L2 channel camping) -- variants e..h =
# (threads, chunks ahead) 512x4, 512x8, 256x4, 1024x4 with rotation, c = 512x4 without -- standalone at d = 384 / 768.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p3
mkdir -p $O
cd $R
for v in c e f g h; do
  HVAE_LIB=build_var/libhvae_ch$v.so timeout -k 10 200 python -u scripts/bench_chain.py --reps 100 --tag ch$v >> $O/chain_variants.jsonl 2>> $O/err.log || exit 2
done
echo done > $O/done
