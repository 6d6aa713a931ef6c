# Version 4 anatomy at the Syn-10M shard shape: DMA placement, GEMM1 read-ahead, and timing ablations
# (no DMA, no barrier, no softmax; results of the ablation builds are invalid).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v4abl
mkdir -p $O
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for r in 1 2; do
for v in base d4dma1 d4dma2 d4g1a4 d4abl1 d4abl2 d4abl3; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
done
