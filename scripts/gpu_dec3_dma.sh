# v3 LDS-DMA placement A/B at the Syn-10M shard shape (separate libraries, interleaved processes) + d768 tests.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dma
mkdir -p $O
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for r in 1 2; do
for v in base dma1 dma2; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
done
for v in dma1 dma2; do
  env HVAE_LIB=$R/build_var/libhvae_$v.so timeout -k 10 300 python -m pytest tests/test_gpu_large.py -q -x -k "v3_matches or 4096-1000000-768-bf16" --timeout 200 --timeout-method thread > $O/t_$v.log 2>&1
done
