# v3 (dh-specialised loop): correctness at d = 768, then DMA pre-issue count A/B (3 = shipped, 0, 6).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pre
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_large.py tests/test_gpu_kernels.py -q -x -k "768" --timeout 200 --timeout-method thread > $O/t.log 2>&1
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for r in 1 2; do
for v in base pre0 pre6; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
done
