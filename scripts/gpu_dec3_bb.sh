# v3 barrier-B placement / GEMM2 read prefetch A/B at the Syn-10M shard shape (d = 768), after the
# d = 768 parity tests on the shipped build and on one variant.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bb
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_large.py tests/test_gpu_kernels.py -q -x -k "768" --timeout 200 --timeout-method thread > $O/t_base.log 2>&1
HVAE_LIB=$R/build_var/libhvae_bb8p1.so timeout -k 10 300 python -m pytest tests/test_gpu_large.py tests/test_gpu_kernels.py -q -x -k "768" --timeout 200 --timeout-method thread > $O/t_bb8p1.log 2>&1
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for r in 1 2; do
for v in base p1 bb8 bb8p1 bb4p1 bb11p1 bb8p2; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
done
