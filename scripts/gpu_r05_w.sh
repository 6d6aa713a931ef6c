# LDS-DMA GEMM tile choice per shape (A/B library, kernel traces): default rule vs forced 64 x 32 / 64 x 64, d = 768 / 384
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for d in 768 384; do
  for t in def 6432 64; do
    env HVAE_LIB=$R/build_var/libhvae_ab.so $( [ $t != def ] && echo HVAE_GEMM_DMA_TILE=$t ) timeout -k 10 300 \
      rocprofv3 --kernel-trace --output-format csv -d $O/d${d}_$t -o run -- python3 $R/scripts/bench_gemm.py \
      --batch 4096 --d $d --reps 50 --no-torch > $O/d${d}_$t.log 2>&1
    python3 $R/scripts/gemm_trace_summary.py $O/d${d}_$t/run_kernel_trace.csv > $O/d${d}_$t.jsonl
  done
done
