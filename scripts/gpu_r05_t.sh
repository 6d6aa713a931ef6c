# LDS-DMA GEMM tuning at the Syn-10M shapes (kernel traces): ring depth 2 / 3 / 4 (variant builds), and the
# weight gradients' split count (A/B library, HVAE_GEMM_FAST_SPLITS)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 \
    $R/scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 --no-torch > $O/$n.log 2>&1
  python3 $R/scripts/gemm_trace_summary.py $O/$n/run_kernel_trace.csv > $O/$n.jsonl
  echo "== $n"; cat $O/$n.jsonl
}
run dns3 HVAE_LIB=$R/build_var/libhvae_ab.so
run dns4 HVAE_LIB=$R/build_var/libhvae_gdns4.so
run dns2 HVAE_LIB=$R/build_var/libhvae_gdns2.so
run split2 HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_GEMM_FAST_SPLITS=2
run split8 HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_GEMM_FAST_SPLITS=8
run tile32 HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_GEMM_DMA_TILE=32
