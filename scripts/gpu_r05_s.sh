# LDS-DMA GEMM path: parity (GEMM + MLP + train-step tests), then a kernel trace of the Syn-10M shapes with the
# A/B library's HVAE_GEMM_DMA=1 / 0 (one process each) beside torch.mm
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" tests/test_gpu_mlp_rows.py -x -q \
  --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_GEMM_DMA=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d $O/tr$v -o run -- python3 $R/scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 > $O/bench_gemm_$v.log 2>&1
  grep -c hvae_us $O/bench_gemm_$v.log
done
