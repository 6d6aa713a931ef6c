# Fast-path fp32 GEMM: parity tests, then per-shape timings at B = 4096 (d = 384, 768) with the planner's
# tile and with every instantiated tile forced (HVAE_GEMM_FAST_TILE), and the old kernels (HVAE_GEMM_FAST=0).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemmfast
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_dp.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for D in 384 768; do
  timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $D --no-torch > $O/plan_$D.jsonl 2>&1
  HVAE_GEMM_FAST=0 timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $D --no-torch > $O/old_$D.jsonl 2>&1
  for T in 32x32 32x64 64x32 64x64 64x96 64x128 64x192; do
    HVAE_GEMM_FAST_TILE=$T timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d $D --no-torch > $O/t${T}_$D.jsonl 2>&1
  done
done
