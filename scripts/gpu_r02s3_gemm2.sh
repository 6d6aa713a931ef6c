# Weight-gradient GEMMs on the fast path + look-back rowgrad scan: parity tests, per-shape GEMM timings,
# and step-level A/B (HVAE_GEMM_FAST=0 = the register-staged kernel everywhere) at Syn-1M and Syn-10M.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gemm2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_api.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d 384 --no-torch > $O/gemm384.jsonl 2>&1
timeout -k 10 120 python -u scripts/bench_gemm.py --batch 4096 --d 768 --no-torch > $O/gemm768.jsonl 2>&1
for F in 1 0; do
  HVAE_GEMM_FAST=$F timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/syn1m_fast$F.json 2> $O/syn1m_fast$F.log
done
for F in 1 0; do
  HVAE_GEMM_FAST=$F timeout -k 10 400 python -u bench.py --steps 40 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/syn10m_fast$F.json 2> $O/syn10m_fast$F.log
done
