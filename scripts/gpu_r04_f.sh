#!/bin/bash
# round 4 pass f: the GEMMs with the staging depth per instantiation (ring of 4 k-tiles for long K, 2 blocks per
# CU) -- parity and shapes; then pass e's content
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04f
mkdir -p $O
echo "gemm tests"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_kernels.py -k "gemm or colsum" \
  > $O/pytest_gemm.log 2>&1
rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
echo "gemm shapes"
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 --no-torch > $O/gemm_syn10m.jsonl 2> $O/gemm_syn10m.log || exit 5
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 384 --reps 50 --no-torch > $O/gemm_syn1m.jsonl 2> $O/gemm_syn1m.log || exit 5
cut -c1-200 $O/gemm_syn10m.jsonl $O/gemm_syn1m.jsonl
echo "dp tests (CSR-only first exchange)"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_dp_dropin.py \
  > $O/pytest_dp.log 2>&1
rc=$?; tail -4 $O/pytest_dp.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_e.sh
