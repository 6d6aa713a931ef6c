# Round-3 session tests: DP drop-in, top-K (eps bound, extent), the A/B variant's checks, full-shape step vs oracle.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_t1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_dp_dropin.py tests/test_gpu_ab_variant.py tests/test_gpu_topk.py tests/test_gpu_recommend.py tests/test_gpu_dp.py tests/test_gpu_fp8.py > $O/pytest_a.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_large_step.py > $O/pytest_b.log 2>&1
