#!/bin/bash
# round 4: the parity gaps and the ADVICE r3 fixes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_topk.py tests/test_gpu_recommend.py tests/test_gpu_dp.py tests/test_gpu_mlp_rows.py \
  > gpurun_out/r04/pytest_parity.log 2>&1
rc=$?
tail -30 gpurun_out/r04/pytest_parity.log
exit $rc
