#!/bin/bash
# round 4: the 2-rank per-rank-shard validation test (hung silently in the first pass), the row-parallel MLP
# tests, and the train-step parity with the hardware sqrt / rcp Adam
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_dp.py::test_dp_two_ranks_one_gpu" > gpurun_out/r04/pytest_dp2.log 2>&1
rc=$?
tail -5 gpurun_out/r04/pytest_dp2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_mlp_rows.py tests/test_gpu_train.py tests/test_gpu_large_step.py tests/test_gpu_trainable_embeddings.py \
  > gpurun_out/r04/pytest_train.log 2>&1
rc=$?
tail -15 gpurun_out/r04/pytest_train.log
exit $rc
