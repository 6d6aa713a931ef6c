#!/bin/bash
# round 4 pass b: DP per-rank-shard validation, Adam (hardware sqrt / rcp) train-step parity, and the
# consumer-softmax d = 768 sweep (DEC5_CSM): parity against float64 and an interleaved A/B at the Syn-10M shard
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04b
mkdir -p $O
R=$GRAFT_REPO_ROOT
echo "csm parity" && HVAE_LIB=$R/build_var/libhvae_csm.so timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_large.py -k "768" > $O/pytest_csm.log 2>&1
rc=$?; tail -4 $O/pytest_csm.log; [ $rc -eq 0 ] || exit $rc
echo "csm A/B"
for round in 1 2; do
  for a in base csm; do
    lib=$R/build_var/libhvae_$a.so; [ $a = base ] && lib=$R/recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --ab DUMMY=$a --rounds 1 >> $O/csm_ab.jsonl 2>> $O/csm_ab.log || exit 3
  done
done
cat $O/csm_ab.jsonl
echo "dp" && timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_dp.py::test_dp_two_ranks_one_gpu" > $O/pytest_dp2.log 2>&1
rc=$?; tail -3 $O/pytest_dp2.log; [ $rc -eq 0 ] || exit $rc
echo "train" && timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_mlp_rows.py tests/test_gpu_train.py tests/test_gpu_large_step.py tests/test_gpu_trainable_embeddings.py \
  tests/test_gpu_kernels.py -k "adam or clip or lazy or train or mlp or trainable or large_step" > $O/pytest_train.log 2>&1
rc=$?
tail -15 $O/pytest_train.log
exit $rc
