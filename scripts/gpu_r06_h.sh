# Round 6, call H: the weight-gradient GEMMs on a second stream (HVAE_WGRAD_SIDE=1) -- whole-step A/B at Syn-1M and
# the Syn-10M shard (bf16, fp8) and the full-shape train-step parity with it on.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06h
mkdir -p $O
cd $R
for a in "syn1m bf16" "syn10m bf16" "syn10m fp8"; do
  set -- $a
  timeout -k 10 600 python -u scripts/bench_step_ab.py --workload $1 --precision $2 --rounds 2 --steps 120 --warmup 24 \
    --arm base: --arm wside:HVAE_WGRAD_SIDE=1 >> $O/step_ab.jsonl 2>> $O/step_ab.err || exit 1
done
HVAE_WGRAD_SIDE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_large_step.py -m gpu -x -v -s --timeout 850 \
  --timeout-method thread > $O/pytest_large_wside.log 2>&1 || exit 2
echo done > $O/done
