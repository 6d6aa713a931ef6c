# Round 6, call G: the fused trainable-E step against the oracle (small shapes, Syn-1M) and the trainer tests;
# whole-step A/Bs at B = 4096: weight-gradient GEMMs on a second stream (HVAE_TWO_STREAMS=1) and the plan joined
# before the sweep (HVAE_PLAN_JOIN=sweep).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_trainable_embeddings.py -m gpu -x -v -s --timeout 850 \
  --timeout-method thread > $O/pytest_trainE.log 2>&1 || exit 1
for wl in syn1m syn10m; do
  timeout -k 10 600 python -u scripts/bench_step_ab.py --workload $wl --rounds 2 --steps 120 --warmup 24 \
    --arm base: --arm two:HVAE_TWO_STREAMS=1 --arm joinsweep:HVAE_PLAN_JOIN=sweep >> $O/step_ab.jsonl 2>> $O/step_ab.err || exit 2
done
echo done > $O/done
