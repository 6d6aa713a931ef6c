# Round 6, call B: whole-step A/B at B = 4096 (scripts/bench_step_ab.py, one dataset per workload, arms on fresh
# trainers, interleaved): steps per graph replay (HVAE_STEPS_PER_GRAPH 1 | 8) x where the row-gradient plan forks
# off the main stream (HVAE_PLAN_FORK late | early), at Syn-1M and the Syn-10M shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06b
mkdir -p $O
cd $R
for wl in syn1m syn10m; do
  timeout -k 10 500 python -u scripts/bench_step_ab.py --workload $wl --rounds 2 --steps 120 --warmup 24 \
    --arm base: --arm k8:HVAE_STEPS_PER_GRAPH=8 --arm early:HVAE_PLAN_FORK=early \
    --arm k8early:HVAE_STEPS_PER_GRAPH=8,HVAE_PLAN_FORK=early >> $O/step_ab.jsonl 2>> $O/step_ab.err || exit 1
done
echo done > $O/done
