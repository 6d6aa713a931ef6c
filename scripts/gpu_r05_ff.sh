# Paired step-graph instances (HVAE_GRAPH_PAIR=1: replay two executable copies in turn) against one instance, at
# Syn-1M (K = 1 and 4 steps per graph) and Syn-10M (K = 1), two interleaved rounds; the graph = eager tests with
# the pair; a kernel trace of Syn-1M with the pair at K = 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05ff
mkdir -p $O
HVAE_GRAPH_PAIR=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_train.py -k "graph" > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 3; }
tail -2 $O/pytest_pair.log
for round in 1 2; do
  for arm in syn1m:1:0 syn1m:1:1 syn1m:4:0 syn1m:4:1 syn10m:1:0 syn10m:1:1; do
    IFS=: read wl k pair <<< "$arm"
    HVAE_GRAPH_PAIR=$pair HVAE_STEPS_PER_GRAPH=$k timeout -k 10 240 python -u bench.py --workload $wl --steps 48 --warmup 16 \
      --no-cpu-baseline --probe-steps 8 > $O/bench_${wl}_k${k}_p$pair.json 2>> $O/bench.log || exit 4
    python3 -c "
import json; d=json.loads(open('$O/bench_${wl}_k${k}_p$pair.json').read().strip().split(chr(10))[-1])
print(json.dumps({'workload': '$wl', 'steps_per_graph': $k, 'pair': $pair, 'round': $round, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> $O/pair.jsonl
  done
done
cat $O/pair.jsonl
cd /tmp && export TMPDIR=/tmp
HVAE_GRAPH_PAIR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/syn1m_pair -o run -- \
  python3 $R/bench.py --workload syn1m --steps 200 --warmup 16 --no-cpu-baseline --probe-steps 4 > $R/$O/syn1m_pair.log 2>&1 || exit 5
grep '"metric"' $R/$O/syn1m_pair.log | cut -c1-200
