# Steps per graph replay (HVAE_STEPS_PER_GRAPH) at B = 4096: Syn-1M K = 1 (product) / 2 / 4 / 8, Syn-10M K = 1 / 4,
# two interleaved rounds; then a kernel trace of Syn-1M at K = 4 (the step boundary's idle gap)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05ee
mkdir -p $O
for round in 1 2; do
  for arm in syn1m:1 syn1m:2 syn1m:4 syn1m:8 syn10m:1 syn10m:4; do
    wl=${arm%%:*}; k=${arm##*:}
    HVAE_STEPS_PER_GRAPH=$k timeout -k 10 240 python -u bench.py --workload $wl --steps 48 --warmup 16 --no-cpu-baseline \
      --probe-steps 8 > $O/bench_${wl}_k$k.json 2>> $O/bench.log || exit 4
    python3 -c "
import json; d=json.loads(open('$O/bench_${wl}_k$k.json').read().strip().split(chr(10))[-1])
print(json.dumps({'workload': '$wl', 'steps_per_graph': $k, 'round': $round, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> $O/spg.jsonl
  done
done
cat $O/spg.jsonl
cd /tmp && export TMPDIR=/tmp
HVAE_STEPS_PER_GRAPH=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/syn1m_k4 -o run -- \
  python3 $R/bench.py --workload syn1m --steps 200 --warmup 16 --no-cpu-baseline --probe-steps 4 > $R/$O/syn1m_k4.log 2>&1 || exit 5
grep '"metric"' $R/$O/syn1m_k4.log | cut -c1-200
