# HIP graph-launch runtime knobs at Syn-1M (B = 4096, one graph per step): default, DEBUG_HIP_FORCE_GRAPH_QUEUES,
# DEBUG_CLR_GRAPH_PACKET_CAPTURE, DEBUG_HIP_GRAPH_BATCH_SIZE; two interleaved rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05hh
mkdir -p $O
for round in 1 2; do
  for arm in none FQ1 FQ2 PC0 PC1 BS1 BS64; do
    case $arm in
      none) envs="";; FQ1) envs="DEBUG_HIP_FORCE_GRAPH_QUEUES=1";; FQ2) envs="DEBUG_HIP_FORCE_GRAPH_QUEUES=2";;
      PC0) envs="DEBUG_CLR_GRAPH_PACKET_CAPTURE=0";; PC1) envs="DEBUG_CLR_GRAPH_PACKET_CAPTURE=1";;
      BS1) envs="DEBUG_HIP_GRAPH_BATCH_SIZE=1";; BS64) envs="DEBUG_HIP_GRAPH_BATCH_SIZE=64";;
    esac
    env $envs timeout -k 10 240 python -u bench.py --workload syn1m --steps 200 --warmup 20 --no-cpu-baseline \
      --probe-steps 8 > $O/bench_$arm.json 2>> $O/bench.log || { echo "arm $arm failed"; tail -5 $O/bench.log; exit 4; }
    python3 -c "
import json; d=json.loads(open('$O/bench_$arm.json').read().strip().split(chr(10))[-1])
print(json.dumps({'arm': '$arm', 'env': '$envs', 'round': $round, 'ms_per_step': d['ms_per_step'], 'value': d['value']}))" >> $O/knobs.jsonl
  done
done
cat $O/knobs.jsonl
