# Round 6, call N: the early catch-up placed after the sweep (HVAE_EARLY_AT=sweep, beside the finalize and the
# backward) instead of after the plan (call M: its blocks held CUs the sweep wanted). Was: call M, the next batch's catch-up run early (HVAE_EARLY_CATCHUP=1, hvae_adam_lazy_catchup_early):
# bitwise tests, then bench A/B against the plain catch-up and the deferred update at Syn-1M and the Syn-10M shard,
# and a kernel trace of the Syn-1M step with it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "early_catchup or deferred" > $O/pytest_early.log 2>&1 || exit 1
ab() {  # arm workload precision
  local arm=$1 wl=$2 pr=$3 d=0 e=0
  [ $arm = defer ] && d=1; [ $arm = early ] && e=1
  HVAE_ADAM_DEFER=$d HVAE_EARLY_CATCHUP=$e timeout -k 10 300 python -u bench.py --workload $wl --precision $pr \
    --steps 150 --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'arm':'$arm','workload':'$wl','precision':'$pr','ms':d['ms_per_step'],'value':d['value']}))" >> $O/early_ab.jsonl || exit 2
}
for r in 1 2; do
  for arm in off early; do ab $arm syn1m bf16; done
done
for r in 1 2; do
  for arm in defer early; do ab $arm syn10m fp8; done
done
cd /tmp && export TMPDIR=/tmp
HVAE_EARLY_CATCHUP=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn1m -o run -- \
  python3 $R/bench.py --workload syn1m --steps 150 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_syn1m.log 2>&1 || exit 3
cd $R
python3 scripts/step_timeline.py $(find $O/kt_syn1m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn1m.txt || exit 4
echo done > $O/done
