# Round 6, call J: the deferred W1t update (HVAE_ADAM_DEFER=1, hvae_adam_lazy_defer / _pending /
# _catchup_csr_pending): bitwise tests against the undeferred update (single GPU, two ranks on one GPU), then bench
# A/B at Syn-1M and the Syn-10M shard (bf16, fp8), the pending rows moved beside the forward (fwd) or beside the
# finalize (sweep), and a kernel trace of the Syn-1M step with it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06j
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dp.py -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "deferred or lazy_adam_is_bitwise" > $O/pytest_defer.log 2>&1 || exit 1
ab() {  # arm workload precision
  local arm=$1 wl=$2 pr=$3 d=0 at=fwd
  [ $arm = fwd ] && d=1; [ $arm = sweep ] && { d=1; at=sweep; }
  HVAE_ADAM_DEFER=$d HVAE_DEFER_AT=$at timeout -k 10 300 python -u bench.py --workload $wl --precision $pr \
    --steps 150 --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'arm':'$arm','workload':'$wl','precision':'$pr','ms':d['ms_per_step'],'value':d['value']}))" >> $O/defer_ab.jsonl || exit 2
}
for r in 1 2; do
  for arm in off fwd sweep; do ab $arm syn1m bf16; done
done
for arm in off fwd sweep; do ab $arm syn10m bf16; done
for arm in off fwd sweep; do ab $arm syn10m fp8; done
cd /tmp && export TMPDIR=/tmp
HVAE_ADAM_DEFER=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn1m -o run -- \
  python3 $R/bench.py --workload syn1m --steps 150 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_syn1m.log 2>&1 || exit 3
cd $R
python3 scripts/step_timeline.py $(find $O/kt_syn1m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn1m.txt || exit 4
echo done > $O/done
