# Round 6, call O: the large-batch forward chain on f32 MFMA (hvae_mlp_fwd_chain, csrc/hvae_chain.hip): its tests,
# the full-shape steps against the oracle with it, bench A/B against the GEMM chain, a Syn-1M kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_large_step.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest_chain.log 2>&1 || exit 1
ab() {  # arm workload precision
  local arm=$1 wl=$2 pr=$3 c=1
  [ $arm = gemm ] && c=0
  HVAE_FWD_CHAIN=$c timeout -k 10 300 python -u bench.py --workload $wl --precision $pr \
    --steps 150 --warmup 30 --no-cpu-baseline --probe-steps 2 2>> $O/bench.err | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'arm':'$arm','workload':'$wl','precision':'$pr','ms':d['ms_per_step'],'value':d['value']}))" >> $O/chain_ab.jsonl || exit 2
}
for r in 1 2; do
  for arm in gemm chain; do ab $arm syn1m bf16; done
  for arm in gemm chain; do ab $arm syn10m fp8; done
done
for arm in gemm chain; do ab $arm syn10m bf16; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn1m -o run -- \
  python3 $R/bench.py --workload syn1m --steps 150 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_syn1m.log 2>&1 || exit 3
cd $R
python3 scripts/step_timeline.py $(find $O/kt_syn1m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn1m.txt || exit 4
echo done > $O/done
