#!/bin/bash
# round 4 pass t: lazy Adam's replays read the last eight step-table entries from registers (loaded with the
# launch's first loads): lazy == dense parity, bench lines on the three workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04t
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_dp.py \
  > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], {k:v['avg_us'] for k,v in L.items() if v['launches_per_step'] and k in ('adam_rows','adam_catchup','mlp_fwd')})"
}
for r in 1 2; do
  arm r$r all_beauty 400 HVAE_NOTHING=1 || exit 6
  arm r$r syn1m 100 HVAE_NOTHING=1 || exit 6
  arm r$r syn10m 20 HVAE_NOTHING=1 || exit 6
done
