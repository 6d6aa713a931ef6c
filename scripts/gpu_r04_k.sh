#!/bin/bash
# round 4 pass k: the small-batch MLP weight gradients beside the W1 row gather, the clip grid sized to its input
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04k
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_mlp_rows.py \
  tests/test_gpu_ndcg.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], {k:v['avg_us'] for k,v in L.items() if v['launches_per_step']})"
}
for r in 1 2; do
  arm r${r}_beside all_beauty 400 HVAE_NOTHING=1 || exit 5
  arm r${r}_inline all_beauty 400 HVAE_WGRAD_BESIDE=0 || exit 5
done
arm product syn1m 100 HVAE_NOTHING=1 || exit 5
arm product syn10m 20 HVAE_NOTHING=1 || exit 5
arm product appliances 200 HVAE_NOTHING=1 || exit 5
