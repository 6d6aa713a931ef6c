#!/bin/bash
# round 4 pass s: the inline lazy read with the recent step-table window preloaded (no table load in the replay)
# at small batches: parity (lazy == dense bitwise), the A/B, bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mlp_rows.py tests/test_gpu_train.py \
  tests/test_gpu_ndcg.py tests/test_gpu_dp.py > $O/pytest.log 2>&1
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
  arm r${r}_enclazy all_beauty 400 HVAE_NOTHING=1 || exit 6
  arm r${r}_catchup all_beauty 400 HVAE_ENC_LAZY_READ=0 || exit 6
done
arm r1 appliances 200 HVAE_NOTHING=1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ab -o run -- python3 bench.py --workload all_beauty --steps 400 \
  --warmup 10 --no-cpu-baseline > $O/prof_ab.log 2>&1 || exit 7
find $O/prof_ab -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/all_beauty_kernel_stats.csv
rm -rf $O/prof_ab
