#!/bin/bash
# round 4 pass j: one row group per barrier again, quad-DPP row sums of squares (16 fp64 partials per row) for the
# clip: parity, bench lines, the rowsq A/B and the W = 8 emulation with its arms
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04j
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_dp.py \
  tests/test_gpu_kernels.py tests/test_gpu_large_step.py tests/test_gpu_mlp_rows.py > $O/pytest.log 2>&1
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
  for w in syn10m syn1m all_beauty; do
    st=20; [ $w = syn1m ] && st=100; [ $w = all_beauty ] && st=400
    arm r${r}_product $w $st HVAE_NOTHING=1 || exit 5
    arm r${r}_rows $w $st HVAE_LIB=build_var/libhvae_ab.so HVAE_ROWSQ=0 || exit 5
  done
done
echo "dp emul"
timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 1 8 --steps 20 --warmup 6 > $O/dp_emul.jsonl 2> $O/dp_emul.log || exit 7
HVAE_LIB=build_var/libhvae_ab.so HVAE_ROWSQ=0 timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 8 --steps 20 --warmup 6 \
  > $O/dp_emul_rows.jsonl 2>> $O/dp_emul.log || exit 7
HVAE_LIB=build_var/libhvae_ab.so HVAE_ADAM_UNROLL=4 timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 8 --steps 20 --warmup 6 \
  > $O/dp_emul_u4.jsonl 2>> $O/dp_emul.log || exit 7
cat $O/dp_emul.jsonl $O/dp_emul_rows.jsonl $O/dp_emul_u4.jsonl
