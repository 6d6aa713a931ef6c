#!/bin/bash
# round 4 pass i: which of the round-4 lazy-Adam / clip changes pays, per workload (A/B build, one process per arm):
# row-loop unroll (HVAE_ADAM_UNROLL=1 = one row group per barrier), p-only CSR catch-up (HVAE_CATCHUP_PONLY=0 =
# store m, v too), row sums of squares from the apply (HVAE_ROWSQ=0 = the clip reads the rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04i
mkdir -p $O
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env HVAE_LIB=build_var/libhvae_ab.so "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], {k:v['avg_us'] for k,v in L.items() if v['launches_per_step'] and k in ('adam_rows','adam_catchup','rowgrad_apply','clip')})"
}
for r in 1 2; do
  for w in syn10m syn1m all_beauty; do
    st=20; [ $w = syn1m ] && st=100; [ $w = all_beauty ] && st=400
    arm r${r}_default $w $st || exit 5
    arm r${r}_u1 $w $st HVAE_ADAM_UNROLL=1 || exit 5
    arm r${r}_full $w $st HVAE_CATCHUP_PONLY=0 || exit 5
    arm r${r}_rows $w $st HVAE_ROWSQ=0 || exit 5
    arm r${r}_old $w $st HVAE_ADAM_UNROLL=1 HVAE_CATCHUP_PONLY=0 HVAE_ROWSQ=0 || exit 5
  done
done
