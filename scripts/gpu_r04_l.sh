#!/bin/bash
# round 4 pass l: All_Beauty anatomy -- kernel trace of the product step, and the plan-in-rows A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], {k:v['avg_us'] for k,v in L.items() if v['launches_per_step']})"
}
arm plan_in_rows all_beauty 400 HVAE_NOTHING=1 || exit 5
arm plan_inline all_beauty 400 HVAE_PLAN_IN_ROWS=0 || exit 5
arm plan_in_rows2 all_beauty 400 HVAE_NOTHING=1 || exit 5
arm plan_inline2 all_beauty 400 HVAE_PLAN_IN_ROWS=0 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ab -o run -- python3 bench.py --workload all_beauty --steps 400 \
  --warmup 10 --no-cpu-baseline > $O/prof_ab.log 2>&1 || exit 6
find $O/prof_ab -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/all_beauty_kernel_stats.csv
find $O/prof_ab -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/all_beauty_kernel_trace.csv
ls -la $O
