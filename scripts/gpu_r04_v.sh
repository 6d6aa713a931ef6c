#!/bin/bash
# round 4 pass v: GEMM fragment prefetch on every register-staged path (variant libhvae_gpf) and x W^T long k on the
# one-stage instance (HVAE_GEMM_NT1=1): shapes and bench A/B against the product
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04v
mkdir -p $O
shapes() {  # name, d, env...
  local name=$1 d=$2; shift 2
  env "$@" timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d $d --reps 50 --no-torch > $O/gemm_${name}_d$d.jsonl 2>> $O/gemm.log || return 1
  echo "d=$d $name $(python3 -c "
import json
print({list(json.loads(l))[0]: json.loads(l)[list(json.loads(l))[0]]['hvae_us'] for l in open('$O/gemm_${name}_d$d.jsonl')})")"
}
for d in 768 384; do
  shapes product $d HVAE_NOTHING=1 || exit 5
  shapes gpf $d HVAE_LIB=build_var/libhvae_gpf.so || exit 5
  shapes nt1 $d HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_NT1=1 || exit 5
  shapes gpf_nt1 $d HVAE_LIB=build_var/libhvae_gpf.so HVAE_GEMM_NT1=1 || exit 5
done
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], 'gemm', L['gemm']['avg_us'])"
}
for r in 1 2; do
  arm r${r}_product syn1m 100 HVAE_NOTHING=1 || exit 6
  arm r${r}_gpf syn1m 100 HVAE_LIB=build_var/libhvae_gpf.so || exit 6
done
