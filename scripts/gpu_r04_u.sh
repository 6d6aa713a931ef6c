#!/bin/bash
# round 4 pass u: long-k x W data gradients (and long-k register-staged products) on a one-stage instance whose
# k-tile reads every fragment before its MFMAs: GEMM parity, shapes A/B (HVAE_GEMM_NN1=0: the old routing), benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04u
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py \
  tests/test_gpu_large_step.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for d in 768 384; do
  for v in 1 0; do
    HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_NN1=$v timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d $d \
      --reps 50 --no-torch > $O/gemm_nn1_${v}_d$d.jsonl 2>> $O/gemm.log || exit 5
    echo "d=$d NN1=$v $(python3 -c "
import json
print({list(json.loads(l))[0]: json.loads(l)[list(json.loads(l))[0]]['hvae_us'] for l in open('$O/gemm_nn1_${v}_d$d.jsonl')})")"
  done
done
arm() {  # name, workload, steps, env...
  local name=$1 w=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps $st --warmup 10 \
    --no-cpu-baseline > $O/${w}_$name.json 2>> $O/bench.log || return 1
  python3 -c "
import json; d=json.load(open('$O/${w}_$name.json')); L=d['launch_us']
print('$w $name', d['ms_per_step'], {k:v['avg_us'] for k,v in L.items() if v['launches_per_step']})"
}
for r in 1 2; do
  arm r${r}_nn1 syn1m 100 HVAE_NOTHING=1 || exit 6
  arm r${r}_old syn1m 100 HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_NN1=0 || exit 6
  arm r${r}_nn1ab syn1m 100 HVAE_LIB=build_var/libhvae_ab.so || exit 6
done
arm r1_nn1 syn10m 20 HVAE_NOTHING=1 || exit 6
arm r1_old syn10m 20 HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_NN1=0 || exit 6
