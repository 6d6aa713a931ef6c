#!/bin/bash
# round 4 pass h: row-group split of the small-batch MLP (Q blocks per row group), CSR catch-up sliced over
# small batches, on top of pass g's lazy-Adam unroll / sweep period / GEMM ring: parity, then the A/B at the
# All_Beauty shape and the bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04h
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mlp_rows.py \
  tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_ndcg.py tests/test_gpu_dp.py tests/test_gpu_large_step.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "mlp rows A/B (Q = 1 / 2 / 4)"
for q in 1 4 8 2 1 4 8; do
  HVAE_LIB=build_var/libhvae_ab.so HVAE_MLP_Q=$q timeout -k 10 120 python -u scripts/bench_mlp_rows.py --reps 300 \
    --batches 64,200,512 > $O/mlp_q$q.jsonl 2>> $O/mlp.log || exit 5
  echo "Q=$q $(tr '\n' ' ' < $O/mlp_q$q.jsonl)"
done
echo "all_beauty A/B"
for q in 1 4 8 1 4 8; do
  HVAE_LIB=build_var/libhvae_ab.so HVAE_MLP_Q=$q timeout -k 10 200 python -u bench.py --workload all_beauty --steps 400 \
    --warmup 10 --no-cpu-baseline > $O/ab_q$q.json 2>> $O/ab.log || exit 6
  python3 -c "import json; d=json.load(open('$O/ab_q$q.json')); print('Q=$q', d['ms_per_step'])"
done
echo "benches"
for w in syn10m syn1m all_beauty; do
  st=20; [ $w = syn1m ] && st=100; [ $w = all_beauty ] && st=400
  timeout -k 10 300 python -u bench.py --workload $w --steps $st --warmup 10 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.log || exit 7
  python3 -c "
import json; d=json.load(open('$O/bench_$w.json')); L=d['launch_us']
print('$w', d['ms_per_step'], {k:(v['avg_us'],v['launches_per_step']) for k,v in L.items() if v['launches_per_step']})"
done
echo "gemm shapes"
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 --no-torch > $O/gemm_syn10m.jsonl 2> $O/gemm.log || exit 8
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 384 --reps 50 --no-torch > $O/gemm_syn1m.jsonl 2>> $O/gemm.log || exit 8
echo "gemm fast-path A/B for the batch GEMMs"
for d in 384 768; do
  for v in 0 1; do
    HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_FAST_SHORT=$v timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d $d \
      --reps 50 --no-torch > $O/gemm_fs${v}_d$d.jsonl 2>> $O/gemm.log || exit 8
  done
  HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_FAST_SHORT=1 HVAE_GEMM_FAST_TILE=64 timeout -k 10 200 python -u scripts/bench_gemm.py \
    --batch 4096 --d $d --reps 50 --no-torch > $O/gemm_fs1t64_d$d.jsonl 2>> $O/gemm.log || exit 8
done
HVAE_LIB=build_var/libhvae_ab.so HVAE_GEMM_TILE64_MIN=256 timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 384 \
  --reps 50 --no-torch > $O/gemm_t64min256_d384.jsonl 2>> $O/gemm.log || exit 8
echo "dp emul"
timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 1 8 --steps 20 --warmup 6 > $O/dp_emul.jsonl 2> $O/dp_emul.log || exit 9
cat $O/dp_emul.jsonl
