#!/bin/bash
# round 4 pass g: lazy-Adam row loops four row groups per barrier, sweep period by item count, GEMM ring only
# for x W^T: parity (train / lazy / DP / kernels) and the bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04g
mkdir -p $O
echo "tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py \
  tests/test_gpu_large.py tests/test_gpu_large_step.py tests/test_gpu_dp.py tests/test_gpu_mlp_rows.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo "gemm shapes"
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 768 --reps 50 --no-torch > $O/gemm_syn10m.jsonl 2> $O/gemm.log || exit 5
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 384 --reps 50 --no-torch > $O/gemm_syn1m.jsonl 2>> $O/gemm.log || exit 5
echo "benches"
for w in syn10m syn1m all_beauty; do
  st=20; [ $w = syn1m ] && st=100; [ $w = all_beauty ] && st=400
  timeout -k 10 300 python -u bench.py --workload $w --steps $st --warmup 10 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.log || exit 6
  python3 -c "
import json; d=json.load(open('$O/bench_$w.json')); L=d['launch_us']
print('$w', d['ms_per_step'], {k:(v['avg_us'],v['launches_per_step']) for k,v in L.items() if v['launches_per_step']})"
done
echo "dp emul"
timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 1 8 --steps 20 --warmup 6 > $O/dp_emul.jsonl 2> $O/dp_emul.log || exit 7
cat $O/dp_emul.jsonl
