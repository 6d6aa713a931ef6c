# The block-form candidate matrix (evaluator / tuner): the GPU tests of the evaluation protocols, then the neg99
# throughput at All_Beauty and Syn-1M shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05gg
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api.py \
  tests/test_gpu_dp_dropin.py tests/test_gpu_tune.py tests/test_gpu_ndcg.py > $O/pytest_eval.log 2>&1 || { tail -30 $O/pytest_eval.log; exit 3; }
tail -2 $O/pytest_eval.log
timeout -k 10 300 python -u scripts/bench_eval.py --workload all_beauty --probes topk_fused --reps 2 \
  > $O/eval_all_beauty.jsonl 2> $O/eval.err || exit 4
grep neg99 $O/eval_all_beauty.jsonl
timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --probes topk_fused --reps 2 --neg99-users 1024 \
  > $O/eval_syn1m.jsonl 2> $O/eval1m.err || exit 5
grep neg99 $O/eval_syn1m.jsonl
