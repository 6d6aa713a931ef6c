# The AVX-512 99-negative sampler on the GPU box's host: the sampler alone (both forms, worker counts) and the
# evaluation's neg99 throughput at All_Beauty and Syn-1M shapes.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05cc
mkdir -p $O
cd $R
timeout -k 10 300 python -u scripts/bench_negatives.py > $O/neg.jsonl 2> $O/neg.err
cat $O/neg.jsonl
timeout -k 10 300 python -u scripts/bench_eval.py --workload all_beauty --probes topk_fused --reps 2 \
  > $O/eval_all_beauty.jsonl 2> $O/eval.err
grep neg99 $O/eval_all_beauty.jsonl
timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --probes topk_fused --reps 2 --neg99-users 1024 \
  > $O/eval_syn1m.jsonl 2> $O/eval1m.err
grep neg99 $O/eval_syn1m.jsonl
