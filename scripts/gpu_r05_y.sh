# 99-negative protocol throughput with the native sampler (scripts/bench_eval.py, All_Beauty and Syn-1M shapes)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05y
mkdir -p $O
cd $R
for w in all_beauty syn1m; do
  timeout -k 10 400 python -u scripts/bench_eval.py --workload $w > $O/eval_$w.jsonl 2> $O/eval_$w.err
  cat $O/eval_$w.jsonl
done
