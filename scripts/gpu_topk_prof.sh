# Kernel stats of the fused top-K at the Syn-10M shape (LDS scan and global-load scan arms).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/topkprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/scripts/bench_eval.py --workload syn10m --batch 4096 --neg99-users 0 --skip-matrix --reps 3 > $O/prof.log 2>&1
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_recommend.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --batch 4096 --neg99-users 0 > $O/eval_syn1m.jsonl 2> $O/eval_syn1m.err
timeout -k 10 200 python -u scripts/bench_eval.py --workload all_beauty > $O/eval_ab.jsonl 2> $O/eval_ab.err
