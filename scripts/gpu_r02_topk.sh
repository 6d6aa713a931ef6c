# Fused top-K / recommend core: parity tests, the train-step pins, then eval throughput per workload.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/topk
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_recommend.py tests/test_gpu_train.py tests/test_gpu_api.py -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || true
timeout -k 10 200 python -u scripts/bench_eval.py --workload all_beauty > $O/eval_ab.jsonl 2> $O/eval_ab.err
timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --batch 4096 > $O/eval_syn1m.jsonl 2> $O/eval_syn1m.err
timeout -k 10 400 python -u scripts/bench_eval.py --workload syn10m --batch 4096 --neg99-users 0 > $O/eval_syn10m.jsonl 2> $O/eval_syn10m.err
