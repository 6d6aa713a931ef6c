# k_topk_scan with the wave-users block mapping: parity, then eval throughput A/B against the tile-split mapping.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/topk2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_recommend.py -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u scripts/bench_eval.py --workload all_beauty --neg99-users 0 > $O/eval_ab.jsonl 2> $O/eval_ab.err
timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --batch 4096 --neg99-users 0 > $O/eval_syn1m.jsonl 2> $O/eval_syn1m.err
timeout -k 10 400 python -u scripts/bench_eval.py --workload syn10m --batch 4096 --neg99-users 0 > $O/eval_syn10m.jsonl 2> $O/eval_syn10m.err
