# Version 4 of the d = 768 bf16 sweep: parity (every d = 768 test, v4 vs v3 vs v2), then an in-process A/B
# against version 3 at the Syn-10M shard shape.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_kernels.py -q -x -k "768 or versions" --timeout 300 --timeout-method thread > $O/t.log 2>&1
timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 --ab HVAE_DEC_V4=1 HVAE_DEC_V4=0 --rounds 3 > $O/ab.jsonl 2> $O/ab.err
