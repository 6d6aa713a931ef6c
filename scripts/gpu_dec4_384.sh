# Version 4 with 8 waves at d = 384 (HVAE_DEC_V4_384=1): the decoder / train-step parity tests under it, then an
# in-process A/B against version 2's DS = 1 sweep at the Syn-1M shape, and the d = 768 tests (default build).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v4_384
mkdir -p $O
HVAE_DEC_V4_384=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_train.py -q -x -k "decoder or fused or lazy or graph or syn1m" --timeout 300 --timeout-method thread > $O/t384.log 2>&1
timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 20 --ab HVAE_DEC_V4_384=1 HVAE_DEC_V4_384=0 --rounds 3 > $O/ab.jsonl 2> $O/ab.err
timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 20 --train --ab HVAE_DEC_V4_384=1 HVAE_DEC_V4_384=0 --rounds 2 > $O/ab_train.jsonl 2> $O/ab_train.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py -q -x -k "768 or versions" --timeout 300 --timeout-method thread > $O/t768.log 2>&1
