# Version 3 of the d = 768 bf16 sweep: every d = 768 GPU test (old and new), then v3 vs v2 timing at the
# Syn-10M shard shape in one process, then the large-shape parity file.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dec3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fp8.py -x -q -k "768 or d768" --timeout 120 --timeout-method thread > $O/pytest_d768.log 2>&1
timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 --ab HVAE_DEC_V3=1 HVAE_DEC_V3=0 HVAE_DEC_V3=1,HVAE_DEC_SPLITS=8 --rounds 2 > $O/ab.jsonl 2>$O/ab.err
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 600 --timeout-method thread > $O/pytest_large.log 2>&1
