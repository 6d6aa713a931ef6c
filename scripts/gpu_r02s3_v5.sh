# Decoder version 5 (producer / consumer waves) at d = 768: parity against versions 4/3/2, in-process A/B
# of the sweep against version 4 at 4096 x 200,000 and the Syn-10M shard (4096 x 1,000,000); then the
# weight-gradient GEMM step A/B (scripts/gpu_r02s3_gemm2.sh).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5
mkdir -p $O
cd $R
timeout -k 10 240 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q -k versions_agree --timeout 200 --timeout-method thread > $O/pytest_v5.log 2>&1
timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 200000 --D 768 --reps 10 --rounds 3 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_200k.jsonl 2>&1
timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --rounds 3 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_1m.jsonl 2>&1
bash scripts/gpu_r02s3_gemm2.sh
