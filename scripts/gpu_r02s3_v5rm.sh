# Version 5 with the conflict-free GEMM1 row map: d = 768 parity (versions agree, v5 included), then v5 against
# version 4 in one process at the Syn-10M shard, LDS-DMA split DEC5_DMA_B = 0 (default build) and 4 / 6 / 8.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/v5rm
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_kernels.py -m gpu -x -q -k "768 or versions" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
HVAE_LIB=$R/build_var/libhvae_dmab6.so HVAE_DEC_V5=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q -k "versions" --timeout 300 --timeout-method thread > $O/pytest_dmab6.log 2>&1
timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 2 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_dmab0.jsonl 2>&1
for V in dmab4 dmab6 dmab8; do
  HVAE_LIB=$R/build_var/libhvae_$V.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 2 --ab HVAE_DEC_V5=0 HVAE_DEC_V5=1 > $O/ab_$V.jsonl 2>&1
done
