# Version 4 with GEMM2 on 16x16x32 MFMAs (build_var/libhvae_g16.so, DEC4_G2_16=1): d = 768 parity tests on it,
# then the sweep at the Syn-10M shard, alternating default and variant processes.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/g16
mkdir -p $O
cd $R
HVAE_LIB=$R/build_var/libhvae_g16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py tests/test_gpu_train.py -m gpu -x -q -k "768 or versions or fused_step or d768" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/base_$i.jsonl 2>&1
  HVAE_LIB=$R/build_var/libhvae_g16.so timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 6 --rounds 1 > $O/g16_$i.jsonl 2>&1
done
