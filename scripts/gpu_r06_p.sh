# Round 6, call P: the forward chain kernel's variants standalone (scripts/bench_chain.py: threads per block x
# weight chunks in flight, each as a whole library -- build_var/libhvae_ch{a,b,c,d}.so = 512x8, 256x8, 512x4,
# 1024x4; the product = 512x8) against the GEMM chain, at the Syn-1M (d = 384) and Syn-10M (d = 768) shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p2
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_chain.log 2>&1 || exit 3
timeout -k 10 200 python -u scripts/bench_chain.py --reps 100 --tag product >> $O/chain_variants.jsonl 2>> $O/err.log || exit 1
for v in b c d; do
  HVAE_LIB=build_var/libhvae_ch$v.so timeout -k 10 200 python -u scripts/bench_chain.py --reps 100 --tag ch$v >> $O/chain_variants.jsonl 2>> $O/err.log || exit 2
done
echo done > $O/done
