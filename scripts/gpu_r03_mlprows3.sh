# Row-parallel MLP: per-launch times (A/B build: rows per block x rotation), its tests, the All_Beauty bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_mlprows3}
mkdir -p $O
cd $R
for r in 1 2 4; do for rot in 0 1; do
  HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_MLP_R=$r HVAE_MLP_ROT=$rot timeout -k 10 120 python scripts/bench_mlp_rows.py --batches 64,512 > $O/ab_r${r}_rot${rot}.jsonl 2> $O/ab_r${r}_rot${rot}.err
done; done
timeout -k 10 120 python scripts/bench_mlp_rows.py --batches 64,256,512,1024 > $O/product.jsonl 2> $O/product.err
timeout -k 10 120 python scripts/bench_mlp_rows.py --batches 64,1024 --d 768 > $O/product_d768.jsonl 2> $O/product_d768.err
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp_rows.py -x -q --timeout 120 --timeout-method thread > $O/pytest_mlp.log 2>&1
timeout -k 10 300 python bench.py --workload all_beauty --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
