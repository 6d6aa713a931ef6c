# All_Beauty step vs the decoder's item-split count (A/B build, HVAE_DEC_SPLITS; the product plan picks 88 at B = 64).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_splits}
mkdir -p $O
cd $R
for s in 0 24 40 56 72 88 120; do
  HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_DEC_SPLITS=$s timeout -k 10 200 python bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_s$s.json 2> $O/bench_s$s.log
done
