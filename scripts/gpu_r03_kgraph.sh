# All_Beauty / Appliances step vs the number of consecutive steps per graph replay (HVAE_STEPS_PER_GRAPH) with
# the row-parallel MLP step.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_kgraph}
mkdir -p $O
cd $R
for k in 1 8 16 32; do
  HVAE_STEPS_PER_GRAPH=$k timeout -k 10 200 python bench.py --workload all_beauty --steps 320 --warmup 32 --probe-steps 10 --no-cpu-baseline > $O/all_beauty_k$k.json 2> $O/all_beauty_k$k.log
done
