# Two-exchange DP step (CSR packets before the forward, union plan beside it): a 2-rank one-GPU gloo rehearsal
# of bench.py's DP path (All_Beauty global sharding and the Syn-10M shard shape).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dp3
mkdir -p $O
cd $R
HVAE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload all_beauty --steps 20 --warmup 5 --probe-steps 2 --no-cpu-baseline > $O/bench_dp2_ab.log 2>&1
HVAE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 6 --warmup 2 --probe-steps 1 --no-cpu-baseline > $O/bench_dp2_syn10m.log 2>&1
