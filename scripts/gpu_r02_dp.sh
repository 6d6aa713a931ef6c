# Data-parallel rework: every GPU test (incl. the 2-rank-vs-union and global-sharding DP tests), smoke, and a
# 2-rank one-GPU gloo rehearsal of bench.py's DP path (All_Beauty global sharding and the Syn-10M shard shape).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dp
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
HVAE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload all_beauty --steps 20 --warmup 5 --probe-steps 2 > $O/bench_dp2_ab.log 2>&1
HVAE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 6 --warmup 2 --probe-steps 1 > $O/bench_dp2_syn10m.log 2>&1
