# Data-parallel rehearsal on one GPU: GPU tests, then a 2-rank bench.py (gloo transport, both ranks on the one MI355X).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest.log 2>&1
HVAE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 40 --warmup 5 --no-cpu-baseline --probe-steps 2 > gpurun_out/bench_dp2.log 2>&1
timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/bench.log 2>&1
