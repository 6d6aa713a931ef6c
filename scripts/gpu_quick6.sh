# train-step tests (lazy Adam bitwise vs dense, golden), default bench, rocprof kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
timeout -k 10 300 python bench.py --workload syn1m --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > gpurun_out/bench_syn1m.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 --no-cpu-baseline --probe-steps 5 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
