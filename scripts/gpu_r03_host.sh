# Host enqueue time per step against the GPU step time (bench.py host_enqueue_ms_per_step), one step per graph
# replay against K steps per replay (HVAE_STEPS_PER_GRAPH), at All_Beauty, Syn-1M and the Syn-10M shard; the
# train / API / tune GPU tests with the K-step replay on.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_host}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_api.py tests/test_gpu_tune.py tests/test_gpu_dp.py > $O/pytest.log 2>&1
for k in 1 8; do
  HVAE_STEPS_PER_GRAPH=$k timeout -k 10 300 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty_k$k.json 2> $O/bench_all_beauty_k$k.log
done
for k in 1 4; do
  HVAE_STEPS_PER_GRAPH=$k timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m_k$k.json 2> $O/bench_syn1m_k$k.log
done
timeout -k 10 420 python -u bench.py --steps 100 --warmup 10 --probe-steps 5 --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log
