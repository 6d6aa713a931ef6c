# The last LayerNorm backward fused into the row-parallel MLP backward: tests, the GPU suite, benches, trace.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_lnfused}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp_rows.py -x -v --timeout 120 --timeout-method thread > $O/pytest_mlp.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python bench.py --workload all_beauty --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
timeout -k 10 300 python bench.py --workload appliances --no-cpu-baseline > $O/bench_appliances.json 2> $O/bench_appliances.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
