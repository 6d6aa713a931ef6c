# Row-parallel MLP with 1024 threads and 16 loads in flight per lane: its tests, the All_Beauty bench and trace,
# and two Syn-1M benches (the previous pass read 1.51 ms/step with every kernel at its usual time).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_mlprows2}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp_rows.py -x -v --timeout 120 --timeout-method thread > $O/pytest_mlp.log 2>&1
timeout -k 10 300 python bench.py --workload all_beauty --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
timeout -k 10 300 python bench.py --workload syn1m --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 300 python bench.py --workload syn1m --no-cpu-baseline > $O/bench_syn1m_b.json 2> $O/bench_syn1m_b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
