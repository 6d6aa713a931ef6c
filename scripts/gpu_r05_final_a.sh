# Round-5 final evidence, part A (the tree the round ends on): every GPU test, smoke, the default bench (Syn-10M
# shard, bf16, CPU baseline), rocprofv3 kernel-trace stats of the default bench and of the fp8 bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_final}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 420 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 $R/bench.py --precision fp8 --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof_fp8.log 2>&1
