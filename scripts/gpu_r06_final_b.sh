# Round-6 final evidence, part B (after part A's PMC passes were stamped into profiles/pmc_*.json, so that these
# lines carry roofline.traffic): smoke, the default bench (Syn-10M shard, bf16, CPU baseline), rocprofv3
# kernel-trace stats of the default and the fp8 bench, and the other bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_final}
mkdir -p $O
cd $R
# the A/B library rebuilt from the end tree's sources (part A's suite ran a stale one)
timeout -k 10 600 python -u -m pytest tests/test_gpu_ab_variant.py -m gpu -q --timeout 500 --timeout-method thread > $O/pytest_ab.log 2>&1 || exit 10
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 420 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 $R/bench.py --precision fp8 --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof_fp8.log 2>&1 || exit 4
cd $R
timeout -k 10 420 python -u bench.py --precision fp8 --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_syn10m_fp8.json 2> $O/bench_syn10m_fp8.log || exit 5
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log || exit 6
timeout -k 10 300 python -u bench.py --workload syn1m --precision fp8 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_syn1m_fp8.json 2> $O/bench_syn1m_fp8.log || exit 7
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log || exit 8
timeout -k 10 300 python -u bench.py --workload appliances --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_appliances.json 2> $O/bench_appliances.log || exit 9
echo done > $O/done_b
