# Round-3 final evidence (second pass), part 2, with the stamped PMC traffic in the tree: the default bench (CPU
# baseline), rocprofv3 kernel-trace stats of the bf16 and fp8 Syn-10M benches, the other bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_final2}
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log
timeout -k 10 420 python -u bench.py --precision fp8 --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/bench_syn10m_fp8.json 2> $O/bench_syn10m_fp8.log
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 300 python -u bench.py --workload syn1m --precision fp8 --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m_fp8.json 2> $O/bench_syn1m_fp8.log
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
timeout -k 10 300 python -u bench.py --workload appliances --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_appliances.json 2> $O/bench_appliances.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fp8 -o run -- python3 $R/bench.py --precision fp8 --steps 30 --warmup 5 --no-cpu-baseline --probe-steps 3 > $O/prof_fp8.log 2>&1
