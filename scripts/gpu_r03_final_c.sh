# Round-3 final evidence, part C: the bench lines again with the stamped PMC traffic in the tree (roofline.traffic).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_final_c}
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log
timeout -k 10 420 python -u bench.py --precision fp8 --steps 60 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/bench_syn10m_fp8.json 2> $O/bench_syn10m_fp8.log
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 300 python -u bench.py --workload syn1m --precision fp8 --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m_fp8.json 2> $O/bench_syn1m_fp8.log
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
