# Round-5 final evidence, part B: FETCH_SIZE / WRITE_SIZE PMC passes (separate runs, one counter each) of the five
# bench workloads on the final tree (stamped locally by scripts/pmc_to_traffic.py), then the other bench lines.
# (the bench lines at the default --probe-steps 50: the probe brackets eager steps, and a run_epoch call's first
# steps carry a heavier catch-up, so 5 probe steps read the fp8 adam_catchup at 430-470 us against 118 in the trace)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r05_final}
mkdir -p $O
KRX='k_dec|k_gemm|k_adam_lazy|k_encoder_sparse_fwd|k_mlp'
cd /tmp && export TMPDIR=/tmp
pmc() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_fetch -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_write -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_write.log 2>&1
}
pmc syn10m --steps 8 --warmup 2 --probe-steps 2
pmc syn10m_fp8 --precision fp8 --steps 8 --warmup 2 --probe-steps 2
pmc syn1m --workload syn1m --steps 20 --warmup 3 --probe-steps 3
pmc syn1m_fp8 --workload syn1m --precision fp8 --steps 20 --warmup 3 --probe-steps 3
pmc all_beauty --workload all_beauty --steps 40 --warmup 5 --probe-steps 5
cd $R
timeout -k 10 420 python -u bench.py --precision fp8 --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_syn10m_fp8.json 2> $O/bench_syn10m_fp8.log
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 300 python -u bench.py --workload syn1m --precision fp8 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_syn1m_fp8.json 2> $O/bench_syn1m_fp8.log
timeout -k 10 300 python -u bench.py --workload all_beauty --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_all_beauty.json 2> $O/bench_all_beauty.log
timeout -k 10 300 python -u bench.py --workload appliances --steps 300 --warmup 30 --probe-steps 20 --no-cpu-baseline > $O/bench_appliances.json 2> $O/bench_appliances.log
