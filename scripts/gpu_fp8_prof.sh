# fp8 decoder evidence: Syn-10M (d = 768) benches bf16 vs fp8, Syn-1M fp8 rocprofv3 kernel stats, and the
# FETCH_SIZE / WRITE_SIZE passes for the fp8 sweep (profiles/pmc_syn1m_fp8.json).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc8
timeout -k 10 400 python -u bench.py --workload syn10m --precision fp8 --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/bench_syn10m_fp8.log 2>&1
timeout -k 10 400 python -u bench.py --workload syn10m --steps 20 --warmup 3 --probe-steps 2 --no-cpu-baseline > gpurun_out/bench_syn10m.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_syn8 -o run -- python3 $R/bench.py --workload syn1m --precision fp8 --steps 30 --warmup 3 --no-cpu-baseline --probe-steps 2 > $R/gpurun_out/prof_syn8.log 2>&1
BEN="python3 $R/bench.py --workload syn1m --precision fp8 --steps 10 --warmup 2 --no-cpu-baseline --probe-steps 1"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_fp8|k_adam_lazy|k_dec_finalize' --output-format csv -d $R/gpurun_out/pmc8/p$i -o run -- $BEN > $R/gpurun_out/pmc8/p$i.log 2>&1
done
