# Instruction-fetch PMC passes over the default bench (the latency-bound All_Beauty step).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
BEN="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --probe-steps 2"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc3/ab$i -o run -- $BEN > $R/gpurun_out/pmc3/ab$i.log 2>&1
done
