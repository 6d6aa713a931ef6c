# configs[4] shape evidence: rocprofv3 kernel-trace stats of the Syn-10M fp8 bench and the fp8 sweep's PMC
# counters at d = 768 (3-slot ring), plus FETCH/WRITE for profiles/pmc_syn10m_fp8.json
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/p10
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p10/prof -o run -- python3 $R/bench.py --workload syn10m --precision fp8 --steps 8 --warmup 2 --no-cpu-baseline --probe-steps 1 > $R/gpurun_out/p10/prof.log 2>&1
DEC="python3 $R/scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 200000 --D 768 --reps 5"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_fp8' --output-format csv -d $R/gpurun_out/p10/d$i -o run -- $DEC > $R/gpurun_out/p10/d$i.log 2>&1
done
BEN="python3 $R/bench.py --workload syn10m --precision fp8 --steps 3 --warmup 1 --no-cpu-baseline --probe-steps 1"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_fp8|k_adam_lazy|k_dec_finalize' --output-format csv -d $R/gpurun_out/p10/t$i -o run -- $BEN > $R/gpurun_out/p10/t$i.log 2>&1
done
