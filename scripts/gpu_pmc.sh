# PMC passes (one counter group per run, each under its own time limit) for the decoder sweep
# at Syn-1M shape and for the All_Beauty bench's kernels. Output: gpurun_out/pmc/<pass>/...
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1 || true
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 5"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_bf16' --output-format csv -d $R/gpurun_out/pmc/dec$i -o run -- $DEC > $R/gpurun_out/pmc/dec$i.log 2>&1
done
BEN="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --probe-steps 2"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "$P1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_bf16|k_adam_lazy|k_dec_finalize' --output-format csv -d $R/gpurun_out/pmc/ab$i -o run -- $BEN > $R/gpurun_out/pmc/ab$i.log 2>&1
done
