# PMC passes (one counter group per run) for the bf16 decoder sweep at the Syn-1M shape.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 5"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_dec2_bf16' --output-format csv -d $R/gpurun_out/pmc2/dec$i -o run -- $DEC > $R/gpurun_out/pmc2/dec$i.log 2>&1
done
