# PMC passes for the fp8 sweep (k_dec_fp8) at Syn-1M shape (d = 384) and the Syn-10M shape (d = 768)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcf
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
for D in 384 768; do
  N=100000; [ $D = 768 ] && N=200000
  DEC="python3 $R/scripts/bench_decoder.py --dtype fp8 --nb 4096 --N $N --D $D --reps 5"
  timeout -k 10 120 $DEC > $R/gpurun_out/pmcf/time_$D.log 2>&1
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_dec_fp8' --output-format csv -d $R/gpurun_out/pmcf/d${D}_$i -o run -- $DEC > $R/gpurun_out/pmcf/d${D}_$i.log 2>&1
  done
done
