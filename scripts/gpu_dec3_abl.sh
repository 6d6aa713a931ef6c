# v3 d = 768 sweep ablations (Syn-10M shard shape) + PMC of the shipped v3 sweep.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/abl3
mkdir -p $O
DEC="scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10"
for v in base abl1 abl2 abl3 abl4; do
  if [ $v = base ]; then L=""; else L="HVAE_LIB=$R/build_var/libhvae_$v.so"; fi
  env $L timeout -k 10 120 python $DEC > $O/$v.json 2>$O/$v.err && sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" $O/$v.json >> $O/all.jsonl
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
DECP="python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 3"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_dec3_bf16' --output-format csv -d $O/pmc$i -o run -- $DECP > $O/pmc$i.log 2>&1
done
