# Round-5 counters of the version-6 bf16 sweep (k_dec6_bf16) beside version 5 (k_dec5_bf16) at the Syn-10M shard:
# SQ pass (MFMA busy, waits, LDS) and an L2 / VMEM pass (hits, misses, instruction counts). One pass per run.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec6_bf16' --output-format csv -d $O/v6_sq -o run -- $DEC > $O/v6_sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P2 --kernel-include-regex 'k_dec6_bf16' --output-format csv -d $O/v6_l2 -o run -- $DEC > $O/v6_l2.log 2>&1
export HVAE_DEC_V6=0
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_bf16' --output-format csv -d $O/v5_sq -o run -- $DEC > $O/v5_sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P2 --kernel-include-regex 'k_dec5_bf16' --output-format csv -d $O/v5_l2 -o run -- $DEC > $O/v5_l2.log 2>&1
python3 $R/scripts/pmc_summary.py $O/v6_sq $O/v6_l2 $O/v5_sq $O/v5_l2 > $O/pmc_summary.txt
