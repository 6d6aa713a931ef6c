# Version 5 (the d = 768 default) counters at the Syn-10M shard: LDS conflicts, MFMA busy, stall buckets.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_v5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_bf16' --output-format csv -d $O/p1 -o run -- $DEC > $O/p1.log 2>&1
python3 $R/scripts/pmc_summary.py $O/p1 > $O/pmc_summary.txt
