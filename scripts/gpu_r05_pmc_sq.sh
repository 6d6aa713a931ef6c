# Round-5 final-tree SQ / GRBM counters of the d = 768 sweeps at the Syn-10M shard (bf16 k_dec5_bf16, fp8 k_dec5_f8):
# MFMA busy, wait buckets, LDS conflicts. One pass per kernel (8 SQ + 1 GRBM counters).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_pmc_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_bf16' --output-format csv -d $O/bf16 -o run -- python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 > $O/bf16.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_f8' --output-format csv -d $O/fp8 -o run -- python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --dtype fp8 --reps 4 > $O/fp8.log 2>&1
python3 $R/scripts/pmc_summary.py $O/bf16 $O/fp8 > $O/pmc_summary.txt
