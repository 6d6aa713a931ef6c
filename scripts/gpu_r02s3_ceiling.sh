# The sustained bf16 MFMA ceiling on the box (scripts/probe_mfma_ceiling.hip, built into build_probe/ on the
# CPU container) and the version-4 sweep's own counters at the Syn-10M shard: MFMA busy cycles and the effective
# clock (GRBM_GUI_ACTIVE / 8 / wall), stall buckets, LDS activity.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ceiling
mkdir -p $O
timeout -k 10 120 $R/build_probe/probe_mfma_ceiling > $O/probe.jsonl 2> $O/probe.log
cd /tmp && export TMPDIR=/tmp
DEC="python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4"
timeout -k 10 200 $DEC > $O/dec_wall.log 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec4_bf16' --output-format csv -d $O/p1 -o run -- $DEC > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $P2 --kernel-include-regex 'k_dec4_bf16' --output-format csv -d $O/p2 -o run -- $DEC > $O/p2.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_dec4_bf16' --output-format csv -d $O/kt -o run -- $DEC > $O/kt.log 2>&1
python3 $R/scripts/pmc_summary.py $O/p1 $O/p2 > $O/pmc_summary.txt
