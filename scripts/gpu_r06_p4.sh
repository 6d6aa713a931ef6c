# Round 6, call P4: SQ counters of the forward chain kernel (k_chain_fwd, variant c = 512 threads x 4 chunks ahead)
# at d = 768: where its cycles go.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
HVAE_LIB=$R/build_var/libhvae_chc.so timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex 'k_chain_fwd' --output-format csv -d $O/sq -o run -- python3 $R/scripts/bench_chain.py --D 768 --reps 20 > $O/sq.log 2>&1 || exit 1
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
HVAE_LIB=$R/build_var/libhvae_chc.so timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-include-regex 'k_chain_fwd' --output-format csv -d $O/sq2 -o run -- python3 $R/scripts/bench_chain.py --D 768 --reps 20 > $O/sq2.log 2>&1 || exit 2
echo done > $O/done
