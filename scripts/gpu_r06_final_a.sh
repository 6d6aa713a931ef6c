# Round-6 final evidence, part A (run once, on the tree the round ends on, BEFORE the bench lines so that they carry
# roofline.traffic): FETCH_SIZE / WRITE_SIZE passes (separate runs, one counter each) of the five bench workloads,
# and one SQ / GRBM pass of each d = 768 sweep. Stamped locally (scripts/pmc_to_traffic.py, scripts/pmc_sq_stamp.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r06_final}
mkdir -p $O
KRX='k_dec|k_gemm|k_adam_lazy|k_encoder_sparse_fwd|k_mlp'
cd /tmp && export TMPDIR=/tmp
pmc() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_fetch -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_fetch.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_write -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_write.log 2>&1 || exit 1
}
pmc syn10m --steps 8 --warmup 2 --probe-steps 2
pmc syn10m_fp8 --precision fp8 --steps 8 --warmup 2 --probe-steps 2
pmc syn1m --workload syn1m --steps 20 --warmup 3 --probe-steps 3
pmc syn1m_fp8 --workload syn1m --precision fp8 --steps 20 --warmup 3 --probe-steps 3
pmc all_beauty --workload all_beauty --steps 40 --warmup 5 --probe-steps 5
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_bf16' --output-format csv -d $O/sq_bf16 -o run -- python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 4 > $O/sq_bf16.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc $P1 --kernel-include-regex 'k_dec5_f8' --output-format csv -d $O/sq_fp8 -o run -- python3 $R/scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --dtype fp8 --reps 4 > $O/sq_fp8.log 2>&1 || exit 2
echo done > $O/done_a
