# Round-4 final evidence, PMC part: FETCH_SIZE / WRITE_SIZE passes (separate runs) of the other bench workloads on the
# final tree, stamped locally by scripts/pmc_to_traffic.py
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_final}
mkdir -p $O
KRX='k_dec|k_gemm|k_adam_lazy|k_encoder_sparse_fwd|k_mlp'
cd /tmp && export TMPDIR=/tmp
pmc() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_fetch -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_fetch.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_write -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_write.log 2>&1
}
pmc syn10m_fp8 --precision fp8 --steps 8 --warmup 2 --probe-steps 2
pmc syn1m --workload syn1m --steps 20 --warmup 3 --probe-steps 3
pmc all_beauty --workload all_beauty --steps 40 --warmup 5 --probe-steps 5
