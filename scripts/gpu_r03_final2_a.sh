# Round-3 final evidence (second pass, after the GEMM register ring), part 1: every GPU test, smoke, and the
# FETCH_SIZE / WRITE_SIZE passes of the five bench workloads (stamped locally by scripts/pmc_to_traffic.py).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_final2}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
KRX='k_dec|k_gemm|k_adam_lazy|k_encoder_sparse_fwd|k_mlp'
cd /tmp && export TMPDIR=/tmp
pmc() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_fetch -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" --output-format csv -d $O/pmc_${n}_write -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/pmc_${n}_write.log 2>&1
}
pmc syn10m --steps 8 --warmup 2 --probe-steps 2
pmc syn10m_fp8 --precision fp8 --steps 8 --warmup 2 --probe-steps 2
pmc syn1m --workload syn1m --steps 20 --warmup 3 --probe-steps 3
pmc syn1m_fp8 --workload syn1m --precision fp8 --steps 20 --warmup 3 --probe-steps 3
pmc all_beauty --workload all_beauty --steps 40 --warmup 5 --probe-steps 5
