# Session start on MI355X: every GPU test, smoke, GEMM per-shape timings at B = 4096 (d = 384, 768),
# and SQ / cache counters of two representative GEMMs.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s3start
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 384 > $O/gemm384.jsonl 2>&1
timeout -k 10 200 python -u scripts/bench_gemm.py --batch 4096 --d 768 > $O/gemm768.jsonl 2>&1
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum"
for S in fwd_proj_b bwd_dWb; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'k_gemm' --output-format csv -d $O/pmc_${S}_$i -o run -- python3 $R/scripts/bench_gemm.py --batch 4096 --d 384 --only $S --reps 20 --no-torch > $O/pmc_${S}_$i.log 2>&1
  done
done
