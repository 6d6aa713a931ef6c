# Fused top-K scan with the per-user LDS heaps at an odd stride (default build) against the even stride
# (build_var/libhvae_tkold.so): the top-K / recommend / eval parity tests on the default, then the Syn-1M and
# Syn-10M eval scan in alternating processes, and the scan's LDS counters.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tkheap
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "topk or recommend or rank or evaluat" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  for w in syn1m syn10m; do
    timeout -k 10 200 python -u scripts/bench_eval.py --workload $w --probes topk_fused --skip-matrix --batch 4096 --reps 3 > $O/new_${w}_$i.txt 2>&1
    HVAE_LIB=$R/build_var/libhvae_tkold.so timeout -k 10 200 python -u scripts/bench_eval.py --workload $w --probes topk_fused --skip-matrix --batch 4096 --reps 3 > $O/old_${w}_$i.txt 2>&1
  done
done
cd /tmp && export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex 'k_topk' --output-format csv -d $O/pmc -o run -- python3 $R/scripts/bench_eval.py --workload syn1m --probes topk_fused --skip-matrix --reps 2 > $O/pmc.log 2>&1
python3 $R/scripts/pmc_summary.py $O/pmc > $O/pmc_summary.txt
