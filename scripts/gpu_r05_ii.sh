# SQ counters of the lazy-Adam kernels at the Syn-10M shard (the catch-up's replays: VALU- or memory-bound?):
# one pass of 8 SQ + GRBM_GUI_ACTIVE over k_adam_catchup_csr / k_adam_lazy, then FETCH_SIZE and WRITE_SIZE passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ii
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $P1 --kernel-include-regex 'k_adam' --output-format csv -d $O/sq -o run -- \
  python3 $R/bench.py --steps 8 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 3; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_adam' --output-format csv -d $O/fetch -o run -- \
  python3 $R/bench.py --steps 8 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex 'k_adam' --output-format csv -d $O/kt -o run -- \
  python3 $R/bench.py --steps 8 --warmup 2 --probe-steps 2 --no-cpu-baseline > $O/kt.log 2>&1 || exit 5
python3 $R/scripts/pmc_summary.py $O/sq $O/fetch > $O/summary.txt
cat $O/summary.txt
grep -i adam $O/kt/run_kernel_stats.csv | cut -c1-200
