# Steady-state SQ / FETCH counters of the lazy-Adam kernels at the Syn-10M shard (60 warm-up steps first, so the
# catch-up's replays have their steady length); scripts/pmc_tail.py averages the last dispatches only
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05jj
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-include-regex 'k_adam_lazy|k_adam_catchup_csr' --output-format csv -d $O/sq -o run -- \
  python3 $R/bench.py --steps 10 --warmup 60 --probe-steps 2 --no-cpu-baseline > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_adam_lazy|k_adam_catchup_csr' --output-format csv -d $O/fetch -o run -- \
  python3 $R/bench.py --steps 10 --warmup 60 --probe-steps 2 --no-cpu-baseline > $O/fetch.log 2>&1 || exit 4
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_adam_lazy|k_adam_catchup_csr' --output-format csv -d $O/write -o run -- \
  python3 $R/bench.py --steps 10 --warmup 60 --probe-steps 2 --no-cpu-baseline > $O/write.log 2>&1 || exit 5
timeout -s KILL 240 rocprofv3 --kernel-trace --kernel-include-regex 'k_adam_lazy|k_adam_catchup_csr' --output-format csv -d $O/kt -o run -- \
  python3 $R/bench.py --steps 10 --warmup 60 --probe-steps 2 --no-cpu-baseline > $O/kt.log 2>&1 || exit 6
python3 $R/scripts/pmc_tail.py 10 $O/sq $O/fetch $O/write $O/kt > $O/summary.txt
cat $O/summary.txt
