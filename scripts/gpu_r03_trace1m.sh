# rocprofv3 kernel trace of the Syn-1M bench (graph-mode step timeline), sorted row-gradient plan.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_trace1m}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload syn1m --steps 50 --warmup 10 --no-cpu-baseline --probe-steps 2 > $O/prof.log 2>&1
