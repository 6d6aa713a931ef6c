# rocprofv3 kernel-trace stats of the Syn-1M bench.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_syn -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload syn1m --steps 30 --warmup 3 --no-cpu-baseline --probe-steps 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_syn.log 2>&1
