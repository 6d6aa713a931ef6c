# Syn-1M (configs[2]) step anatomy: kernel trace + stats of the bench line (graph replays)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/syn1m -o run -- python3 $R/bench.py \
  --workload syn1m --steps 300 --warmup 30 --no-cpu-baseline --probe-steps 5 > $O/syn1m.log 2>&1
grep '"metric"' $O/syn1m.log | cut -c1-300
