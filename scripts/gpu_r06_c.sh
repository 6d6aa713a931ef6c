# Round 6, call C: kernel traces of the current tree's Syn-1M and Syn-10M steps (the step timelines of
# scripts/step_timeline.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for wl in syn1m syn10m; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$wl -o run -- \
    python3 $R/bench.py --workload $wl --steps 100 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_$wl.log 2>&1 || exit 1
done
cd $R
for wl in syn1m syn10m; do
  python3 scripts/step_timeline.py $(find $O/kt_$wl -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_$wl.txt || exit 2
done
echo done > $O/done
