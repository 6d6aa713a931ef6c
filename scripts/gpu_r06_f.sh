# Round 6, call F: bench lines of every workload on the current tree (host-loop fix + sorted plan), no CPU
# baseline, and the Syn-1M step timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
for a in "all_beauty bf16" "appliances bf16" "syn1m bf16" "syn1m fp8" "syn10m bf16" "syn10m fp8"; do
  set -- $a
  timeout -k 10 300 python -u bench.py --workload $1 --precision $2 --no-cpu-baseline --probe-steps 10 \
    > $O/bench_$1_$2.json 2>> $O/bench.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn1m -o run -- \
  python3 $R/bench.py --workload syn1m --steps 150 --warmup 20 --no-cpu-baseline --probe-steps 2 > $O/kt_syn1m.log 2>&1 || exit 2
cd $R
python3 scripts/step_timeline.py $(find $O/kt_syn1m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn1m.txt || exit 3
echo done > $O/done
