# Round 6, call I: step timelines of All_Beauty and the Syn-10M shard on the current tree (weight gradients on the
# side stream by default), and the data-parallel W = 8 one-GPU emulation in bf16 and fp8 (projection inputs).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_all_beauty -o run -- \
  python3 $R/bench.py --workload all_beauty --steps 400 --warmup 40 --no-cpu-baseline --probe-steps 2 > $O/kt_all_beauty.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt_syn10m -o run -- \
  python3 $R/bench.py --workload syn10m --steps 60 --warmup 10 --no-cpu-baseline --probe-steps 2 > $O/kt_syn10m.log 2>&1 || exit 2
cd $R
python3 scripts/step_timeline.py $(find $O/kt_all_beauty -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_all_beauty.txt || exit 3
python3 scripts/step_timeline.py $(find $O/kt_syn10m -name "*kernel_trace.csv" | head -1) --sweep k_dec > $O/timeline_syn10m.txt || exit 4
for P in bf16 fp8; do
  timeout -k 10 500 python3 -u scripts/bench_dp_emul.py --world 1 8 --steps 60 --warmup 10 --precision $P > $O/emul_$P.log 2>&1 || exit 5
done
echo done > $O/done
