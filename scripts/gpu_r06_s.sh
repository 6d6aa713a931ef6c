# Round 6, call S (the end tree): the data-parallel W = 8 one-GPU emulation in bf16 and fp8 (projection inputs),
# and rocprofv3 kernel-trace stats of the Syn-1M and All_Beauty bench commands (in-step GEMM family per step).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s
mkdir -p $O
cd $R
for P in bf16 fp8; do
  timeout -k 10 500 python3 -u scripts/bench_dp_emul.py --world 1 8 --steps 60 --warmup 10 --precision $P > $O/emul_$P.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_syn1m -o run -- python3 $R/bench.py --workload syn1m --steps 200 --warmup 20 --no-cpu-baseline --probe-steps 3 > $O/prof_syn1m.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_all_beauty -o run -- python3 $R/bench.py --workload all_beauty --steps 300 --warmup 30 --no-cpu-baseline --probe-steps 5 > $O/prof_all_beauty.log 2>&1 || exit 3
echo done > $O/done
