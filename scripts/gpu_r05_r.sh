# W = 8 one-GPU emulation (scripts/bench_dp_emul.py), bf16 and fp8, each in ONE run that records the wall time,
# per-phase hipEvents of every step (three graphs, two exchanges) and a rocprofv3 kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for P in bf16 fp8; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$P -o run -- python3 -u \
    $R/scripts/bench_dp_emul.py --world 1 8 --steps 60 --warmup 10 --precision $P > $O/emul_$P.log 2>&1
  grep '"probe"' $O/emul_$P.log
done
