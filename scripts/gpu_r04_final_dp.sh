# Round-4 final evidence, data parallel: one W = 8 rank's step emulated on one GPU (scripts/bench_dp_emul.py) on the
# final tree, and its kernel-trace stats
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r04_final}
mkdir -p $O
cd $R
timeout -k 10 400 python -u scripts/bench_dp_emul.py --world 1 8 --steps 20 --warmup 6 > $O/dp_emul.jsonl 2> $O/dp_emul.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dp -o run -- python3 $R/scripts/bench_dp_emul.py --world 8 --steps 14 --warmup 4 > $O/prof_dp.log 2>&1
cat $O/dp_emul.jsonl
