# Round-3 start: the default bench and the d = 768 sweep alone on the tree as round 2 left it.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_base
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log
timeout -k 10 200 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 10 > $O/dec.jsonl 2> $O/dec.log
