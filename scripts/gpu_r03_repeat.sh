# Two more runs of the default bench (Syn-10M shard, bf16) on the final tree: run-to-run spread of the headline.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_repeat}
mkdir -p $O
cd $R
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m_1.json 2> $O/bench_syn10m_1.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m_2.json 2> $O/bench_syn10m_2.log
