# Concurrent configuration packing of the grid search: its equality test, and an 8-configuration grid (All_Beauty
# stand-in, 10 epochs at B = 512, annealed beta) at concurrency 1, 2, 4.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_tune_conc}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_tune.py -x -v --timeout 300 --timeout-method thread > $O/pytest_tune.log 2>&1
timeout -k 10 700 python -u scripts/bench_tune.py --concurrent 1 2 4 > $O/tune_conc.jsonl 2> $O/tune_conc.log
