# Round-3 re-entry check on the committed tree: every GPU test, smoke, the default bench (CPU baseline included).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_check}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 420 python -u bench.py > $O/bench_syn10m.json 2> $O/bench_syn10m.log
