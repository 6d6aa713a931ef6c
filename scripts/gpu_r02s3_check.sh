# Whole GPU suite + smoke on the current tree, then Syn-1M and Syn-10M bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/syn1m.json 2> $O/syn1m.log
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --probe-steps 5 --no-cpu-baseline > $O/syn10m.json 2> $O/syn10m.log
