# Round 6, call L: the final PMC passes (scripts/gpu_r06_final_a.sh) on the tree with the deferred update, then the
# whole GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_r06_final_a.sh || exit $?
O=$R/gpurun_out/r06_final
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 5
echo done > $O/done_l
