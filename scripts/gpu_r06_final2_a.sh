# Round-6 final evidence, part A on the tree the round ends on (after the finalize change moved the kernel digest):
# the PMC passes of scripts/gpu_r06_final_a.sh into gpurun_out/r06_final2, then the whole GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
export OUT=r06_final2
bash $R/scripts/gpu_r06_final_a.sh || exit $?
O=$R/gpurun_out/r06_final2
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 5
echo done > $O/done_pytest
