# NDCG@10 on the planted All_Beauty stand-in (profiles/r01_ndcg_planted_gpu*.log).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ndcg.py -m gpu -x -v -s --timeout 900 --timeout-method thread > gpurun_out/pytest_ndcg.log 2>&1
