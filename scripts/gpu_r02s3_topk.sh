# Top-K scan: non-blocking bound publish + periodic reads of the other waves' bounds (HVAE_TK_TAU_PERIOD):
# parity tests, then eval throughput at the Syn-10M and Syn-1M shapes for periods 8 / 32 / 128.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/topk3
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_recommend.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for P in ${PERIODS:-8 32 128}; do
  HVAE_TK_TAU_PERIOD=$P timeout -k 10 300 python -u scripts/bench_eval.py --workload syn10m --batch 4096 --probes topk_fused --neg99-users 0 > $O/syn10m_p$P.jsonl 2>&1
  HVAE_TK_TAU_PERIOD=$P timeout -k 10 300 python -u scripts/bench_eval.py --workload syn1m --batch 4096 --probes topk_fused --neg99-users 0 > $O/syn1m_p$P.jsonl 2>&1
done
