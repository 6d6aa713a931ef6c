# GEMM long-K register ring (kRingStages = 4): GEMM and MLP tests, per-shape timings at B = 4096 (d = 384, 768),
# and the Syn-10M / Syn-1M bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_gemmring}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mlp_rows.py -x -q -k "gemm or mlp or plan" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python3 scripts/bench_gemm.py --batch 4096 --no-torch > $O/gemm_b4096.jsonl 2> $O/gemm_b4096.err
timeout -k 10 200 python3 scripts/bench_gemm.py --batch 4096 --d 768 --no-torch > $O/gemm_b4096_d768.jsonl 2> $O/gemm_b4096_d768.err
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log
timeout -k 10 300 python -u bench.py --workload syn1m --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
