# Row-gradient plan by radix sort: the rowgrad / train / DP / large-step GPU tests on the product library, the A/B
# check (sorted == atomic, bitwise), the union row-gradient cost by world size, the Syn-1M and Syn-10M bench lines.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_rgsort}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_dp_dropin.py tests/test_gpu_ab_variant.py > $O/pytest.log 2>&1
timeout -k 10 300 python -u scripts/bench_rowgrad.py > $O/rowgrad.jsonl 2> $O/rowgrad.log
HVAE_LIB=$R/build_var/libhvae_ab.so HVAE_RG_SORTED=0 timeout -k 10 300 python -u scripts/bench_rowgrad.py >> $O/rowgrad.jsonl 2>> $O/rowgrad.log
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench_syn10m.json 2> $O/bench_syn10m.log
