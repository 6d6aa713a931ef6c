# d = 384 128-user producer / consumer sweep (k_dec5w_bf16): decoder parity tests (product library), the full
# Syn-1M shape, the A/B check against version 2; then version 5w against version 2 at the Syn-1M shape (A/B build,
# one process) and the Syn-1M bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_v5w}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "decoder" tests/test_gpu_large.py tests/test_gpu_ab_variant.py > $O/pytest.log 2>&1
HVAE_LIB=$R/build_var/libhvae_ab.so timeout -k 10 300 python -u scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --reps 20 --ab HVAE_DEC_V5W=1 HVAE_DEC_V5W=0 --rounds 3 > $O/ab.jsonl 2> $O/ab.log
timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 20 --probe-steps 10 --no-cpu-baseline > $O/bench_syn1m.json 2> $O/bench_syn1m.log
