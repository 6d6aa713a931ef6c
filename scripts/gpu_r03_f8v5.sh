# fp8 d = 768 version 5 (k_dec5_f8, producer / consumer waves): the fp8 decoder tests on the product library
# (v5 is its d = 768 sweep), the A/B variants' checks (ring, k_dec4_f8), then v5 against the ring at the Syn-10M
# shard in one process (A/B build), interleaved rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_f8v5}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_ab_variant.py > $O/pytest.log 2>&1
HVAE_LIB=$R/build_var/libhvae_ab.so timeout -k 10 300 python -u scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 1000000 --D 768 --reps 10 --ab HVAE_DEC_F8V5=1 HVAE_DEC_F8V5=0 --rounds 3 > $O/ab.jsonl 2> $O/ab.log
