# fp8 sweep at d = 768 with version 4's structure (k_dec4_f8, HVAE_DEC_F8V4=1): the fp8 tests on both kernels,
# then an in-process A/B against the D-split ring at 4096 x 200,000 and the Syn-10M shard.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/f8v4
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 200000 --D 768 --reps 10 --rounds 2 --ab HVAE_DEC_F8V4=0 HVAE_DEC_F8V4=1 > $O/ab_200k.jsonl 2>&1
timeout -k 10 300 python -u scripts/bench_decoder.py --dtype fp8 --nb 4096 --N 1000000 --D 768 --reps 4 --rounds 2 --ab HVAE_DEC_F8V4=0 HVAE_DEC_F8V4=1 > $O/ab_1m.jsonl 2>&1
