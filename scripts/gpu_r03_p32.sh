# bf16 d = 768 version-5 variants: producers of 32 users over one item half (DEC5_P32, GEMM1 reads each tile twice
# instead of four times), branch-free DMA issue, static priority. Parity of the P32 build on the d = 768 decoder
# tests, then the Syn-10M shard sweep, each arm in its own process, interleaved rounds.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r03_p32}
mkdir -p $O
cd $R
HVAE_LIB=$R/build_var/libhvae_p32.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "d768" > $O/pytest_p32.log 2>&1
HVAE_LIB=$R/build_var/libhvae_p32.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_large.py -k "768" >> $O/pytest_p32.log 2>&1
for round in 1 2 3; do
  for a in ${ARMS:-abl0 p32 bfree p32prio1}; do
    HVAE_LIB=$R/build_var/libhvae_$a.so timeout -k 10 120 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 5 --ab DUMMY=$a --rounds 1 >> $O/ab.jsonl 2>> $O/ab.log
  done
done
