# Round 6, call D: the host loop's per-step batch-capacity sort removed (max_batch_nnz cached) -- Syn-1M bench
# lines; the finalize's two entry groups at D <= 512 (FIN_GROUPS=2, build_var/libhvae_fing2.so) against the
# product: finalize alone at the Syn-1M shape (CSR entries 5 + Poisson(15)), whole Syn-1M steps, and the decoder /
# train-step parity tests on that library.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
for r in 1 2 3; do
  for v in prod fing2; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 150 python -u scripts/bench_decoder.py --nb 4096 --N 100000 --D 384 --train \
      --lam 15 --probe decoder_finalize --reps 10 2>> $O/fin_ab.err | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" >> $O/fin_ab.jsonl || exit 1
  done
done
for r in 1 2; do
  for v in prod fing2; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 300 python -u bench.py --workload syn1m --steps 200 --warmup 30 --no-cpu-baseline \
      --probe-steps 3 > $O/bench_syn1m_${v}_$r.json 2>> $O/bench.err || exit 2
  done
done
HVAE_LIB=build_var/libhvae_fing2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py \
  -m gpu -x -v --timeout 300 --timeout-method thread -k "decoder or finalize or golden or step" > $O/pytest_fing2.log 2>&1 || exit 3
echo done > $O/done
