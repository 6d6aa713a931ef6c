# Round 6, call A2 (call A's first part ran: the DMA issue probe and the product's phase budget): the version-5
# sweep's per-tile phase budget of the product, the global_load_lds arm and the consumer register-staging arm
# (DEC5_CRSTAGE); their wall times against the product in alternating processes; the d = 768 decoder parity tests
# on both arms' libraries.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06a2
mkdir -p $O
cd $R
for v in d5tm d5glds_tm d5crs_tm; do
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 150 python -u scripts/probe_dec5_phases.py --label $v --reps 3 \
    >> $O/dec5_phases.jsonl 2>> $O/dec5_phases.err || exit 1
done
for r in 1 2 3; do
  for v in prod d5glds d5crs; do
    lib=build_var/libhvae_$v.so; [ $v = prod ] && lib=recommendation-system_amd/hvae/libhvae.so
    HVAE_LIB=$lib timeout -k 10 150 python -u scripts/bench_decoder.py --nb 4096 --N 1000000 --D 768 --reps 8 \
      2>> $O/dec_ab.err | sed "s/\"arm\": \"\"/\"arm\": \"$v\"/" >> $O/dec_ab.jsonl || exit 1
  done
done
for v in d5crs d5glds; do
  HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v \
    --timeout 200 --timeout-method thread -k "d768" > $O/pytest_$v.log 2>&1 || exit 1
done
echo done > $O/done
