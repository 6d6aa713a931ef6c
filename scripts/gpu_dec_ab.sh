# Decoder A/B over prebuilt variant libraries (scripts/build_variant.sh): parity of the in-tree build,
# then the sweep timing of each variant on the bench shapes.   bash scripts/gpu_dec_ab.sh base ah1 ah2 ...
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "decoder" --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dec.log 2>&1
B=scripts/bench_decoder.py
: > gpurun_out/dec_ab.log
for v in "$@"; do
  for S in "--nb 4096 --N 100000 --D 384" "--nb 64 --N 12101 --D 384" "--nb 4096 --N 200000 --D 768"; do
    echo "# $v $S" >> gpurun_out/dec_ab.log
    HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 120 python $B $S --reps 30 2>&1 | grep -v amdgpu.ids \
      >> gpurun_out/dec_ab.log
  done
done
cat gpurun_out/dec_ab.log
