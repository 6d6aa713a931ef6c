# fp8 sweep A/B over prebuilt variant libraries (scripts/build_variant.sh): sweep timing at d = 384 / 768
set -e
mkdir -p gpurun_out
B=scripts/bench_decoder.py
: > gpurun_out/dec8_ab.log
for v in "$@"; do
  for S in "--nb 4096 --N 100000 --D 384" "--nb 4096 --N 200000 --D 768"; do
    echo "# $v $S" >> gpurun_out/dec8_ab.log
    HVAE_LIB=build_var/libhvae_$v.so timeout -k 10 120 python $B --dtype fp8 $S --reps 30 2>&1 | grep -v amdgpu.ids \
      >> gpurun_out/dec8_ab.log
  done
done
