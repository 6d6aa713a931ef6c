# Build an A/B variant of libhvae.so with ONE source file compiled with extra -D flags.
#   scripts/build_variant_src.sh <name> <source stem, e.g. hvae_optim> [-DFLAG=...]...  -> build_var/libhvae_<name>.so
# A stem under csrc/ab/ (the retired sweeps, e.g. hvae_decoder6) builds on the A/B library's objects (-DHVAE_AB=1).
set -e
name=$1; shift
stem=$1; shift
cd "$(dirname "$0")/../recommendation-system_amd"
mkdir -p ../build_var
HIPCC=/opt/rocm/bin/hipcc
extra=""
[ "$stem" = "hvae_decoder5" ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
[ "$stem" = "hvae_decoder5w" ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
[ "$stem" = "hvae_decoder6" ] && extra="-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"
if [ -f csrc/ab/$stem.hip ]; then
  make -s lib-ab
  $HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -munsafe-fp-atomics -DHVAE_AB=1 $extra "$@" \
    -c csrc/ab/$stem.hip -o ../build_var/${stem}_$name.o
  objs=$(ls build/ab/*.o | grep -v "/x_$stem.o")
else
  make -s lib
  $HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -munsafe-fp-atomics $extra "$@" \
    -c csrc/$stem.hip -o ../build_var/${stem}_$name.o
  objs=$(ls build/*.o | grep -v "/$stem.o")
fi
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../build_var/libhvae_$name.so $objs ../build_var/${stem}_$name.o
rm -f ../build_var/${stem}_$name.o
echo "built build_var/libhvae_$name.so"
