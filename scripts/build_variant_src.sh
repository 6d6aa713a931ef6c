# Build an A/B variant of libhvae.so with ONE source file compiled with extra -D flags.
#   scripts/build_variant_src.sh <name> <source stem, e.g. hvae_optim> [-DFLAG=...]...  -> build_var/libhvae_<name>.so
set -e
name=$1; shift
stem=$1; shift
cd "$(dirname "$0")/../recommendation-system_amd"
make -s lib
mkdir -p ../build_var
HIPCC=/opt/rocm/bin/hipcc
extra=""
[ "$stem" = "hvae_decoder5" ] && extra="-mllvm -amdgpu-mfma-vgpr-form"
[ "$stem" = "hvae_decoder6" ] && extra="-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -munsafe-fp-atomics $extra "$@" \
  -c csrc/$stem.hip -o ../build_var/${stem}_$name.o
objs=$(ls build/*.o | grep -v "/$stem.o")
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../build_var/libhvae_$name.so $objs ../build_var/${stem}_$name.o
echo "built build_var/libhvae_$name.so"
