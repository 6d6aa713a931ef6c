# Build an A/B variant of libhvae.so with the version-5 decoder compiled with extra -D flags.
#   scripts/build_variant5.sh <name> [-DFLAG=...]...  -> build_var/libhvae_<name>.so (load it with HVAE_LIB=...)
set -e
name=$1; shift
cd "$(dirname "$0")/../recommendation-system_amd"
make -s lib
mkdir -p ../build_var
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form "$@" \
  -c csrc/hvae_decoder5.hip -o ../build_var/dec5_$name.o
objs=$(ls build/*.o | grep -v hvae_decoder5.o)
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../build_var/libhvae_$name.so $objs ../build_var/dec5_$name.o
echo "built build_var/libhvae_$name.so"
