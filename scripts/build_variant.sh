# Build an A/B variant of libhvae.so: the decoder compiled with extra -D flags, linked with the other
# objects of the in-tree build.   scripts/build_variant.sh <name> [-DFLAG=...]...
# -> build_var/libhvae_<name>.so (load it with HVAE_LIB=...)
set -e
name=$1; shift
cd "$(dirname "$0")/../recommendation-system_amd"
make -s lib
mkdir -p ../build_var
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -munsafe-fp-atomics "$@" \
  -c csrc/hvae_decoder.hip -o ../build_var/dec_$name.o
objs=$(ls build/*.o | grep -v hvae_decoder.o)
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../build_var/libhvae_$name.so $objs ../build_var/dec_$name.o
echo "built build_var/libhvae_$name.so"
