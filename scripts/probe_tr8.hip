// Probe of ds_read_b64_tr_b8 (gfx950): lane l supplies address 8 l (+ 512 per 16-lane group); prints, for
// each receiving lane, the LDS byte address each of its 8 result bytes came from.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(int hi, int* out) {
  __shared__ unsigned char s[8192];
  for (int i = threadIdx.x; i < 8192; i += 64) s[i] = hi ? (i >> 8) : (i & 255);
  __syncthreads();
  const int l = threadIdx.x;
  const v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(void*)(s + 8 * l + 512 * (l >> 4)));
  out[2 * l] = r[0]; out[2 * l + 1] = r[1];
}
int main() {
  int* d; std::vector<int> lo(128), hi(128);
  (void)hipMalloc(&d, 512);
  k<<<1, 64>>>(0, d); (void)hipMemcpy(lo.data(), d, 512, hipMemcpyDeviceToHost);
  k<<<1, 64>>>(1, d); (void)hipMemcpy(hi.data(), d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) {
      const int a = (((hi[2 * l + b / 4] >> (8 * (b % 4))) & 255) << 8) | ((lo[2 * l + b / 4] >> (8 * (b % 4))) & 255);
      printf(" %5d", a);
    }
    printf("\n");
  }
  return 0;
}
