// Probe of v_mfma_scale_f32_32x32x64_f8f6f4 operand/scale semantics and v_cvt_pk_fp8_f32 rounding
// (gfx950, OCP e4m3). Exact small-integer data; prints PASS/FAIL per hypothesis.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_mm(const uint8_t* A8, const uint8_t* B8, const int* sa, const int* sb, float* C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int w = 0; w < 8; ++w) {
    a[w] = *(const int*)(A8 + l * 32 + 4 * w);
    b[w] = *(const int*)(B8 + l * 32 + 4 * w);
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 16; ++r) C[l * 16 + r] = acc[r];
}
__global__ void k_cvt(const float* x, uint8_t* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n) {
    const int p = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
    y[2 * i] = p & 255; y[2 * i + 1] = (p >> 8) & 255;
  }
}
static float e4m3_val(uint8_t b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  float v = e == 0 ? ldexpf((float)m, -9) : ldexpf(1.f + m / 8.f, e - 7);
  if (e == 15 && m == 7) v = NAN;
  return s ? -v : v;
}
static uint8_t e4m3_rne(float x) {  // reference: nearest (ties to even code), saturating at 448
  int best = 0; float bd = INFINITY;
  for (int c = 0; c < 256; ++c) {
    const float v = e4m3_val((uint8_t)c);
    if (std::isnan(v)) continue;
    const float d = fabsf(v - x);
    if (d < bd || (d == bd && (c & 1) == 0 && (best & 1))) { bd = d; best = c; }
  }
  return (uint8_t)best;
}
int main() {
  // A[32][64], B[64][32] small ints; lane l holds A[l&31][32(l>>5)+j], B[32(l>>5)+j][l&31] (hypothesis H1)
  std::vector<uint8_t> A8(64 * 32), B8(64 * 32);
  std::vector<float> A(32 * 64), B(64 * 32);
  uint32_t seed = 12345;
  auto rnd = [&] { seed = seed * 1664525u + 1013904223u; return (int)((seed >> 16) % 9) - 4; };
  for (int i = 0; i < 32; ++i) for (int k = 0; k < 64; ++k) A[i * 64 + k] = (float)rnd();
  for (int k = 0; k < 64; ++k) for (int j = 0; j < 32; ++j) B[k * 32 + j] = (float)rnd();
  for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
    A8[l * 32 + j] = e4m3_rne(A[(l & 31) * 64 + 32 * (l >> 5) + j]);
    B8[l * 32 + j] = e4m3_rne(B[(32 * (l >> 5) + j) * 32 + (l & 31)]);
  }
  // scales: A lane l -> 127 + (l % 3) - 1; B lane l -> 127 + (l % 5) - 2 (hypothesis H2: lane scale = (row/col, k-half))
  std::vector<int> sa(64), sb(64);
  for (int l = 0; l < 64; ++l) { sa[l] = 127 + (l % 3) - 1; sb[l] = 127 + (l % 5) - 2; }
  uint8_t *dA, *dB; int *dsa, *dsb; float* dC;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dC, 4096);
  hipMemcpy(dA, A8.data(), 2048, hipMemcpyHostToDevice); hipMemcpy(dB, B8.data(), 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice); hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
  k_mm<<<1, 64>>>(dA, dB, dsa, dsb, dC);
  std::vector<float> C(1024);
  hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
  // hypotheses for the scale block of element j of lane half h (blk) and which lane supplies it
  const char* names[4] = {"blk = h (lane's own 32)", "blk = j >> 4 (interleaved 16s)", "blk = (j >> 3) & 1", "blk = j >> 4, scale lane = row|col only"};
  for (int hyp = 0; hyp < 4; ++hyp) {
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
      const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      double want = 0;
      for (int h = 0; h < 2; ++h) for (int j = 0; j < 32; ++j) {
        const int k = 32 * h + j;  // the logical k this (h, j) slot carries in my layout
        const int blk = hyp == 0 ? h : hyp == 1 ? (j >> 4) : hyp == 2 ? ((j >> 3) & 1) : (j >> 4);
        const int la = hyp == 3 ? row : row + 32 * blk, lb = hyp == 3 ? col : col + 32 * blk;
        want += A[row * 64 + k] * ldexp(1.0, sa[la] - 127) * B[k * 32 + col] * ldexp(1.0, sb[lb] - 127);
      }
      if (fabs(want - C[l * 16 + r]) > 1e-3) ++bad;
    }
    printf("scale hypothesis %d (%s): %s (%d bad)\n", hyp, names[hyp], bad ? "FAIL" : "PASS", bad);
  }
  // per-column-uniform B scales, per-row-uniform A scales (what the decoder relies on)
  for (int l = 0; l < 64; ++l) { sa[l] = 127 + ((l & 31) % 3) - 1; sb[l] = 127 + ((l & 31) % 5) - 2; }
  hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice); hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
  k_mm<<<1, 64>>>(dA, dB, dsa, dsb, dC);
  hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
  {
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
      const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      double want = 0;
      for (int k = 0; k < 64; ++k) want += A[row * 64 + k] * B[k * 32 + col];
      want *= ldexp(1.0, sa[row] - 127) * ldexp(1.0, sb[col] - 127);
      if (fabs(want - C[l * 16 + r]) > 1e-3) { if (bad < 3) printf("  uniform: row %d col %d got %g want %g\n", row, col, C[l * 16 + r], want); ++bad; }
    }
    printf("per-row A / per-column B uniform scales: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
  }
  // uniform-scale check (only A/B mapping consistency)
  for (int l = 0; l < 64; ++l) { sa[l] = 127; sb[l] = 127; }
  hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice); hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
  k_mm<<<1, 64>>>(dA, dB, dsa, dsb, dC);
  hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
    const int col = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    double want = 0;
    for (int k = 0; k < 64; ++k) want += A[row * 64 + k] * B[k * 32 + col];
    if (fabs(want - C[l * 16 + r]) > 1e-3) ++bad;
  }
  printf("H1 (unit scales): %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
  // cvt rounding vs nearest-even e4m3
  const int n = 1 << 16;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) x[i] = ldexpf(1.f + (i % 4096) / 4096.f, (i / 4096) % 16 - 10) * ((i & 1) ? -1.f : 1.f);
  float* dx; uint8_t* dy; hipMalloc(&dx, n * 4); hipMalloc(&dy, n);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k_cvt<<<n / 2 / 256, 256>>>(dx, dy, n);
  std::vector<uint8_t> y(n);
  hipMemcpy(y.data(), dy, n, hipMemcpyDeviceToHost);
  bad = 0;
  for (int i = 0; i < n; ++i) if (fabsf(x[i]) <= 448.f && y[i] != e4m3_rne(x[i])) { if (bad < 5) printf("  cvt %g -> %02x want %02x\n", x[i], y[i], e4m3_rne(x[i])); ++bad; }
  printf("cvt_pk_fp8 == RNE e4m3: %s (%d bad)\n", bad ? "FAIL" : "PASS", bad);
  return 0;
}
