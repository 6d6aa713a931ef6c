// Sustained bf16 MFMA rate on this MI355X: the practical ceiling the decoder sweep's roofline fraction is read
// against. One 256-thread block per CU (96 KiB of dynamic LDS forces it), one wave per SIMD, as in
// k_dec4_bf16. Each wave issues v_mfma_f32_32x32x16_bf16 back to back on 4 independent accumulators:
//   mode 0: operands held in registers (8 A/B fragments)
//   mode 1: both operands re-read from LDS by ds_read_b128 before every MFMA (a GEMM's operand traffic)
// on random or all-zero bf16 data (DVFS: the clock the chip holds depends on the data, MI355X_MICROARCH 'DVFS
// give-back'). Launches run back to back for ~2 s before the timed ones; wave 0 of every block stamps s_memtime /
// s_memrealtime around its loop into a buffer of its own, giving the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 -o probe_mfma_ceiling scripts/probe_mfma_ceiling.hip && ./probe_mfma_ceiling
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kLdsBytes = 96 * 1024;

template <int MODE>
__global__ __launch_bounds__(256) void k_mfma(const u32x4* __restrict__ src, float* __restrict__ out,
                                              long long* __restrict__ clk, int iters) {
  extern __shared__ u32x4 lds[];
  const int t = threadIdx.x, lane = t & 63;
  for (int i = t; i < kLdsBytes / 16; i += 256) lds[i] = src[(blockIdx.x * 97 + i) & 8191];
  __syncthreads();
  bf16x8 a[4], b[4];
  for (int j = 0; j < 4; ++j) {
    a[j] = __builtin_bit_cast(bf16x8, src[(blockIdx.x * 13 + t * 8 + j) & 8191]);
    b[j] = __builtin_bit_cast(bf16x8, src[(blockIdx.x * 29 + t * 8 + 4 + j) & 8191]);
  }
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = f32x16{};
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const int wave = t >> 6;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[j & 3], b[(j >> 1) & 3], acc[j & 3], 0, 0, 0);
    } else {
      // 8 MFMAs, each on a fresh A and B fragment read from LDS (16 B per lane, wave-contiguous: conflict free)
      const int base = ((it & 31) * 8 * 2 * 64 + wave * 32 * 1024 / 16) % (kLdsBytes / 16 - 16 * 64);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bf16x8 fa = __builtin_bit_cast(bf16x8, lds[base + (2 * j) * 64 + lane]);
        const bf16x8 fb = __builtin_bit_cast(bf16x8, lds[base + (2 * j + 1) * 64 + lane]);
        acc[j & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[j & 3], 0, 0, 0);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int j = 0; j < 4; ++j)
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  out[blockIdx.x * 256 + t] = s;
  if (t == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

static uint32_t lcg(uint32_t& s) { s = s * 1664525u + 1013904223u; return s; }

int main() {
  int dev = 0, ncu = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = ncu;
  std::vector<uint32_t> rnd(8192 * 4);
  uint32_t st = 12345;
  for (auto& w : rnd) {
    // two bf16 of magnitude ~[0.5, 2) with random sign and mantissa: no zeros, no denormals
    uint32_t lo = 0x3F00u | (lcg(st) >> 25) | ((lcg(st) >> 31) << 15);
    uint32_t hi = 0x3F00u | (lcg(st) >> 25) | ((lcg(st) >> 31) << 15);
    w = lo | (hi << 16);
  }
  u32x4 *d_rnd, *d_zero;
  float* d_out;
  long long* d_clk;
  CHK(hipMalloc(&d_rnd, 8192 * 16));
  CHK(hipMalloc(&d_zero, 8192 * 16));
  CHK(hipMalloc(&d_out, grid * 256 * 4));
  CHK(hipMalloc(&d_clk, grid * 16));
  CHK(hipMemcpy(d_rnd, rnd.data(), 8192 * 16, hipMemcpyHostToDevice));
  CHK(hipMemset(d_zero, 0, 8192 * 16));
  CHK(hipFuncSetAttribute((const void*)k_mfma<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  CHK(hipFuncSetAttribute((const void*)k_mfma<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int iters = 200000;  // 1.6 M MFMA per wave, ~25 ms per launch at 2 GHz
  const double flop = 32768.0 * 8.0 * iters * 4.0 * grid;
  for (int mode = 0; mode < 2; ++mode)
    for (int zero = 0; zero < 2; ++zero) {
      const u32x4* src = zero ? d_zero : d_rnd;
      auto launch = [&]() {
        if (mode == 0) k_mfma<0><<<grid, 256, kLdsBytes>>>(src, d_out, d_clk, iters);
        else k_mfma<1><<<grid, 256, kLdsBytes>>>(src, d_out, d_clk, iters);
      };
      for (int w = 0; w < 80; ++w) launch();  // ~2 s back to back before the timed launches
      CHK(hipDeviceSynchronize());
      const int reps = 40;
      CHK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<long long> clk(2 * grid);
      CHK(hipMemcpy(clk.data(), d_clk, grid * 16, hipMemcpyDeviceToHost));
      std::vector<double> ghz;
      for (int b = 0; b < grid; ++b) ghz.push_back(clk[2 * b] / (clk[2 * b + 1] / 100e6) / 1e9);
      std::sort(ghz.begin(), ghz.end());
      const double per = ms / reps;
      const double cyc = 32.0 * 8.0 * iters;  // MFMA cycles per SIMD per launch
      printf("{\"probe\": \"mfma_ceiling\", \"operands\": \"%s\", \"data\": \"%s\", \"ms_per_launch\": %.3f, "
             "\"tflops\": %.1f, \"frac_of_2500\": %.3f, \"clock_ghz_median\": %.3f, \"mfma_cycles_per_ghz_ms\": %.3f}\n",
             mode ? "lds_b128" : "registers", zero ? "zero" : "random", per, flop / (per * 1e-3) / 1e12,
             flop / (per * 1e-3) / 2.5e15, ghz[grid / 2], cyc / (ghz[grid / 2] * 1e6));
      fflush(stdout);
    }
  return 0;
}
