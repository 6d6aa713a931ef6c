// What one LDS-DMA piece costs beside MFMAs, by the form it is issued in.
//
// The bf16 sweep (k_dec5_bf16) moves each 48-KiB E tile into LDS as 48 one-KiB pieces per block (6 per wave,
// 8 waves, two per SIMD), issued between the MFMAs of the tile before, waited for (vmcnt(0)) and published by one
// barrier per tile into a 3-slot ring. This probe runs that skeleton alone -- the same grid (one 512-thread block
// per CU, 144 KiB of LDS), the same split -> XCD streaming pattern (block b streams split b % 4 of a 384-MB
// source, so the 64 blocks of a split share their XCDs' L2 as the sweep's do), the same per-SIMD MFMA work per
// tile (2 waves x 24 v_mfma_f32_32x32x16_bf16 = 1536 cycles) and optionally one ds_read_b128 of the landed tile
// per MFMA -- and swaps only the fill mechanism:
//   mode 0  no fill (MFMAs, reads, barrier)
//   mode 1  buffer_load_dwordx4 ... lds, M0 written before every piece (the product's form)
//   mode 2  global_load_lds_dwordx4 (saddr + VGPR offset), M0 written before every piece
//   mode 3  global_load_lds_dwordx4, one M0 per group of 4 pieces, the pieces told apart by the instruction's
//           offset field (which moves the global AND the LDS address: checked first, below)
//   mode 4  register staging: buffer_load_dwordx4 to VGPRs one tile ahead, ds_write_b128 after the barrier
//   mode 5  fill only (buffer ... lds form, waited per tile, no MFMAs / reads)
//   mode 6  fill only, global_load_lds_dwordx4 per-piece M0
// Wave 0 of each block stamps s_memtime / s_memrealtime around the loop (cycles per tile, in-kernel clock).
//   hipcc --offload-arch=gfx950 -O3 -o build_probe/probe_dma_issue scripts/probe_dma_issue.hip
//   build_probe/probe_dma_issue [tiles=2000] [reads=1]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kTile = 48 * 1024;   // bytes per tile (32 items x 768 bf16)
constexpr int kSlots = 3;
constexpr int kLds = kSlots * kTile;
constexpr int kPieces = 6;         // per wave per tile
constexpr int kMfma = 24;          // per wave per tile
constexpr int kSplits = 4;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// where does global_load_lds_dwordx4 ... offset:1024 with M0 = the LDS base put its bytes?
__global__ void k_offset_check(const int* __restrict__ src, int* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_raw[];
  int* lds = reinterpret_cast<int*>(lds_raw);
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = -1;
  __syncthreads();
  const uint32_t m0 = lds_addr(lds);
  const int vo = threadIdx.x * 16;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 offset:1024"
               :: "s"(m0), "v"(vo), "s"(src) : "memory");
  wait_vm0();
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

template <int MODE, bool READS>
__global__ __launch_bounds__(512) void k_probe(const unsigned char* __restrict__ src, int64_t split_bytes, int tiles,
                                               const u32x4* __restrict__ rnd, float* __restrict__ out,
                                               long long* __restrict__ clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int split = blockIdx.x % kSplits;
  const unsigned char* sbase = src + (int64_t)split * split_bytes;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(sbase), (short)0, (int)split_bytes, 0x00020000);
  const uint32_t ring0 = lds_addr(lds);
  const int vo = lane * 16;
  bf16x8 a[4], b[4];
  for (int j = 0; j < 4; ++j) {
    a[j] = __builtin_bit_cast(bf16x8, rnd[(blockIdx.x * 13 + t * 8 + j) & 8191]);
    b[j] = __builtin_bit_cast(bf16x8, rnd[(blockIdx.x * 29 + t * 8 + 4 + j) & 8191]);
  }
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j) acc[j] = f32x16{};
  u32x4 stg[kPieces];
  auto piece_src = [&](int tt, int i) { return (uint32_t)(tt * kTile + (w * kPieces + i) * 1024); };
  auto piece_lds = [&](int slot, int i) { return ring0 + (uint32_t)(slot * kTile + (w * kPieces + i) * 1024); };
  auto issue = [&](int tt, int slot, int i) {
    if constexpr (MODE == 1 || MODE == 5) {
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(piece_lds(slot, i)), "v"(vo), "s"(rsrc), "s"(piece_src(tt, i)) : "memory");
    } else if constexpr (MODE == 2 || MODE == 6) {
      const unsigned char* p = sbase + piece_src(tt, i);
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(piece_lds(slot, i)), "v"(vo), "s"(p) : "memory");
    } else if constexpr (MODE == 3) {
      // pieces i = 4 g + j: M0 and the source base once per group g, j by the offset field
      const unsigned char* p = sbase + piece_src(tt, i & ~3);
      const uint32_t m0 = piece_lds(slot, i & ~3);
      switch (i & 3) {
        case 0: asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" :: "s"(m0), "v"(vo), "s"(p) : "memory"); break;
        case 1: asm volatile("global_load_lds_dwordx4 %0, %1 offset:1024" :: "v"(vo), "s"(p) : "memory"); break;
        case 2: asm volatile("global_load_lds_dwordx4 %0, %1 offset:2048" :: "v"(vo), "s"(p) : "memory"); break;
        default: asm volatile("global_load_lds_dwordx4 %0, %1 offset:3072" :: "v"(vo), "s"(p) : "memory"); break;
      }
    } else if constexpr (MODE == 4) {
      stg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, (int)piece_src(tt, i), 0));
    }
  };
  constexpr bool kFill = MODE != 0;
  constexpr bool kMath = MODE < 5;
  // prologue: tiles 0 and 1
  if constexpr (kFill) {
    for (int i = 0; i < kPieces; ++i) issue(0, 0, i);
    if constexpr (MODE == 4) { wait_vm0(); for (int i = 0; i < kPieces; ++i) *reinterpret_cast<u32x4*>(lds + (w * kPieces + i) * 1024 + vo) = stg[i]; }
    for (int i = 0; i < kPieces; ++i) issue(1, 1, i);
    wait_vm0();
    if constexpr (MODE == 4) for (int i = 0; i < kPieces; ++i) *reinterpret_cast<u32x4*>(lds + kTile + (w * kPieces + i) * 1024 + vo) = stg[i];
  }
  barrier();
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int tt = 0; tt < tiles; ++tt) {
    const int cur = tt % kSlots, nxt2 = (tt + 2) % kSlots;
    if constexpr (kFill) wait_vm0();
    if constexpr (MODE == 4)
      if (tt + 1 < tiles && tt > 0)
        for (int i = 0; i < kPieces; ++i)
          *reinterpret_cast<u32x4*>(lds + ((tt + 1) % kSlots) * kTile + (w * kPieces + i) * 1024 + vo) = stg[i];
    barrier();  // tile tt + 1 landed, slot nxt2 free
    const bool fill = kFill && tt + 2 < tiles;
    const unsigned char* cb = lds + cur * kTile + (w & 3) * 12 * 1024;
#pragma unroll
    for (int m = 0; m < kMfma; ++m) {
      if constexpr (kMath) {
        bf16x8 x = a[m & 3];
        if constexpr (READS) x = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(cb + (m % 12) * 1024 + vo));
        acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, b[(m >> 2) & 3], acc[m & 3], 0, 0, 0);
      }
      if (fill && m < kPieces) issue(tt + 2, nxt2, m);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  wait_vm0();
  float s = 0.f;
  for (int j = 0; j < 4; ++j)
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  if constexpr (MODE == 4) s += (float)stg[0][0];
  out[blockIdx.x * 512 + t] = s + (float)lds[(t * 16) % kLds];
  if (t == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

static uint32_t lcg(uint32_t& s) { s = s * 1664525u + 1013904223u; return s; }

template <int MODE, bool READS>
static int run(const unsigned char* src, int64_t split_bytes, int tiles, const u32x4* rnd, float* out,
               long long* clk, int grid) {
  CHK(hipFuncSetAttribute((const void*)k_probe<MODE, READS>, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  auto launch = [&]() { k_probe<MODE, READS><<<grid, 512, kLds>>>(src, split_bytes, tiles, rnd, out, clk); };
  for (int w = 0; w < 20; ++w) launch();
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const int reps = 10;
  CHK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> c(2 * grid);
  CHK(hipMemcpy(c.data(), clk, grid * 16, hipMemcpyDeviceToHost));
  std::vector<double> cyc, ghz;
  for (int b = 0; b < grid; ++b) {
    cyc.push_back((double)c[2 * b] / tiles);
    ghz.push_back(c[2 * b] / (c[2 * b + 1] / 100e6) / 1e9);
  }
  std::sort(cyc.begin(), cyc.end());
  std::sort(ghz.begin(), ghz.end());
  const double per = ms / reps;
  const double fill_bytes = (MODE == 0) ? 0.0 : (double)grid * tiles * kTile;
  printf("{\"probe\": \"dma_issue\", \"mode\": %d, \"reads\": %d, \"tiles\": %d, \"ms_per_launch\": %.4f, "
         "\"us_per_tile\": %.4f, \"cycles_per_tile_median\": %.1f, \"cycles_per_tile_max\": %.1f, "
         "\"clock_ghz_median\": %.3f, \"fill_tb_s\": %.2f, \"fill_B_per_clk_cu\": %.1f}\n",
         MODE, (int)READS, tiles, per, per * 1e3 / tiles, cyc[grid / 2], cyc[grid - 1], ghz[grid / 2],
         fill_bytes / (per * 1e-3) / 1e12, (MODE == 0) ? 0.0 : kTile / cyc[grid / 2]);
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const int tiles = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int reads = argc > 2 ? std::atoi(argv[2]) : 1;
  int dev = 0, ncu = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = ncu;
  // the offset-field check
  {
    int *d_src, *d_out;
    std::vector<int> h(4096), o(1024);
    for (int i = 0; i < 4096; ++i) h[i] = i;
    CHK(hipMalloc(&d_src, 4096 * 4));
    CHK(hipMalloc(&d_out, 1024 * 4));
    CHK(hipMemcpy(d_src, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    k_offset_check<<<1, 64, 8192>>>(d_src, d_out);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(o.data(), d_out, 1024 * 4, hipMemcpyDeviceToHost));
    const bool at0 = o[0] == 256 && o[255] == 511;           // global +1024 landed at LDS +0
    const bool at1024 = o[256] == 256 && o[511] == 511 && o[0] == -1;  // ... at LDS +1024
    printf("{\"probe\": \"glds_offset_field\", \"lds_gets_offset\": %s, \"lds_ignores_offset\": %s, \"lds0\": %d, \"lds256\": %d}\n",
           at1024 ? "true" : "false", at0 ? "true" : "false", o[0], o[256]);
    fflush(stdout);
    CHK(hipFree(d_src));
    CHK(hipFree(d_out));
  }
  const int64_t split_bytes = (int64_t)tiles * kTile;
  unsigned char* d_src;
  CHK(hipMalloc(&d_src, split_bytes * kSplits));
  {
    std::vector<uint32_t> rnd(8192 * 4);
    uint32_t st = 12345;
    for (auto& w : rnd) {
      uint32_t lo = 0x3F00u | (lcg(st) >> 25) | ((lcg(st) >> 31) << 15);
      uint32_t hi = 0x3F00u | (lcg(st) >> 25) | ((lcg(st) >> 31) << 15);
      w = lo | (hi << 16);
    }
    for (int64_t off = 0; off < split_bytes * kSplits; off += (int64_t)rnd.size() * 4)
      CHK(hipMemcpy(d_src + off, rnd.data(), std::min<int64_t>(rnd.size() * 4, split_bytes * kSplits - off),
                    hipMemcpyHostToDevice));
  }
  u32x4* d_rnd;
  float* d_out;
  long long* d_clk;
  CHK(hipMalloc(&d_rnd, 8192 * 16));
  CHK(hipMalloc(&d_out, grid * 512 * 4));
  CHK(hipMalloc(&d_clk, grid * 16));
  CHK(hipMemcpy(d_rnd, d_src, 8192 * 16, hipMemcpyDeviceToDevice));
  for (int round = 0; round < 2; ++round) {
    if (reads) {
      if (run<0, true>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<1, true>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<2, true>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<3, true>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<4, true>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
    } else {
      if (run<0, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<1, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<2, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<3, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
      if (run<4, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
    }
    if (run<5, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
    if (run<6, false>(d_src, split_bytes, tiles, d_rnd, d_out, d_clk, grid)) return 1;
  }
  return 0;
}
