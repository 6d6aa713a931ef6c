// hvae_dec5_shared.h -- version 5's tile constants, packing helpers and schedule switches, shared by the product
// sweeps in hvae_decoder5.hip and the retired d = 384 variant in ab/hvae_decoder5w.hip (A/B library only).
#pragma once
#include <cstdint>

#include "hvae_common.h"

namespace hvae {
// GEMM1 row map (version 4's DEC4_ROWMAP): MFMA row block b reads own-item block dec5_rowblk(b) of a tile half,
// which makes every ds_read_b128 lane group of the 16x16x32 A operand conflict-free in the image's chunk XOR
#ifndef DEC5_ROWMAP
#define DEC5_ROWMAP 0x1320
#endif
__device__ __forceinline__ constexpr int dec5_rowblk(int b) { return (DEC5_ROWMAP >> (4 * b)) & 3; }

namespace dec5 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kTI = 32;                  // items per tile
constexpr float kOffsetSpan = 60.0f;     // = hvae_decoder.hip
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kMinL = 8.75651e-27f;

struct Out {
  int* flag;
  float* m;
  float* l;
  float* O;
  float* lse;
  int direct;
};

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

template <int n>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14));
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

#ifndef DEC5_G1_AHEAD
#define DEC5_G1_AHEAD 2  // GEMM1 A operand k-steps in flight
#endif
#ifndef DEC5_DMA_B
#define DEC5_DMA_B 6  // of each (ug, dh)'s 12 LDS-DMA pieces per tile, how many the consumer wave issues
#endif
// Timing-ablation builds only (scripts/build_variant5.sh; outputs invalid by construction), a bit mask:
// 1 no LDS-DMA pieces in the loop (and no vmcnt waits), 2 no per-tile barrier, 4 no exponentials / P out,
// 8 GEMM1 A operands not re-read from LDS, 16 GEMM2 E^T operands not re-read, 32 no GEMM1 MFMAs,
// 64 no GEMM2 MFMAs, 128 LDS-DMA pieces issued but never waited for, 256 only the even pieces issued
#ifndef DEC5_ABL
#define DEC5_ABL 0
#endif
// Placement of the LDS-DMA pieces: producer piece i at GEMM1 k-step DEC5_PDMA_AT + DEC5_DMA_STRIDE i, consumer piece
// i at GEMM2 MFMA DEC5_CDMA_AT + DEC5_DMA_STRIDE i (as early as possible: the fill latency is the sweep's limit)
#ifndef DEC5_PDMA_AT
#define DEC5_PDMA_AT 0
#endif
#ifndef DEC5_DMA_STRIDE
#define DEC5_DMA_STRIDE 1  // MFMA gaps between a wave's consecutive pieces (profiles/r03_dec5_dma_placement_ab.jsonl)
#endif
#ifndef DEC5_CDMA_AT
#define DEC5_CDMA_AT 0
#endif
// DEC5_RSTAGE=1 (A/B): the producer stages its 12 - DEC5_DMA_B pieces of its (ug, dh) through registers (buffer_load_dwordx4
// to VGPRs one tile ahead, ds_write_b128 into the image after the barrier that frees the slot) instead of LDS-DMA
#ifndef DEC5_RSTAGE
#define DEC5_RSTAGE 0
#endif
#ifndef DEC5_DMA_BURST
#define DEC5_DMA_BURST 0  // A/B: each wave issues its pieces back to back at its first DMA slot
#endif
#ifndef DEC5_XMIX
#define DEC5_XMIX 0  // A/B (below; +1.4 %)
#endif
#ifndef DEC5_ROT
#define DEC5_ROT 0  // A/B (below; +72 %: the blocks of a split must stream their L2 lines in lockstep)
#endif
#ifndef DEC5_BFREE
#define DEC5_BFREE 0  // A/B: branch-free LDS-DMA issue in the loop
#endif
// Exponential offload (A/B builds): DEC5_EXPPOLY of the 4 item pairs per user half and tile take a packed-f32
// polynomial exp2 (exp2_pk) instead of two v_exp_f32
#ifndef DEC5_EXPPOLY
#define DEC5_EXPPOLY 0
#endif
#ifndef DEC5_EXPPOLY8  // the same for the fp8 producers' 8 pairs per lane and tile
#define DEC5_EXPPOLY8 0
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef int i32x2v __attribute__((ext_vector_type(2)));
// 2^x for a pair on the packed f32 VALU (v_pk_add_f32 / v_pk_fma_f32): Cody-Waite split x = n + f, n = rint(x)
// by the 1.5 * 2^23 shift, f in [-1/2, 1/2], 2^f by a degree-4 polynomial (relative error 4e-5, far below the
// bf16 rounding of P), 2^n added into the exponent field; x below -126 clamps (2^-126, not 0)
__device__ __forceinline__ f32x2 exp2_pk(f32x2 x) {
  const f32x2 lo = {-126.f, -126.f}, sh = {12582912.f, 12582912.f};
  x = __builtin_elementwise_max(x, lo);
  const f32x2 t = x + sh;
  const f32x2 f = x - (t - sh);
  f32x2 p = {0.0096181291f, 0.0096181291f};
  p = __builtin_elementwise_fma(p, f, f32x2{0.0555041087f, 0.0555041087f});
  p = __builtin_elementwise_fma(p, f, f32x2{0.2402265070f, 0.2402265070f});
  p = __builtin_elementwise_fma(p, f, f32x2{0.6931471806f, 0.6931471806f});
  p = __builtin_elementwise_fma(p, f, f32x2{1.f, 1.f});
  const i32x2v e = (__builtin_bit_cast(i32x2v, t) - 0x4B400000) << 23;
  return __builtin_bit_cast(f32x2, __builtin_bit_cast(i32x2v, p) + e);
}
#ifndef DEC5_P32
#define DEC5_P32 1  // producers of 32 users over one item half (GEMM1 reads each tile twice, not four times);
                    // 0 (A/B): producers of 16 users over both halves
#endif
#ifndef DEC5_PRIO
#define DEC5_PRIO 0  // A/B: static s_setprio 1 before the loop for 1 the consumer waves (4..7), 2 the producers
#endif

constexpr int D = 768;
constexpr int NS = 3;                    // tile slots
constexpr int TB = (D / 128) * 8192;     // tile bytes (48 KiB)
constexpr int PST = 80;                  // P row stride (bytes)
constexpr int LDS_BYTES = NS * TB + 2 * 2 * 32 * PST + 4 * 64 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "k_dec5_bf16 LDS");

}  // namespace dec5
}  // namespace hvae
