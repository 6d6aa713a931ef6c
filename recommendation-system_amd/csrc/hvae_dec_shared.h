// hvae_dec_shared.h -- what the decoder sweeps share across translation units: the product sweeps in
// hvae_decoder.hip and the retired A/B variants in ab/hvae_decoder_ab.hip (built only by `make lib-ab`). The
// bf16 tile-image and fp8 tile-image layouts, the fixed-offset constants, the partial-output record and the
// sweep plan live here so that both compile against one definition.
#pragma once
#include <algorithm>
#include <cstdint>

#include "hvae_common.h"
#include "hvae_dec6.h"

namespace hvae {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

// Deferred-rescale threshold (natural-log units): O and l are rescaled only
// when a user's running max grows by more than kThr, so P = exp(s - m) stays
// <= e^kThr (bf16/fp32 range is ample; N * e^kThr << FLT_MAX for N <= 2^31).
constexpr float kThr = 20.0f;
// bf16 kernel: fixed offset within kOffsetSpan of the score bound; a user whose
// real max is more than kUnderflowSpan below its offset is recomputed exactly.
constexpr float kOffsetSpan = 60.0f;
constexpr float kUnderflowSpan = 70.0f;

struct DecOut {
  int* flag;    // [nb] (direct) / [splits][nb] (partial): 1 = recompute this user exactly (bf16 path)
  float* m;     // [splits][nb] running max      (partial mode)
  float* l;     // [splits][nb] sum exp(s - m)   (partial mode)
  float* O;     // [splits][nb][D] partial O, or final O [nb][D] (direct mode)
  float* lse;   // [nb] (direct mode)
  int direct;
};

// ------------------------------------------------------------------ bf16 ---
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two fp32 -> one packed bf16 pair (v_cvt_pk_bf16_f32, round to nearest even)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

constexpr int kBfTI = 32;          // items per tile
constexpr int kBfUsersPerWave = 32;
constexpr int kBfUsersPerBlock = 128;

__device__ __forceinline__ int bf_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
// byte offset of 16-B chunk `chunk` (0 .. D/8-1) of tile row `row` (0..31)
__device__ __forceinline__ int bf_off(int row, int chunk) {
  return ((chunk >> 4) << 13) + (row << 8) + (((chunk & 15) ^ bf_swz(row)) << 4);
}

template <int D>
constexpr int bf_tile_bytes() { return ((D + 127) / 128) * 8192; }
// The transposed tile image Et: per 32-item tile, [D rows][32 items] bf16 with the
// items of each 16-group in the k order the P operand of GEMM2 carries (middle
// two 4-groups swapped), so a GEMM2 A fragment is one 16-B ds_read_b128. (The
// ds_read_b64_tr_b16 alternative makes the compiler drain every in-flight
// LDS-DMA before each read, which serialises the tile ring on HBM latency.)
template <int D>
constexpr int bf_ttile_bytes() { return D * 64; }
__host__ __device__ constexpr int et_item_of_pos(int p) {  // tile position -> item within the tile
  return 16 * (p >> 4) + 4 * ((p >> 3) & 1) + 8 * ((p & 7) >> 2) + (p & 3);
}
// LDS ring depth: as many (E, Et) tile pairs in flight as fit in ~150 KB
template <int D>
constexpr int bf_stages() {
  return (150 * 1024) / (bf_tile_bytes<D>() + bf_ttile_bytes<D>()) >= 4
             ? 4
             : ((150 * 1024) / (bf_tile_bytes<D>() + bf_ttile_bytes<D>()) >= 3 ? 3 : 2);
}
// bf16 decoder image: E as bf16 [N][D], then (256-B aligned) Et [ntiles][D][32]
static inline int64_t et_offset_bytes(int64_t N, int64_t D) { return (N * D * 2 + 255) / 256 * 256; }

// s_waitcnt vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int n>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14));
}

constexpr float kLog2e = 1.4426950408889634f;
#ifndef DEC2_G1_AHEAD
#define DEC2_G1_AHEAD 2
#endif
#ifndef DEC2_G2_AHEAD
#define DEC2_G2_AHEAD 1
#endif
// Timing ablations of the sweep (A/B builds only, results invalid): 1 = no LDS-DMA in the loop and no
// vmcnt waits, 2 = DMA issued but never waited for, 3 = no exponentials, 4 = no DS = 2 partial-S exchange
#ifndef DEC2_ABL
#define DEC2_ABL 0
#endif
// a split's ltot below e^-60 means its max term lost precision (see k_dec2_bf16)
constexpr float kMinL = 8.75651e-27f;

template <int D, int DS>
constexpr int d2_tile_bytes() { return ((D + 127) / 128) * 8192; }
// DS = 2 exchange buffers: double-buffered by tile parity, or single (one more barrier per tile) where the
// tile is large (d = 768) so that the ring keeps three stages
template <int D>
constexpr int d2_xbufs() { return D > 384 ? 1 : 2; }
template <int D, int DS, int NW>
constexpr int d2_xbytes() { return DS == 2 ? d2_xbufs<D>() * NW * 4096 : 0; }
template <int D, int DS, int NW>
constexpr int d2_stages() {
  return (160 * 1024 - d2_xbytes<D, DS, NW>()) / d2_tile_bytes<D, DS>() >= 6
             ? 6
             : (160 * 1024 - d2_xbytes<D, DS, NW>()) / d2_tile_bytes<D, DS>();
}
template <int D, int DS, int NW>
constexpr int d2_lds_bytes() {
  return d2_stages<D, DS, NW>() * d2_tile_bytes<D, DS>() + d2_xbytes<D, DS, NW>();
}

// LDS image of one 32-item tile (version 2): per 128-column segment (8 KiB) 8-row x 32-column
// subtiles of 512 B with a 2-bit chunk XOR (cdna_hip_programming.md T10 image (a)). Row reads of the
// 32x32x16 A operand and the transposed reads both hit every bank once, and the reads of one GEMM
// differ by lane-constant offsets, so two base registers serve all of them.
__device__ __forceinline__ int d2_off(int row, int ch) {
  return ((ch >> 4) << 13) + ((row >> 3) << 11) + (((ch & 15) >> 2) << 9) + ((row & 7) << 6) +
         (((ch & 3) ^ ((row >> 2) & 3)) << 4);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ------------------------------------------------------------------- fp8 ---
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr int kF8TI = 64;  // items per tile
#ifndef F8_G2_AHEAD
#define F8_G2_AHEAD 2
#endif
#ifndef F8_SPREAD
#define F8_SPREAD 0
#endif
#ifndef F8_G1_AHEAD
#define F8_G1_AHEAD 1  // GEMM1 operand k-steps in flight (Syn-1M shape: 1 = 335 us, 2 = 344 us)
#endif
#ifndef F8_DS2_RING
#define F8_DS2_RING 1  // D = 768: 3-slot ring with the softmax split over the wave pair (0: 2-slot sequence)
#endif
#ifndef F8_DS2_AHEAD
#define F8_DS2_AHEAD 1  // d = 768 (200 K items): 1, 2, 3 ahead = 1713, 1724-1732, 1757 us
#endif

template <int D>
constexpr int f8_tile_bytes() { return 64 * D; }
template <int D>
constexpr int f8_xbytes() { return D > 384 ? 4 * (F8_DS2_RING ? 4096 : 8192) : 0; }  // DS = 2 exchange, 4 waves
template <int D>
constexpr int f8_stages() {
  return D > 384 ? (F8_DS2_RING ? 3 : 2)
                 : ((160 * 1024) / f8_tile_bytes<D>() >= 6 ? 6 : (160 * 1024) / f8_tile_bytes<D>());
}
// fp8 image: bf16 E [N][D] (exact fixups, score bound) | e4m3 tiles [ntiles][64][D] (swizzled) | int ke
static inline int64_t f8_offset_bytes(int64_t N, int64_t D) { return et_offset_bytes(N, D); }
static inline int64_t f8_tail_offset(int64_t N, int64_t D) {
  return f8_offset_bytes(N, D) + (N + kF8TI - 1) / kF8TI * 64 * D;
}
// chunk swizzle of item row `it` (only its low 4 bits matter): 3 bits where D / 16 is a multiple of 8,
// 4 bits where it is a multiple of 16 (rows 768 B / 256 B apart all start in the same bank)
__host__ __device__ constexpr int f8_sw(int D, int it) {
  return D % 256 == 0 ? (((it & 1) << 1) | (((it >> 1) & 1) << 2) | (((it >> 3) & 1) << 3) | ((it >> 2) & 1))
                      : (((it >> 1) & 1) | ((((it >> 1) ^ (it >> 2)) & 1) << 1) | (((it >> 3) & 1) << 2));
}
__host__ __device__ constexpr int f8_off(int D, int it, int ch) { return it * D + 16 * (ch ^ f8_sw(D, it)); }
// item (within its tile) of element j of lane half h of a GEMM2 B operand: the row order of the two 32x32
// S^T accumulators (j < 16: first, j >= 16: second), so P packs from them in place
__host__ __device__ constexpr int f8_item_of(int h, int j) {
  return 32 * (j >> 4) + (j & 3) + 8 * ((j & 15) >> 2) + 4 * h;
}
__device__ __forceinline__ int pack_fp8x4(float a, float b, float c, float d) {
  const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);
}

// ------------------------------------------------------------- planning ---
struct DecPlan {
  int splits;
  int64_t tiles_per_split;
  int64_t blocks;
  size_t lds;
  int v2;    // bf16 version-2 sweep (k_dec2_bf16)
  int v3;    // bf16 version-3 sweep (k_dec3_bf16, D = 768)
  int v4;    // bf16 version-4 sweep (k_dec4_bf16: D = 768 with 4 waves, D = 384 with 8)
  int v5;    // bf16 version-5 sweep (k_dec5_bf16, D = 768: 8 waves, GEMM1 and GEMM2 on different waves)
  int v6;    // bf16 version-6 sweep (k_dec6_bf16, D = 768: 96 users per E tile, task plan p6)
  Dec6Plan p6;
  int ds;    // its D split (1 or 2)
  int nw;    // its waves per block (4, or 8 with ds = 2)
  int64_t upb;
};

#if HVAE_AB
// The retired sweeps (ab/hvae_decoder_ab.hip): version 1 at D <= 384, versions 3 and 4 at D = 768 (4 at 384 too),
// the fp8 sweep with version 4's structure at D = 768. Same arguments as the product launchers.
int ab_dec_v1(bool wo, int D, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st);
int ab_dec_v3(bool wo, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st);
int ab_dec_v4(bool wo, int D, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st);
int ab_dec_f8v4(bool wo, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                const DecPlan& p, DecOut o, hipStream_t st);
#endif

}  // namespace hvae
