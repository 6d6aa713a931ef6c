// hvae_decoder6.hip -- version 6 of the bf16 decoder sweep at d = 768 (k_dec6_bf16): 96 users per E tile.
//
// What bounds version 5: every 48-KiB E tile that reaches LDS serves 64 users, so a Syn-10M
// sweep moves 64 user blocks x 1.5 GB = 98 GB from L2 into LDS, 48 one-KiB LDS-DMA pieces per tile and block,
// and the SIMD's instruction issue (the pieces, the operand reads, the MFMAs' issue slots) is what runs out. The
// register file caps the users per tile: a user's O (fp32) and U (bf16) over d = 768 take 4.5 KiB, 96 users 432
// of the CU's 512 KiB.
//
// Here a block is 4 waves, one per SIMD with the whole 512-register file each, and holds 96 users = two groups
// of 48. Wave w = (g, h) = (w >> 1, w & 1) owns group g's users over D half h (dims 384 h .. 384 h + 383):
//   * U of its 48 users over its half (144 VGPRs): GEMM1 gives the PARTIAL S^T = E_tile[:, half] U^T of all 32
//     items of a tile (v_mfma_f32_16x16x32_bf16, 72 per tile, one ds_read_b128 A operand per 3 MFMAs);
//   * the pair (g, 0), (g, 1) completes S through LDS: each wave owns item half h of the tile (16 items), sends
//     the partner its partial of the partner's half (3 KiB) and adds the partner's partial of its own;
//   * it exponentiates its 16 items x 48 users (12 per lane) and keeps the packed P half in registers, in the
//     accumulator's lane layout, which is GEMM2's B operand as it stands; the partner's P half arrives through
//     the same LDS region (written over the partial the owner has just read, so no extra barrier);
//   * O of its 48 users over its half (288 registers): GEMM2 O^T += E^T P^T (16x16x32, 72 per tile) with E^T by
//     two ds_read_b64_tr_b16 per 16-dim block -- k slots 0..3 are the wave's own items, 4..7 the partner's, the
//     same permuted k order on both operands.
// So each E tile in LDS serves 96 users: the L2 -> LDS stream of a Syn-10M sweep drops from 98 to 65 GB and the
// 48 pieces per tile are issued for 1.5x the MFMA work. Per tile and wave: 144 MFMAs (2304 cycles), 12 pieces,
// 24 + 48 operand reads, 12 exponentials; two barriers:
//   [L: tile t + 1 landed, P(t) published]  GEMM1(t + 1) | GEMM2(t) first half | DMA of t + 2 | partial out
//   [B1: partials published]  partner partial in, softmax of t + 1, P(t + 1) out | GEMM2(t) second half
// The image, DMA piece map and the fixed-offset / flag rules are version 2's (hvae_decoder.hip); the image's chunk
// XOR is 2 * ((row >> 2) & 1), with which both the GEMM1 row reads and the GEMM2 transposed reads are bank-
// conflict free in natural row order (scripts/check_dec6_banks.py, run by tests/test_fp8_layout_cpu.py).
//
// Work assignment. 96 users do not tile a batch of 4096 over 256 CUs in equal rectangles (43 user blocks x 6
// item splits = 258 tasks), and CUs that stream the same E tiles must run on one XCD at the same time to share
// its L2. Tasks are (user block, item split) in split-major order; the first min(tasks, 256) are the main tasks
// (block b takes task (b & 7) * (grid / 8) + (b >> 3): the 32 blocks of an XCD take consecutive tasks, so each
// split is streamed by two or three XCDs, as version 5's four splits were by two). The X tasks past 256 (the last
// user blocks of the last split) are cut into P = 256 / X pieces each, and block b < X P takes piece b after its
// main task. Every task writes an (m, l, O) partial into slot rows [slot][96]; k_dec_finalize merges a user's
// slots in a fixed order (dec6_slot_of below, shared with hvae_decoder.hip).
#include <algorithm>
#include <array>

#include "../hvae_common.h"
#include "../hvae_dec6.h"

namespace hvae {
namespace dec6 {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int D = kDec6D;
constexpr int TI = 32;                  // items per tile
constexpr int NS = 3;                   // ring slots
constexpr int TB = TI * D * 2;          // tile bytes (48 KiB)
constexpr int UPB = kDec6Users;         // users per block (96)
constexpr int GU = UPB / 2;             // users per group (48)
constexpr int KS = 12;                  // GEMM1 k-steps (K = 32) over a D half
constexpr int NDB = 24;                 // GEMM2 16-dim blocks over a D half
constexpr int XB = GU * 16 * 4;         // exchange region per wave (3 KiB)
constexpr int XOFF = NS * TB;
constexpr int MOFF = XOFF + 4 * XB;     // [4 waves][48] floats: |u|^2 halves, first-tile maxima, l halves
constexpr int VOFF = MOFF + 4 * GU * 4;  // [4 waves][48] floats: the users' fixed offsets m (epilogue)
constexpr int LDS_BYTES = VOFF + 4 * GU * 4;
static_assert(LDS_BYTES <= 160 * 1024, "k_dec6_bf16 LDS");
constexpr float kOffsetSpan = 60.0f;    // = hvae_decoder.hip
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kMinL = 8.75651e-27f;

#ifndef DEC6_G2A
#define DEC6_G2A 12  // GEMM2 d-blocks run beside GEMM1 (the rest beside the softmax)
#endif
// Timing-ablation builds only (outputs invalid by construction; scripts/build_variant_src.sh), a bit mask of what
// the sweep loop leaves out: 1 the LDS-DMA pieces (and their waits), 2 the two barriers, 4 the softmax (exp2, sums,
// P packing), 8 GEMM1's A operand reads, 16 GEMM2's E^T reads, 32 GEMM1's MFMAs, 64 GEMM2's MFMAs, 128 the waits
// for the pieces (issued, never waited), 256 the partial / P exchange through LDS
// LDS-DMA placement: the last DEC6_DMAP of a tile's 12 pieces go one per phase-2 step (beside GEMM2 and the
// softmax, where a piece costs less issue time than among phase 1's operand reads); the others spread evenly
// over phase 1's 12 steps
#ifndef DEC6_DMAP
#define DEC6_DMAP 0
#endif
constexpr int kDmaP2 = DEC6_DMAP, kDmaP1 = 12 - DEC6_DMAP;
static_assert(kDmaP2 >= 0 && kDmaP2 <= 12, "DEC6_DMAP");
template <int ks>
constexpr int p1_piece() {  // the phase-1 piece issued at step ks, or -1
  constexpr int p = kDmaP1 == 0 ? 0 : (ks * kDmaP1 + 11) / 12;
  return (kDmaP1 > 0 && p < kDmaP1 && p * 12 / kDmaP1 == ks) ? p : -1;
}
#ifndef DEC6_ABL
#define DEC6_ABL 0
#endif
constexpr int kAbl = DEC6_ABL;
// Timing build only (scripts/probe_dec6_phases.py): each wave adds s_memtime deltas of the sweep loop's phases
// (wait for [L], phase 1, put + [B1], phase 2), its tile count and its kernel time into dec6_tm
#ifndef DEC6_TIMING
#define DEC6_TIMING 0
#endif
#if DEC6_TIMING
__device__ unsigned long long dec6_tm[1024 * 8];
#define DEC6_T(...) __VA_ARGS__
#else
#define DEC6_T(...)
#endif

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

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GEMM2's O accumulators: 72 f32x4 = 288 registers, more than the 256 AGPRs, beside U (144) and GEMM1's
// scores. The file is compiled with -mllvm -amdgpu-mfma-vgpr-form (the compiler's MFMAs -- GEMM1 -- write
// VGPRs); GEMM2's MFMAs are written here with the accumulator's register file named: the first 64 in AGPRs, the
// last 8 in VGPRs. The compiler neither counts nor pads an asm MFMA's latency: its B operand is made opaque one
// s_nop 1 after the VALU that builds it, and the O reads after the sweep sit behind a sched_barrier + s_nops.
constexpr int kOInAgpr = 64;
template <bool AG>
__device__ __forceinline__ void mfma_o(f32x4& c, const bf16x8& a, const bf16x8& b) {
  if constexpr (AG)
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// LDS-DMA piece i (0..11) of this wave's rows of a tile: M0 = lbase + 8192 (i >> 1) + 1024 (i & 1), source
// soff + 128 i + vlane; the first of a group waits out the readfirstlane of its SGPR operands (s_nop 4). Both
// come in computed: an s_add inside the asm would write SCC behind the compiler's back (a loop branch on SCC then
// ran the sweep's loop far past its end), and the instruction's offset field moves the LDS destination too (the
// LDS address is M0 + inst_offset + 16 lane), so the piece's source offset goes in soffset
template <int i>
__device__ __forceinline__ void dma_piece(uint32_t soff, uint32_t lbase, int vlane, __amdgpu_buffer_rsrc_t rsrc) {
  const uint32_t m0 = lbase + (uint32_t)((i >> 1) * 8192 + (i & 1) * 1024);
  const uint32_t so = soff + (uint32_t)(128 * i);
  if constexpr (i == 0)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(m0), "v"(vlane), "s"(rsrc), "s"(so) : "memory");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(m0), "v"(vlane), "s"(rsrc), "s"(so) : "memory");
}

template <bool WITH_O>
__global__ void __launch_bounds__(256, 1) k_dec6_bf16(Dec6Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, lane = tid & 63, c16 = lane & 15, kg = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = w >> 1, h = w & 1;
  float* xm = reinterpret_cast<float*>(lds + MOFF);
  float* mvl = reinterpret_cast<float*>(lds + VOFF);
  unsigned char* xw = lds + XOFF + w * XB;        // this wave's exchange region
  unsigned char* xp = lds + XOFF + (w ^ 1) * XB;  // the partner's
  const int64_t nb = a.nb;

  // LDS-DMA into version 2's image with chunk XOR 2 ((row >> 2) & 1): wave w fills rows 8 w .. 8 w + 7 of a
  // tile, 12 one-KiB pieces i = 2 seg + half (dims 128 seg + 64 half .. + 63); a piece's source offset is an
  // immediate (128 i) and its LDS place M0 = slot base + 8192 seg + 1024 half, so the loop keeps two SGPRs of
  // DMA state (the tile's byte offset, the slot's LDS base) beside the buffer resource
  const int vlane = (8 * w + ((lane >> 2) & 7)) * (D * 2) + 64 * (lane >> 5) +
                    16 * ((lane & 3) ^ (2 * ((lane >> 4) & 1)));
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a.E), (short)0, (int)(a.N * D * 2), 0x00020000);
  const uint32_t lds0 = lds_addr(lds) + (uint32_t)(w * 2048);
  auto slot_base = [&](int slot) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)(slot * TB)));
  };
  auto tile_soff = [&](int t) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)t * (uint32_t)TB));
  };
  auto issue_tile = [&](uint32_t soff, uint32_t lbase) {
    static_for<0, 12>([&](auto ic) { dma_piece<decltype(ic)::value>(soff, lbase, vlane, rsrc); });
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // GEMM1 A operand: lane (c16, kg) reads item row 16 ib + c16, dims 384 h + 32 ks + 8 kg .. + 7; ib = h (own
  // item half) and 1 - h (the partner's)
  const int laneA = (c16 >> 3) * 2048 + (c16 & 7) * 64 + 16 * (kg ^ (2 * ((c16 >> 2) & 1))) + h * (3 * 8192);
  const int aOwn = laneA + h * 4096, aPrt = laneA + (h ^ 1) * 4096;
  auto rdA = [&](const unsigned char* buf, int base, int ks) {
    return __builtin_bit_cast(bf16x8,
                              *reinterpret_cast<const uint4*>(buf + base + ((ks >> 2) << 13) + ((ks & 3) << 9)));
  };
  // GEMM2 A operand (E^T, 16 dims x 32 k slots): lane 16 kg + 4 q + p reads rows 16 ib + 4 kg + q (q = 0..3),
  // dims 384 h + 16 db + 4 p .. + 3 by ds_read_b64_tr_b16; ib = h gives k slots 0..3, ib = 1 - h slots 4..7
  const int q4 = (lane >> 2) & 3, p4 = lane & 3;
  int tOwn[2], tPrt[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int lt = (kg >> 1) * 2048 + (4 * (kg & 1) + q4) * 64 + 16 * (2 * (par ^ (kg & 1)) + (p4 >> 1)) +
                   8 * (p4 & 1) + h * (3 * 8192);
    tOwn[par] = lt + h * 4096;
    tPrt[par] = lt + (h ^ 1) * 4096;
  }
  auto rdT = [&](const unsigned char* buf, int db) {
    const int dbo = ((db >> 3) << 13) + (((db & 7) >> 1) << 9);
    auto* p0 = (__attribute__((address_space(3))) s16x4*)(void*)(buf + tOwn[db & 1] + dbo);
    auto* p1 = (__attribute__((address_space(3))) s16x4*)(void*)(buf + tPrt[db & 1] + dbo);
    const s16x4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p0);
    const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1);
    const s16x8 v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x4 O[WITH_O ? NDB : 1][3];
  DEC6_T(unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}; const unsigned long long tk0 = __builtin_amdgcn_s_memtime();)
  for (int task = 0; task < 2; ++task) {
    // ------------------------------------------------------------------------- the block's task ---
    int u, t_beg, t_end, slot;
    if (task == 0) {
      const int grid = (int)gridDim.x;
      const int b = (int)blockIdx.x;
      const int k = (grid & 7) == 0 ? (b & 7) * (grid >> 3) + (b >> 3) : b;
      const int s = k / a.nub;
      u = k - s * a.nub;
      t_beg = s * a.tps;
      t_end = min(a.ntiles, t_beg + a.tps);
      slot = k;
    } else {
      const int b = (int)blockIdx.x;
      if (a.X == 0 || b >= a.X * a.P) break;
      const int e = b / a.P, pi = b - e * a.P;
      const int K = a.main + e, s = K / a.nub;
      u = K - s * a.nub;
      const int s0 = s * a.tps, len = min(a.ntiles, s0 + a.tps) - s0;
      t_beg = s0 + (int)((int64_t)len * pi / a.P);
      t_end = s0 + (int)((int64_t)len * (pi + 1) / a.P);
      slot = a.main + b;
    }
    u = __builtin_amdgcn_readfirstlane(u);
    t_beg = __builtin_amdgcn_readfirstlane(t_beg);
    t_end = __builtin_amdgcn_readfirstlane(t_end);
    const int64_t ubase = (int64_t)u * UPB + g * GU;     // this wave's first user
    const int64_t rbase = (int64_t)slot * UPB + g * GU;  // its first partial row

    if (t_beg >= t_end) {  // an empty piece (tiny N): a neutral partial
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        const int64_t row = rbase + 16 * ub + c16;
        if (ubase + 16 * ub + c16 < nb) {
          if (h == 0 && kg == 0) { a.m[row] = -INFINITY; a.l[row] = 0.f; a.flag[row] = 0; }
          if (WITH_O) {
            float* orow = a.O + row * D + 384 * h + 4 * kg;
#pragma unroll 1
            for (int d = 0; d < 384; d += 16) *reinterpret_cast<float4*>(orow + d) = make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
      }
      continue;
    }

    // ---- U of the wave's 48 users over its D half (GEMM1's B operand) and the |u|^2 halves
    bf16x8 uf[3][KS];
    float bound[3];
    {
      float usq[3];
      const float* up = nullptr;
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        const int64_t user = ubase + 16 * ub + c16;
        const int64_t ur = user < nb ? user : nb - 1;  // rows past nb load row nb - 1, zeroed
        const float keep = user < nb ? 1.f : 0.f;
        up = a.U + ur * a.ldu + 384 * h + 8 * kg;
        if (ub > 0) asm volatile("" : "+v"(up) : "v"(uf[ub - 1][KS - 1]));  // one user block's loads at a time
        float s = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          float4 x0 = *reinterpret_cast<const float4*>(up + 32 * ks);
          float4 x1 = *reinterpret_cast<const float4*>(up + 32 * ks + 4);
          x0.x *= keep; x0.y *= keep; x0.z *= keep; x0.w *= keep;
          x1.x *= keep; x1.y *= keep; x1.z *= keep; x1.w *= keep;
          s += (x0.x * x0.x + x0.y * x0.y) + (x0.z * x0.z + x0.w * x0.w) + (x1.x * x1.x + x1.y * x1.y) +
               (x1.z * x1.z + x1.w * x1.w);
          uf[ub][ks] = bf16x8{(__bf16)x0.x, (__bf16)x0.y, (__bf16)x0.z, (__bf16)x0.w,
                              (__bf16)x1.x, (__bf16)x1.y, (__bf16)x1.z, (__bf16)x1.w};
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        usq[ub] = s;
      }
      if (kg == 0) {
#pragma unroll
        for (int ub = 0; ub < 3; ++ub) xm[w * GU + 16 * ub + c16] = usq[ub];
      }
      // tiles t_beg, t_beg + 1 -> slots 0, 1 (a second tile past t_end fills the free slot: unused)
      issue_tile(tile_soff(t_beg), slot_base(0));
      issue_tile(tile_soff(t_beg + 1), slot_base(1));
      wait_vmcnt<0>();
      barrier();  // [P0] tiles t_beg, t_beg + 1 landed; |u|^2 halves published
      const float emax = *a.e_maxnorm;
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        const float v = xm[(2 * g) * GU + 16 * ub + c16] + xm[(2 * g + 1) * GU + 16 * ub + c16];
        bound[ub] = sqrtf(v) * emax * 1.02f;
      }
    }
    if constexpr (WITH_O) {
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int ub = 0; ub < 3; ++ub) O[d][ub] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // GEMM1 of a tile: sO = own item half, sP = the partner's, partial over this D half
    f32x4 sO[3], sP[3];
    auto mask_tail = [&](int t) {  // items past N of the last tile -> -inf
      if (t == a.ntiles - 1 && (a.N & (TI - 1)) != 0) {
        const int lim = (int)(a.N - (int64_t)t * TI) - 16 * h - 4 * kg;
#pragma unroll
        for (int ub = 0; ub < 3; ++ub)
#pragma unroll
          for (int r = 0; r < 4; ++r) sO[ub][r] = r >= lim ? -INFINITY : sO[ub][r];
      }
    };
    auto put_partial = [&] {  // the partner's half of my partial -> my region
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) *reinterpret_cast<f32x4*>(xw + ub * 1024 + lane * 16) = sP[ub];
    };

    // ---- first tile: its max sets each user's fixed offset m (version 2's rule)
    float mL[3], lsum[3] = {0.f, 0.f, 0.f}, mv[3];
    uint2 pn[3];  // packed P of my item half (the next tile's), GEMM2 B operand elements 0..3
    {
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) { sO[ub] = f32x4{0.f, 0.f, 0.f, 0.f}; sP[ub] = sO[ub]; }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 x0 = rdA(lds, aOwn, ks), x1 = rdA(lds, aPrt, ks);
#pragma unroll
        for (int ub = 0; ub < 3; ++ub) sO[ub] = mfma(x0, uf[ub][ks], sO[ub]);
#pragma unroll
        for (int ub = 0; ub < 3; ++ub) sP[ub] = mfma(x1, uf[ub][ks], sP[ub]);
        __builtin_amdgcn_sched_barrier(0);
      }
      put_partial();
      barrier();  // [P1] partials of the first tile
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) sO[ub] += *reinterpret_cast<const f32x4*>(xp + ub * 1024 + lane * 16);
      mask_tail(t_beg);
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        float mx = fmaxf(fmaxf(sO[ub][0], sO[ub][1]), fmaxf(sO[ub][2], sO[ub][3]));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        mv[ub] = mx;
      }
      if (kg == 0) {
#pragma unroll
        for (int ub = 0; ub < 3; ++ub) xm[w * GU + 16 * ub + c16] = mv[ub];
      }
      barrier();  // [P2] half maxima of the pair
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        const float m = fmaxf(fmaxf(mv[ub], xm[(w ^ 1) * GU + 16 * ub + c16]), bound[ub] - kOffsetSpan);
        if (kg == 0) mvl[w * GU + 16 * ub + c16] = m;
        mL[ub] = m * kLog2e;
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sO[ub][r], kLog2e, -mL[ub]));
          lsum[ub] += pv[r];
        }
        pn[ub] = make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
        *reinterpret_cast<uint2*>(xp + ub * 512 + lane * 8) = pn[ub];  // over the partial I just read
      }
    }

    // ---- the sweep: iteration t runs GEMM2(t) and GEMM1(t + 1) (past t_end on a stale slot, results unused)
    int c0 = 0;
    for (int t = t_beg; t < t_end; ++t) {
      const int c1 = c0 == 2 ? 0 : c0 + 1, c2 = c1 == 2 ? 0 : c1 + 1;
      DEC6_T(const unsigned long long tm0 = __builtin_amdgcn_s_memtime();)
      if constexpr (!(kAbl & (1 | 128))) wait_vmcnt<0>();
      if constexpr (!(kAbl & 2)) barrier();  // [L] tile t + 1 landed, the partner's P(t) in my region, GEMM2(t - 1) done
                                              // with slot c2
      bf16x8 pb[3];  // P(t)^T: k slots 0..3 my items, 4..7 the partner's
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) {
        const uint2 pq = (kAbl & 256) ? pn[ub] : *reinterpret_cast<const uint2*>(xw + ub * 512 + lane * 8);
        pb[ub] = __builtin_bit_cast(bf16x8, make_uint4(pn[ub].x, pn[ub].y, pq.x, pq.y));
      }
      asm volatile("s_nop 1" : "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]));  // VALU write -> asm MFMA B read
      DEC6_T(const unsigned long long tm1 = __builtin_amdgcn_s_memtime();)
      const unsigned char* b0 = lds + c0 * TB;  // tile t
      const unsigned char* b1 = lds + c1 * TB;  // tile t + 1
      const uint32_t soff2 = tile_soff(t + 2), lb2 = slot_base(c2);
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) { sO[ub] = f32x4{0.f, 0.f, 0.f, 0.f}; sP[ub] = sO[ub]; }
      // phase 1: GEMM1(t + 1) | GEMM2(t) d-blocks 0 .. 11 | the 12 LDS-DMA pieces of tile t + 2 into slot c2
      bf16x8 x0 = rdA(b1, aOwn, 0), x1 = rdA(b1, aPrt, 0);
      bf16x8 y = rdT(b0, 0);
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, KS>([&](auto kc) {
        constexpr int ks = decltype(kc)::value;
        // each operand register is refilled right after the MFMAs that read it have issued, so every LDS read has
        // the other two MFMA triples (96 cycles) to land in
        if constexpr (!(kAbl & 32)) {
#pragma unroll
          for (int ub = 0; ub < 3; ++ub) sO[ub] = mfma(x0, uf[ub][ks], sO[ub]);
        } else {
#pragma unroll
          for (int ub = 0; ub < 3; ++ub) sO[ub][0] += (float)x0[ub] * (float)uf[ub][ks][0];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ks + 1 < KS && !(kAbl & 8)) x0 = rdA(b1, aOwn, ks + 1);
        if constexpr (!(kAbl & 32)) {
#pragma unroll
          for (int ub = 0; ub < 3; ++ub) sP[ub] = mfma(x1, uf[ub][ks], sP[ub]);
        } else {
#pragma unroll
          for (int ub = 0; ub < 3; ++ub) sP[ub][0] += (float)x1[ub];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ks + 1 < KS && !(kAbl & 8)) x1 = rdA(b1, aPrt, ks + 1);
        if constexpr (WITH_O) {
          if constexpr (!(kAbl & 64)) {
            mfma_o<(ks * 3 + 0 < kOInAgpr)>(O[ks][0], y, pb[0]);
            mfma_o<(ks * 3 + 1 < kOInAgpr)>(O[ks][1], y, pb[1]);
            mfma_o<(ks * 3 + 2 < kOInAgpr)>(O[ks][2], y, pb[2]);
          } else {
            O[ks][0][0] += (float)y[0] * (float)pb[0][0];
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!(kAbl & 16)) y = rdT(b0, ks + 1);
        }
        if constexpr (!(kAbl & 1) && p1_piece<ks>() >= 0) dma_piece<p1_piece<ks>()>(soff2, lb2, vlane, rsrc);
        __builtin_amdgcn_sched_barrier(0);
      });
      DEC6_T(const unsigned long long tm2 = __builtin_amdgcn_s_memtime();)
      if constexpr (!(kAbl & 256)) put_partial();
      if constexpr (!(kAbl & 2)) barrier();  // [B1] partials of tile t + 1
      DEC6_T(const unsigned long long tm3 = __builtin_amdgcn_s_memtime();)
      // phase 2: the partner's partial in, softmax of tile t + 1, P(t + 1) out | GEMM2(t) d-blocks 12 .. 23. GEMM1's
      // operand registers are dead here, so E^T is read two d-blocks ahead (y: even blocks, y2: odd) and each read
      // has two MFMA triples to land; the partner's partial is consumed one step after the barrier, and the 12
      // exponentials run 2, 1, 1, ... over steps 1 .. 11
      f32x4 xq[3];
#pragma unroll
      for (int ub = 0; ub < 3; ++ub)
        xq[ub] = (kAbl & 256) ? sP[ub] : *reinterpret_cast<const f32x4*>(xp + ub * 1024 + lane * 16);
      bf16x8 y2 = y;
      if constexpr (!(kAbl & 16)) y2 = rdT(b0, KS + 1);
      __builtin_amdgcn_sched_barrier(0);
      uint2 pq[3];
      auto soft = [&](auto ec) {  // exponential e = 4 ub + r; the block's P piece packed and stored after its 4th
        constexpr int e = decltype(ec)::value, ub = e >> 2, r = e & 3;
        if constexpr (!(kAbl & 4)) {
          sO[ub][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sO[ub][r], kLog2e, -mL[ub]));
          lsum[ub] += sO[ub][r];
        }
        if constexpr (r == 3) {
          pq[ub] = (kAbl & 4) ? make_uint2(__float_as_uint(sO[ub][0]), __float_as_uint(sO[ub][1]))
                              : make_uint2(pack_bf16x2(sO[ub][0], sO[ub][1]), pack_bf16x2(sO[ub][2], sO[ub][3]));
          if constexpr (!(kAbl & 256))
            *reinterpret_cast<uint2*>(xp + ub * 512 + lane * 8) = pq[ub];  // over the partner's partial (read above)
        }
        (void)ub; (void)r;
      };
      static_for<KS, NDB>([&](auto dc) {
        constexpr int db = decltype(dc)::value, j = db - KS;
        if constexpr (WITH_O) {
          bf16x8& yc = (db & 1) ? y2 : y;
          if constexpr (!(kAbl & 64)) {
            mfma_o<(db * 3 + 0 < kOInAgpr)>(O[db][0], yc, pb[0]);
            mfma_o<(db * 3 + 1 < kOInAgpr)>(O[db][1], yc, pb[1]);
            mfma_o<(db * 3 + 2 < kOInAgpr)>(O[db][2], yc, pb[2]);
          } else {
            O[db][0][0] += (float)yc[0] * (float)pb[0][0];
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (db + 2 < NDB && !(kAbl & 16)) yc = rdT(b0, db + 2);
        }
        if constexpr (j == 1) {
#pragma unroll
          for (int u2 = 0; u2 < 3; ++u2) sO[u2] += xq[u2];
          mask_tail(t + 1);
          if (t + 1 >= t_end) {  // past the task: the stale tile's scores contribute nothing
#pragma unroll
            for (int u2 = 0; u2 < 3; ++u2) sO[u2] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
          }
          soft(std::integral_constant<int, 0>{});
          soft(std::integral_constant<int, 1>{});
        }
        if constexpr (j >= 2) soft(std::integral_constant<int, j>{});
        if constexpr (!(kAbl & 1) && j < kDmaP2) dma_piece<kDmaP1 + j>(soff2, lb2, vlane, rsrc);
        if constexpr ((kAbl & 4) && j == 11) {
#pragma unroll
          for (int u2 = 0; u2 < 3; ++u2) lsum[u2] += 1.f;  // l >= 1: no user flagged
        }
        __builtin_amdgcn_sched_barrier(0);
      });
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) pn[ub] = pq[ub];
      c0 = c1;
      DEC6_T(const unsigned long long tm4 = __builtin_amdgcn_s_memtime(); tacc[0] += tm1 - tm0; tacc[1] += tm2 - tm1;
             tacc[2] += tm3 - tm2; tacc[3] += tm4 - tm3; tacc[4] += 1;)
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // the last asm MFMAs' results settle
    __builtin_amdgcn_sched_barrier(0);
    wait_vmcnt<0>();  // the last iteration's pieces (past t_end) before the slots are reused
#pragma unroll
    for (int ub = 0; ub < 3; ++ub) {
      lsum[ub] += __shfl_xor(lsum[ub], 16, 64);  // over the 4 lanes kg of the user
      lsum[ub] += __shfl_xor(lsum[ub], 32, 64);
    }
    barrier();  // [E0]
    if (kg == 0) {
#pragma unroll
      for (int ub = 0; ub < 3; ++ub) xm[w * GU + 16 * ub + c16] = lsum[ub];
    }
    barrier();  // [E1]
#pragma unroll
    for (int ub = 0; ub < 3; ++ub) {
      const int64_t user = ubase + 16 * ub + c16;
      if (user >= nb) continue;
      const int64_t row = rbase + 16 * ub + c16;
      const float l = xm[(2 * g) * GU + 16 * ub + c16] + xm[(2 * g + 1) * GU + 16 * ub + c16];  // l(half 0) + l(half 1)
      if (h == 0 && kg == 0) {
        a.m[row] = mvl[w * GU + 16 * ub + c16];
        a.l[row] = l;
        a.flag[row] = kAbl ? 0 : !(l >= kMinL);  // ablation builds: never the exact fixup (outputs invalid anyway)
      }
      if constexpr (WITH_O) {
        float* orow = a.O + row * D + 384 * h + 4 * kg;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
          *reinterpret_cast<float4*>(orow + 16 * db) = make_float4(O[db][ub][0], O[db][ub][1], O[db][ub][2], O[db][ub][3]);
      }
    }
    barrier();  // [E2] the exchange words are read before a next task's prologue rewrites them
  }
#if DEC6_TIMING
  tacc[5] = __builtin_amdgcn_s_memtime() - tk0;
  if (lane == 0 && blockIdx.x < 256)
    for (int i = 0; i < 6; ++i) dec6_tm[(blockIdx.x * 4 + w) * 8 + i] = tacc[i];
#endif
}

}  // namespace dec6

#if DEC6_TIMING
extern "C" int hvae_dec6_timing_fetch(unsigned long long* out) {  // [1024 waves][8], timing builds only
  HVAE_HIP(hipDeviceSynchronize());
  HVAE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dec6::dec6_tm), sizeof(dec6::dec6_tm)));
  return HVAE_OK;
}
#endif

bool dec6_plan(int64_t nb, int64_t N, Dec6Plan& p) {
  p = Dec6Plan{};
  if (nb <= 64 || N <= 0) return false;
  const int64_t ntiles = (N + 31) / 32;
  const int64_t nub = (nb + kDec6Users - 1) / kDec6Users;
  if (nub > 128 || ntiles >= (1ll << 31) / (32 * kDec6D * 2)) return false;
  int64_t S = (256 + nub - 1) / nub;
  S = std::max<int64_t>(1, std::min<int64_t>(S, ntiles / 8 > 0 ? ntiles / 8 : 1));
  const int64_t tps = (ntiles + S - 1) / S;
  S = (ntiles + tps - 1) / tps;
  const int64_t total = nub * S;
  p.nub = (int)nub;
  p.S = (int)S;
  p.tps = (int)tps;
  p.ntiles = (int)ntiles;
  if (total <= 256) {
    p.main = (int)total;
    p.X = 0;
    p.P = 0;
  } else {
    p.main = 256;
    p.X = (int)(total - 256);
    p.P = 256 / p.X;
    if (p.P < 2) return false;
  }
  p.grid = p.main;
  p.slots = p.main + p.X * p.P;
  return true;
}

// Launch of the version-6 sweep with plan p; flag / m / l / O are the slot rows [p.slots][96] (O: [.][768])
int dec6_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                const Dec6Plan& p, int* flag, float* m, float* l, float* O, hipStream_t st) {
  using namespace dec6;
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec6_bf16<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 LDS_BYTES));
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec6_bf16<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 LDS_BYTES));
    attr_set = true;
  }
  Dec6Args a{U, ldu, (const bf16_t*)E, enorm, nb, N, p.nub, p.S, p.tps, p.main, p.X, p.P, p.ntiles, flag, m, l, O};
  if (with_o)
    k_dec6_bf16<true><<<(unsigned)p.grid, 256, LDS_BYTES, st>>>(a);
  else
    k_dec6_bf16<false><<<(unsigned)p.grid, 256, LDS_BYTES, st>>>(a);
  HVAE_LAUNCH_CHECK("k_dec6_bf16");
  return HVAE_OK;
}

}  // namespace hvae
