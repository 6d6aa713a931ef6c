// hvae_decoder5.hip -- version 5 of the bf16 decoder sweep at d = 768 (k_dec5_bf16) and its fp8 form
// (k_dec5_f8): GEMM1 and GEMM2 on different waves (producer / consumer specialisation, two waves per SIMD).
//
// Version 4 (hvae_decoder.hip, k_dec4_bf16, A/B build) runs one wave per SIMD that does everything for its
// (user group ug, D half dh): the LDS-DMA of the next tiles, GEMM1 S^T = E_tile U^T for its 16 items
// over all of D, the exponentials, and GEMM2 O^T += E_tile^T P^T for its D half. At one wave per
// SIMD nothing covers the issue cost of the 12 LDS-DMA pieces per tile, nor any LDS-read latency an
// MFMA waits on (profiles/r02_dec4_ablations.jsonl: the sweep is 18 % faster without the DMA).
//
// Here a block is 8 waves, two per SIMD (waves q and q + 4 share one: the workgroup's waves go to the
// SIMDs in a cyclic order of 4). For q = 0..3, (ug, dh) = (q & 1, q >> 1):
//   * producer wave q (role 0): U of user group ug's 32 users over all of D (192 VGPRs; DEC5_P32); per
//     tile: its share of the LDS-DMA pieces of tile t + 2, GEMM1 of tile t + 1 for items 16 dh .. 16 dh + 15
//     (48 16x16x32 MFMAs, one A read serving both 16-user halves), its 8 exponentials, its P piece -> LDS;
//     DEC5_P32=0 (A/B) gives the producer 16 users over both item halves (96 VGPRs, twice the GEMM1 reads);
//   * consumer wave q + 4 (role 1): O of user group ug over D half dh (192 VGPRs: the file is compiled
//     with -mllvm -amdgpu-mfma-vgpr-form, so that no AGPR block is allocated beside the producer's
//     VGPRs and each wave fits the 256 registers of two waves per SIMD); per tile: GEMM2 of tile t
//     over both item halves (24 32x32x16 MFMAs) with P(t) read back from LDS, and its share of the pieces.
// The SIMD's two instruction streams interleave in hardware, so one wave's DMA issue, LDS waits and
// exponentials run under the other's MFMAs. The MFMA work per SIMD and tile is version 4's (1536
// cycles), as are the LDS image, the DMA piece map, the P layout and the fixed-offset / flag rules. One
// barrier per tile:
//   [barrier: tile t + 1 landed, P(t) published, GEMM2(t - 1) done]
//   producers: DMA of t + 2 into the slot GEMM2(t - 1) freed | GEMM1(t + 1) | softmax | P(t + 1) out
//   consumers: GEMM2(t) from slot t % 3 and P(t)
// What bounds it (profiles/r03_dec5_ablation_*.jsonl): the E stream. 64 users per 48-KiB tile
// is 98 GB of L2 -> LDS traffic per Syn-10M sweep; the stream alone, waited per tile as the ring needs,
// takes 9.4 ms of the 10.1-10.4, while the MFMAs alone take 6.9.
#include <algorithm>
#include <array>

#include "hvae_common.h"
#include "hvae_dec5_shared.h"

namespace hvae {
namespace dec5 {

// Timing build only (DEC5_TIMING=1, scripts/probe_dec5_phases.py; outputs unchanged): each wave of k_dec5_bf16 adds
// s_memtime deltas of its loop's phases -- producer: [vmcnt wait | barrier | GEMM1 with its DMA pieces | tail mask,
// exponentials, P out]; consumer: [vmcnt wait | barrier | P read, GEMM2 with its DMA pieces | -] -- its tile
// count, its kernel cycles, the s_memrealtime span of the same interval (in-kernel clock) and its role into dec5_tm
#ifndef DEC5_TIMING
#define DEC5_TIMING 0
#endif
#if DEC5_TIMING
__device__ unsigned long long dec5_tm[2048 * 8];
#define DEC5_T(...) __VA_ARGS__
#else
#define DEC5_T(...)
#endif
// DEC5_GLDS=1 (A/B): the LDS-DMA pieces as global_load_lds_dwordx4 (64-bit SGPR base + the lane's VGPR offset, no
// buffer descriptor) instead of buffer_load_dwordx4 ... lds. Rows past N of the last tile then read the image's
// next bytes (the tile-transposed copy: finite bf16) instead of the descriptor's zeros; their P is 0 (tail mask)
#ifndef DEC5_GLDS
#define DEC5_GLDS 0
#endif
#ifndef DEC5_CRSTAGE
#define DEC5_CRSTAGE 0
#endif

template <bool WITH_O>
__global__ void __launch_bounds__(512) k_dec5_bf16(const float* __restrict__ U, int64_t ldu,
                                                   const bf16_t* __restrict__ E, const float* __restrict__ e_maxnorm,
                                                   int64_t nb, int64_t N, int splits, int64_t tiles_per_split,
                                                   Out out) {
  constexpr int DW = D / 2;      // GEMM2: dims owned by one consumer wave
  constexpr int DB = DW / 32;    // GEMM2 d-blocks (12)
  constexpr int KS = D / 32;     // GEMM1 k-steps (24)
  constexpr int PW = 12;         // 1-KiB LDS-DMA pieces per (ug, dh) per tile
  constexpr int PB = DEC5_DMA_B;
  constexpr int PA = PW - PB;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* pbuf = lds + NS * TB;                                  // [2 parity][2 ug][32 users][PST]
  float* xm = reinterpret_cast<float*>(lds + NS * TB + 2 * 2 * 32 * PST);  // [2 ug][l 32 | m 32]

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int c16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int role = w >> 2, q = w & 3;
  const int ug = q & 1, dh = q >> 1;
  DEC5_T(unsigned long long tacc[4] = {0, 0, 0, 0}, ntl = 0;
         const unsigned long long tk0 = __builtin_amdgcn_s_memtime(), rk0 = __builtin_amdgcn_s_memrealtime();
         auto tm_store = [&] {
           if (lane == 0 && blockIdx.x < 256) {
             unsigned long long* o = dec5_tm + (blockIdx.x * 8 + w) * 8;
             o[0] = tacc[0]; o[1] = tacc[1]; o[2] = tacc[2]; o[3] = tacc[3]; o[4] = ntl;
             o[5] = __builtin_amdgcn_s_memtime() - tk0; o[6] = __builtin_amdgcn_s_memrealtime() - rk0; o[7] = role;
           }
         };)
  // block -> (user block, split): by default split = b % splits, so with 4 splits each XCD (b % 8) streams one
  // split; DEC5_XMIX (A/B) deals each XCD's blocks over all splits (b / 8 picks the split) when the grid allows
  int split, ublk;
  if (DEC5_XMIX && gridDim.x % (8 * splits) == 0) {
    const int r = blockIdx.x / 8;
    split = r % splits;
    ublk = (r / splits) * 8 + (blockIdx.x & 7);
  } else {
    split = blockIdx.x % splits;
    ublk = blockIdx.x / splits;
  }
  const int64_t u0 = (int64_t)ublk * 64 + ug * 32;
  const int64_t ntiles = (N + kTI - 1) / kTI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const int dbase = dh * DW;

  // LDS-DMA into version 2's image (version 3's pieces): piece p = q * 12 + i
  int vlane[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int row = 8 * pb + ((lane >> 2) & 7);
    vlane[pb] = ((lane >> 2) & 7) * (D * 2) + 64 * (lane >> 5) + 16 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(E), (short)0, (int)(N * D * 2), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(q * PW * 1024);
#ifndef DEC5_DMA_NT
#define DEC5_DMA_NT 0  // A/B: non-temporal cache policy on the LDS-DMA pieces
#endif
#if DEC5_DMA_NT
#define DEC5_POL " nt"
#else
#define DEC5_POL ""
#endif
  auto issue_piece = [&](uint32_t soff, int slot_i, int i, bool fresh) {
    if ((DEC5_ABL & 256) && (i & 1)) return;
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
    const int p = q * PW + i;
    const uint32_t so = soff + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (p & 1));
    const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
#if DEC5_GLDS
    const unsigned char* src = reinterpret_cast<const unsigned char*>(E) + so;  // wave-uniform: an SGPR pair
    if (fresh)
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" DEC5_POL
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(src) : "memory");
    else
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" DEC5_POL
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(src) : "memory");
#else
    if (fresh)
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen" DEC5_POL " lds"
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
    else
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen" DEC5_POL " lds"
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
#endif
  };
  auto tile_soff = [&](int64_t t) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)(kTI * D * 2)));
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto p_row = [&](int par, int uu) { return pbuf + ((par * 2 + ug) * 32 + uu) * PST; };
  // DEC5_ROT (A/B): the i-th piece a wave issues in a tile is piece (i + user block) mod its count, so that the
  // blocks of one split, which stream the same tiles from their XCD's L2 in near lockstep, ask for different
  // lines at a time
  const int rot = __builtin_amdgcn_readfirstlane(ublk);
  auto prot = [&](int i, int n) { return DEC5_ROT ? (i + rot) % n : i; };
  if ((DEC5_PRIO == 1 && role == 1) || (DEC5_PRIO == 2 && role == 0)) __builtin_amdgcn_s_setprio(1);

  if (DEC5_P32 && role == 0) {
    // ------------------------------------------------------- producer, 32 users (A/B) ---
    // producer q = (ug, ih) owns item half ih of every tile for all 32 users of ug (version 4's GEMM1: U over
    // all of D for 32 users in 192 VGPRs, one A read per k-step serving both 16-user halves), so the producers
    // read each tile twice from LDS instead of four times; the first tile's max crosses once between the two
    // producers of a user group (xmax), and l = l(half 0) + l(half 1) at the end
    const int ih = dh;
    float* xmax = xm + 128;  // [4 producers][32 users]
    const float emax = *e_maxnorm;
    bf16x8 uf[2][KS];  // GEMM1's B operand: lane holds U[u0 + 16 uh + c16][32 ks + 8 g .. + 7]
    float bound[2];
#pragma unroll
    for (int uh = 0; uh < 2; ++uh) {
      const int64_t ub = u0 + 16 * uh + c16;
      const int64_t ur = ub < nb ? ub : nb - 1;  // rows past nb load row nb - 1, zeroed
      const float keep = ub < nb ? 1.f : 0.f;
      float usq = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const float* up = U + ur * ldu + 32 * ks + 8 * g;
        if (ks > 0) asm volatile("" : "+v"(up) : "v"(uf[uh][ks - 1]));  // one k-step's loads live at a time
        float4 a = *reinterpret_cast<const float4*>(up);
        float4 b = *reinterpret_cast<const float4*>(up + 4);
        a.x *= keep; a.y *= keep; a.z *= keep; a.w *= keep;
        b.x *= keep; b.y *= keep; b.z *= keep; b.w *= keep;
        usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
        uf[uh][ks] = bf16x8{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                            (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
      }
      usq += __shfl_xor(usq, 16, 64);
      usq += __shfl_xor(usq, 32, 64);
      bound[uh] = sqrtf(usq) * emax * 1.02f;
    }
    const int gi = dec5_rowblk(g);  // MFMA rows 4 g .. 4 g + 3 hold items 4 gi .. 4 gi + 3 of the half
    const int r1 = 16 * ih + 4 * dec5_rowblk(c16 >> 2) + (c16 & 3);
    const int laneA = ((r1 >> 3) << 11) + ((r1 & 7) << 6) + ((g ^ ((r1 >> 2) & 3)) << 4);
    auto gemm1 = [&](const unsigned char* buf, f32x4 (&s)[2], auto&& fill) {
#pragma unroll
      for (int uh = 0; uh < 2; ++uh)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[uh][r] = 0.f;
      auto rdA = [&](int ks) {
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(buf + laneA + ((ks >> 2) << 13) +
                                                                         ((ks & 3) << 9)));
      };
      constexpr int AH = DEC5_G1_AHEAD;
      bf16x8 a[AH];
#pragma unroll
      for (int j = 0; j < AH; ++j) a[j] = rdA(j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 c = a[ks % AH];
        if (ks + AH < KS) a[ks % AH] = rdA(ks + AH);
        s[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, uf[0][ks], s[0], 0, 0, 0);
        s[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, uf[1][ks], s[1], 0, 0, 0);
        fill(ks);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    float m[2] = {0.f, 0.f}, mL[2] = {0.f, 0.f}, lsum[2] = {0.f, 0.f};
    f32x4 s_nx[2];
    auto mask_tail = [&](f32x4 (&s)[2], int64_t t) {
      if (t == ntiles - 1 && (N % kTI) != 0) {
        const int lim = (int)(N - t * kTI) - 16 * ih - 4 * gi;
#pragma unroll
        for (int uh = 0; uh < 2; ++uh)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[uh][r] = r >= lim ? -INFINITY : s[uh][r];
      }
    };
    auto p_out = [&](int par) {  // 8 exponentials (4 items x 2 users), the sums, the packed P row pieces -> LDS
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (uh * 2 + (r >> 1) < DEC5_EXPPOLY) {  // A/B: the pair (r, r + 1) on the packed polynomial
            if ((r & 1) == 0) {
              const f32x2 x = {__builtin_fmaf(s_nx[uh][r], kLog2e, -mL[uh]), __builtin_fmaf(s_nx[uh][r + 1], kLog2e, -mL[uh])};
              const f32x2 y = exp2_pk(x);
              pv[r] = y[0];
              pv[r + 1] = y[1];
              lsum[uh] += pv[r];
              lsum[uh] += pv[r + 1];
            }
            continue;
          }
          pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[uh][r], kLog2e, -mL[uh]));
          lsum[uh] += pv[r];
        }
        *reinterpret_cast<uint2*>(p_row(par, 16 * uh + c16) + 2 * (16 * ih + 8 * (gi & 1) + 4 * (gi >> 1))) =
            make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
      }
    };
    if (t_beg < t_end) {
      for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg), 0, i, i == 0);
      if (t_beg + 1 < t_end)
        for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
      wait_vmcnt<0>();
    }
    barrier();  // [P0] tiles t_beg (and t_beg + 1) landed (consumers' pieces too)
    float mh[2] = {0.f, 0.f};
    if (t_beg < t_end) {
      gemm1(lds, s_nx, [](int) {});
      mask_tail(s_nx, t_beg);
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        float mx = fmaxf(fmaxf(s_nx[uh][0], s_nx[uh][1]), fmaxf(s_nx[uh][2], s_nx[uh][3]));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        mh[uh] = mx;
        if (g == 0) xmax[q * 32 + 16 * uh + c16] = mx;
      }
    }
    barrier();  // [PX] the first tile's half maxima of both producers of the user group
    if (t_beg < t_end) {
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        m[uh] = fmaxf(fmaxf(mh[uh], xmax[(q ^ 2) * 32 + 16 * uh + c16]), bound[uh] - kOffsetSpan);
        mL[uh] = m[uh] * kLog2e;
      }
      p_out(0);  // P(t_beg) -> parity 0
    }
    barrier();  // [P1]
    for (int64_t t = t_beg; t < t_end; ++t) {
      const int li = (int)(t - t_beg);
      const int nxt = (li + 1) % NS, s_dma = (li + 2) % NS, par = li & 1;
      DEC5_T(const unsigned long long tm0 = __builtin_amdgcn_s_memtime();)
      if (!(DEC5_ABL & (1 | 128))) wait_vmcnt<0>();
      DEC5_T(const unsigned long long tm1 = __builtin_amdgcn_s_memtime();)
      barrier();  // [L] tile t + 1 landed, P(t) published, GEMM2(t - 1) done
      DEC5_T(const unsigned long long tm2 = __builtin_amdgcn_s_memtime(); unsigned long long tm3 = tm2;)
      if (t + 1 < t_end) {
        const uint32_t soff_dma = tile_soff(t + 2);  // branch-free: past the split the pieces fill the free slot
        gemm1(lds + nxt * TB, s_nx, [&](int ks) {
          const int kk = ks - DEC5_PDMA_AT;
          if (!(DEC5_ABL & 1) && kk >= 0 && kk % DEC5_DMA_STRIDE == 0 && kk / DEC5_DMA_STRIDE < PA) issue_piece(soff_dma, s_dma, prot(kk / DEC5_DMA_STRIDE, PA), kk == 0);
        });
        DEC5_T(tm3 = __builtin_amdgcn_s_memtime();)
        mask_tail(s_nx, t + 1);
        p_out(par ^ 1);
      }
      DEC5_T(const unsigned long long tm4 = __builtin_amdgcn_s_memtime(); tacc[0] += tm1 - tm0; tacc[1] += tm2 - tm1;
             tacc[2] += tm3 - tm2; tacc[3] += tm4 - tm3; ++ntl;)
    }
    wait_vmcnt<0>();
#pragma unroll
    for (int uh = 0; uh < 2; ++uh) {
      lsum[uh] += __shfl_xor(lsum[uh], 16, 64);  // over the 4 lanes g of the user
      lsum[uh] += __shfl_xor(lsum[uh], 32, 64);
    }
    barrier();  // [PE0]
    if (g == 0) {
      xmax[q * 32 + c16] = lsum[0];
      xmax[q * 32 + 16 + c16] = lsum[1];
    }
    barrier();  // [E0]
    if (ih == 0 && g == 0) {  // l = l(half 0) + l(half 1), in that order
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        xm[ug * 64 + 16 * uh + c16] = lsum[uh] + xmax[(q ^ 2) * 32 + 16 * uh + c16];
        xm[ug * 64 + 32 + 16 * uh + c16] = m[uh];
      }
    }
    barrier();  // [E1]
    DEC5_T(tm_store();)
    return;
  }
  if (role == 0) {
    // ------------------------------------------------------------------ producer ---
    // producer q owns users u0 + 16 uh + c16 (uh = q >> 1) over both item halves of every tile: U of
    // its 16 users over all of D in 96 VGPRs (version 4 held 32 users' U in 192 and split the items)
    const int uh = dh;
    const int64_t ub = u0 + 16 * uh + c16;
    const float emax = *e_maxnorm;
    bf16x8 uf[KS];  // GEMM1's B operand: lane holds U[ub][32 ks + 8 g .. + 7]
    float usq = 0.f;
    {
      const int64_t ur = ub < nb ? ub : nb - 1;  // branch-free: rows past nb load row nb - 1, zeroed
      const float keep = ub < nb ? 1.f : 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        float4 a = *reinterpret_cast<const float4*>(U + ur * ldu + 32 * ks + 8 * g);
        float4 b = *reinterpret_cast<const float4*>(U + ur * ldu + 32 * ks + 8 * g + 4);
        a.x *= keep; a.y *= keep; a.z *= keep; a.w *= keep;
        b.x *= keep; b.y *= keep; b.z *= keep; b.w *= keep;
        usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
        uf[ks] = bf16x8{(__bf16)a.x, (__bf16)a.y, (__bf16)a.z, (__bf16)a.w,
                        (__bf16)b.x, (__bf16)b.y, (__bf16)b.z, (__bf16)b.w};
      }
    }
    float bound;
    {
      float v = usq;
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      bound = sqrtf(v) * emax * 1.02f;
    }
    // GEMM1: S^T[32 items][16 users] over all of D, item halves ih: A = image row 16 ih + 4 dec5_rowblk(c16 >> 2)
    // + (c16 & 3) (version 4's conflict-free row map), chunk 4 ks + g
    int laneA[2];
    const int gi = dec5_rowblk(g);  // MFMA rows 4 g .. 4 g + 3 hold items 4 gi .. 4 gi + 3 of each half
#pragma unroll
    for (int ih = 0; ih < 2; ++ih) {
      const int r1 = 16 * ih + 4 * dec5_rowblk(c16 >> 2) + (c16 & 3);
      laneA[ih] = ((r1 >> 3) << 11) + ((r1 & 7) << 6) + ((g ^ ((r1 >> 2) & 3)) << 4);
    }
    auto gemm1 = [&](const unsigned char* buf, f32x4 (&s)[2], auto&& fill) {
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[ih][r] = 0.f;
      auto rdA = [&](int ih, int ks) {
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(buf + laneA[ih] + ((ks >> 2) << 13) +
                                                                         ((ks & 3) << 9)));
      };
      constexpr int AH = DEC5_G1_AHEAD;
      bf16x8 a[AH][2];
#pragma unroll
      for (int j = 0; j < AH; ++j) { a[j][0] = rdA(0, j); a[j][1] = rdA(1, j); }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 c0 = a[ks % AH][0], c1 = a[ks % AH][1];
        if (!(DEC5_ABL & 8) && ks + AH < KS) { a[ks % AH][0] = rdA(0, ks + AH); a[ks % AH][1] = rdA(1, ks + AH); }
        if (!(DEC5_ABL & 32)) {
          s[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c0, uf[ks], s[0], 0, 0, 0);
          s[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c1, uf[ks], s[1], 0, 0, 0);
        } else {
          s[0][0] += (float)c0[0] * (float)uf[ks][0];
          s[1][0] += (float)c1[0] * (float)uf[ks][0];
        }
        fill(ks);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    float m = 0.f, mL = 0.f, lsum = 0.f;
    f32x4 s_nx[2];
    auto mask_tail = [&](f32x4 (&s)[2], int64_t t) {
      if (t == ntiles - 1 && (N % kTI) != 0) {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          const int lim = (int)(N - t * kTI) - 16 * ih - 4 * gi;
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ih][r] = r >= lim ? -INFINITY : s[ih][r];
        }
      }
    };
    auto p_out = [&](int par) {  // the 8 exponentials of s_nx, their sum, the packed P row pieces -> LDS
      unsigned char* prow = p_row(par, 16 * uh + c16);
#pragma unroll
      for (int ih = 0; ih < 2; ++ih) {
        float pv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[ih][r], kLog2e, -mL));
          lsum += pv[r];
        }
        *reinterpret_cast<uint2*>(prow + 2 * (16 * ih + 8 * (gi & 1) + 4 * (gi >> 1))) =
            make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
      }
    };
#if DEC5_RSTAGE
    uint4 stg[PA > 0 ? PA : 1];
    auto rs_load = [&](int64_t tt, int i) {
      const int p = q * PW + i;
      const uint32_t so = tile_soff(tt) + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (p & 1));
      const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
      stg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, (int)so, 0));
    };
    auto rs_write = [&](int slot_i, int i) {
      *reinterpret_cast<uint4*>(lds + slot_i * TB + q * PW * 1024 + i * 1024 + lane * 16) = stg[i];
    };
#endif
    if (t_beg < t_end) {
      for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg), 0, i, i == 0);
      if (t_beg + 1 < t_end)
        for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
      wait_vmcnt<0>();
#if DEC5_RSTAGE
      if (t_beg + 2 < t_end)
        for (int i = 0; i < PA; ++i) rs_load(t_beg + 2, i);
#endif
    }
    barrier();  // [P0] tiles t_beg (and t_beg + 1) landed (consumers' pieces too)
    if (t_beg < t_end) {
      // first tile: its max sets the user's fixed offset m (version 2's rule)
      gemm1(lds, s_nx, [](int) {});
      mask_tail(s_nx, t_beg);
      float mx = fmaxf(fmaxf(fmaxf(s_nx[0][0], s_nx[0][1]), fmaxf(s_nx[0][2], s_nx[0][3])),
                       fmaxf(fmaxf(s_nx[1][0], s_nx[1][1]), fmaxf(s_nx[1][2], s_nx[1][3])));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      m = fmaxf(mx, bound - kOffsetSpan);
      mL = m * kLog2e;
      p_out(0);  // P(t_beg) -> parity 0
    }
    barrier();  // [P1]
    for (int64_t t = t_beg; t < t_end; ++t) {
      const int li = (int)(t - t_beg);
      const int nxt = (li + 1) % NS, s_dma = (li + 2) % NS, par = li & 1;
#if !DEC5_RSTAGE
      if (!(DEC5_ABL & (1 | 128))) wait_vmcnt<0>();
#endif
      if (!(DEC5_ABL & 2)) barrier();  // [L] tile t + 1 landed, P(t) published, GEMM2(t - 1) done
      if (t + 1 < t_end) {
        const bool dma = !(DEC5_ABL & 1) && (DEC5_BFREE || t + 2 < t_end);
#if DEC5_RSTAGE
        const bool ld3 = t + 3 < t_end;
        gemm1(lds + nxt * TB, s_nx, [&](int ks) {
          if (dma && ks < PA) rs_write(s_dma, ks);  // tile t + 2, loaded one iteration ago
          if (ld3 && ks >= KS - PA) rs_load(t + 3, ks - (KS - PA));
        });
#else
        const uint32_t soff_dma = tile_soff(dma ? t + 2 : t);
        gemm1(lds + nxt * TB, s_nx, [&](int ks) {
#if DEC5_DMA_BURST
          if (dma && ks == DEC5_PDMA_AT)
            for (int i = 0; i < PA; ++i) issue_piece(soff_dma, s_dma, i, i == 0);
#else
          const int kk = ks - DEC5_PDMA_AT;
          if (dma && kk >= 0 && kk % DEC5_DMA_STRIDE == 0 && kk / DEC5_DMA_STRIDE < PA) issue_piece(soff_dma, s_dma, prot(kk / DEC5_DMA_STRIDE, PA), kk == 0);
#endif
        });
#endif
        mask_tail(s_nx, t + 1);
        if (!(DEC5_ABL & 4)) p_out(par ^ 1);
        else lsum += (s_nx[0][0] + s_nx[1][0] > 1e30f) ? 0.f : 1.f;  // keeps GEMM1 live, l >= 1: no user flagged
      }
    }
    wait_vmcnt<0>();
    lsum += __shfl_xor(lsum, 16, 64);  // over the 4 lanes g of the user
    lsum += __shfl_xor(lsum, 32, 64);
    barrier();  // [E0]
    if (g == 0) {
      xm[ug * 64 + 16 * uh + c16] = lsum;
      xm[ug * 64 + 32 + 16 * uh + c16] = m;
    }
    barrier();  // [E1]
    return;
  }

  // -------------------------------------------------------------------- consumer ---
  // GEMM2 (version 3's reads): O^T[DW][32 users] += E^T P^T over k-steps 0 (items 0..15) and 1 (16..31)
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int g1 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  const int cseg = (dbase / 128) << 13;
  auto dboff = [](int db) { return ((db >> 2) << 13) + ((db & 3) << 9); };
  const int laneT0 = ((4 * h + qq) << 6) + (((2 * g1 + (pp >> 1)) ^ ((0 + h) & 3)) << 4) + 8 * (pp & 1);
  const int laneT1 = ((4 * h + qq) << 6) + (((2 * g1 + (pp >> 1)) ^ ((2 + h) & 3)) << 4) + 8 * (pp & 1);
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  constexpr int BH = 2;
  auto rdT = [&](const unsigned char* buf, int i) {
    const int kh = i / DB, db = i % DB;
    const unsigned char* tt = buf + cseg + (kh << 12);
    auto* p0 = (__attribute__((address_space(3))) s16x4*)(void*)(tt + laneT0 + dboff(db));
    auto* p1 = (__attribute__((address_space(3))) s16x4*)(void*)(tt + laneT1 + (1 << 11) + dboff(db));
    return std::array<s16x4, 2>{__builtin_amdgcn_ds_read_tr16_b64_v4i16(p0), __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1)};
  };
  auto gemm2 = [&](const unsigned char* buf, const uint4& pf0, const uint4& pf1, auto&& fill) {
    if constexpr (WITH_O) {
      std::array<s16x4, 2> n[BH];
#pragma unroll
      for (int j = 0; j < BH; ++j) n[j] = rdT(buf, j);
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) {
        const std::array<s16x4, 2> c = n[i % BH];
        if (!(DEC5_ABL & 16) && i + BH < 2 * DB) n[i % BH] = rdT(buf, i + BH);
        const s16x8 a = {c[0][0], c[0][1], c[0][2], c[0][3], c[1][0], c[1][1], c[1][2], c[1][3]};
        if (!(DEC5_ABL & 64))
          o[i % DB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                             __builtin_bit_cast(bf16x8, i < DB ? pf0 : pf1), o[i % DB],
                                                             0, 0, 0);
        else
          o[i % DB][0] += (float)__builtin_bit_cast(bf16x8, a)[0];
        fill(i);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) fill(i);
    }
  };
  if constexpr (PB > 0) {
    if (t_beg < t_end) {
      for (int i = PA; i < PW; ++i) issue_piece(tile_soff(t_beg), 0, i, i == PA);
      if (t_beg + 1 < t_end)
        for (int i = PA; i < PW; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
      wait_vmcnt<0>();
    }
  }
#if DEC5_CRSTAGE
  // DEC5_CRSTAGE=1 (A/B): the consumer's PB pieces of each tile through registers instead of LDS-DMA -- loaded by
  // buffer_load_dwordx4 in GEMM2(t)'s first gaps (tile t + 2; past the split the loads re-read tile t and are not
  // written), written by ds_write_b128 into the same image bytes before the next iteration's barrier
  uint4 cst[PB > 0 ? PB : 1];
  auto c_load = [&](uint32_t soff, int k) {
    const int p = q * PW + PA + k;
    const uint32_t so = soff + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (p & 1));
    const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
    cst[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo, (int)so, 0));
  };
  auto c_write = [&](int slot_i) {
#pragma unroll
    for (int k = 0; k < PB; ++k)
      *reinterpret_cast<uint4*>(lds + slot_i * TB + (q * PW + PA + k) * 1024 + lane * 16) = cst[k];
  };
#endif
  barrier();  // [P0]
  if (DEC5_P32) barrier();  // [PX]
  barrier();  // [P1]
  for (int64_t t = t_beg; t < t_end; ++t) {
    const int li = (int)(t - t_beg);
    const int cur = li % NS, s_dma = (li + 2) % NS, par = li & 1;
    DEC5_T(const unsigned long long tm0 = __builtin_amdgcn_s_memtime();)
    if constexpr (PB > 0) if (!(DEC5_ABL & (1 | 128))) wait_vmcnt<0>();
#if DEC5_CRSTAGE
    if (li >= 1 && t + 1 < t_end) c_write((li + 1) % NS);  // tile t + 1, loaded in the previous iteration
#endif
    DEC5_T(const unsigned long long tm1 = __builtin_amdgcn_s_memtime();)
    if (!(DEC5_ABL & 2)) barrier();  // [L]
    DEC5_T(const unsigned long long tm2 = __builtin_amdgcn_s_memtime();)
    // P(t) in GEMM2's B layout: user col, positions 8 h .. 8 h + 7 of k-steps 0 and 1
    const uint4 pf0 = *reinterpret_cast<const uint4*>(p_row(par, col) + 16 * h);
    const uint4 pf1 = *reinterpret_cast<const uint4*>(p_row(par, col) + 32 + 16 * h);
    // DEC5_BFREE (A/B): issue the pieces of tile t + 2 unconditionally (past the split they fill the free slot)
    const bool dma = !(DEC5_ABL & 1) && (DEC5_BFREE || t + 2 < t_end);
    const uint32_t soff_dma = tile_soff(dma ? t + 2 : t);
#if DEC5_CRSTAGE
    const uint32_t soff_ld = tile_soff(t + 2 < t_end ? t + 2 : t);
#endif
    gemm2(lds + cur * TB, pf0, pf1, [&](int i) {
      const int ii = i - DEC5_CDMA_AT;
#if DEC5_CRSTAGE
      if constexpr (PB > 0)
        if (ii >= 0 && ii < PB) c_load(soff_ld, ii);
#elif DEC5_DMA_BURST
      if constexpr (PB > 0)
        if (dma && ii == 0)
          for (int k = 0; k < PB; ++k) issue_piece(soff_dma, s_dma, PA + k, k == 0);
#else
      if constexpr (PB > 0)
        if (dma && ii >= 0 && ii % DEC5_DMA_STRIDE == 0 && ii / DEC5_DMA_STRIDE < PB) issue_piece(soff_dma, s_dma, PA + prot(ii / DEC5_DMA_STRIDE, PB), ii == 0);
#endif
    });
    DEC5_T(const unsigned long long tm3 = __builtin_amdgcn_s_memtime(); tacc[0] += tm1 - tm0; tacc[1] += tm2 - tm1;
           tacc[2] += tm3 - tm2; ++ntl;)
  }
  if constexpr (PB > 0) wait_vmcnt<0>();
  if (DEC5_P32) barrier();  // [PE0]
  barrier();  // [E0]
  barrier();  // [E1] producers' (l, m) published
  DEC5_T(tm_store();)
  if (!wave_active || t_beg >= t_end || user >= nb) return;
  const float ltot = xm[ug * 64 + col], mu = xm[ug * 64 + 32 + col];
  if (h == 0 && dh == 0) out.flag[out.direct ? user : (int64_t)split * nb + user] = !(ltot >= kMinL);
  const int64_t row = out.direct ? user : (int64_t)split * nb + user;
  if (h == 0 && dh == 0) {
    if (out.direct) out.lse[user] = mu + logf(ltot);
    else { out.m[row] = mu; out.l[row] = ltot; }
  }
  if (WITH_O) {
    const float sc = out.direct ? 1.0f / ltot : 1.0f;
#pragma unroll
    for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(out.O + row * D + dd) =
            make_float4(o[d][4 * g4] * sc, o[d][4 * g4 + 1] * sc, o[d][4 * g4 + 2] * sc, o[d][4 * g4 + 3] * sc);
      }
  }
}


// ===================================================================================== fp8, d = 768 ---
// k_dec5_f8: version 5's producer / consumer structure for the block-scaled fp8 sweep
// (v_mfma_scale_f32_32x32x64_f8f6f4, e4m3 operands; the image, the exponent rules and the fixed offset are
// k_dec_fp8's in hvae_decoder.hip). A tile is 64 items (48 KiB of e4m3 at d = 768); 8 waves, two per SIMD;
// for q = 0..3, (ug, hq) = (q & 1, q >> 1):
//   * producer q (role 0): U of user group ug (32 users) over all of D as e4m3 (96 VGPRs; fp8 halves the
//     bf16 producer's registers per user, so it keeps 32 users and reads only its item half of each tile);
//     per tile: GEMM1 S^T of items 32 hq .. 32 hq + 31 (k-block hq of GEMM2) for its 32 users (12 MFMAs),
//     the half's max, block exponent, 16 exponentials per lane and the packed e4m3 P half + exponent -> LDS;
//   * consumer q + 4 (role 1): O of ug over D half hq (192 VGPRs), GEMM2 of tile t over both item halves
//     (12 MFMAs, K = the tile's 64 items) with both P halves read back, each half's exponent as its k-block's
//     B scale (the MFMA takes k-block b's scale from lane column + 32 b).
// One barrier per tile as in the bf16 version; the first tile's max crosses once between the two producers
// of a user group for their common offset m, and l = l(half 0) + l(half 1) at the end.
namespace f8 {
constexpr int TI = 64;
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr int TB8 = TI * D;                 // tile bytes (48 KiB)
constexpr int PBY = 1024 + 256;            // per producer and parity: P half (64 lanes x 16 B) + exponents
constexpr int LDS_BYTES = NS * TB8 + 2 * 4 * PBY + 4 * 64 * 4 + 2 * 64 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "k_dec5_f8 LDS");
// = hvae_decoder.hip's f8_sw / f8_item_of at D = 768 (D % 256 == 0 form)
__device__ __forceinline__ constexpr int sw(int it) {
  return ((it & 1) << 1) | (((it >> 1) & 1) << 2) | (((it >> 3) & 1) << 3) | ((it >> 2) & 1);
}
__device__ __forceinline__ constexpr int item_of(int h, int j) {
  return 32 * (j >> 4) + (j & 3) + 8 * ((j & 15) >> 2) + 4 * h;
}
__device__ __forceinline__ int pack4(float a, float b, float c, float d) {
  const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);
}
}  // namespace f8

#ifndef DEC5F8_DMA_B
#define DEC5F8_DMA_B 6  // of each (ug, hq)'s 12 LDS-DMA pieces per tile, how many the consumer issues
#endif
#ifndef DEC5F8_G1_AHEAD
#define DEC5F8_G1_AHEAD 2
#endif
#ifndef DEC5F8_PRIO
#define DEC5F8_PRIO 0  // A/B: static s_setprio 1 for 1 the consumers, 2 the producers
#endif
// Timing-ablation builds only (DEC5_ABL's bits for the fp8 sweep; scripts/build_variant5.sh, outputs invalid by
// construction): 1 no LDS-DMA pieces in the loop (and no vmcnt waits), 2 no per-tile barrier, 4 no exponentials /
// P out, 8 GEMM1 A operands not re-read from LDS, 16 GEMM2 operands not re-read, 32 no GEMM1 MFMAs, 64 no GEMM2
// MFMAs, 128 LDS-DMA pieces issued but never waited for (profiles/r04_dec5_f8_ablation.jsonl)
#ifndef DEC5F8_ABL
#define DEC5F8_ABL 0
#endif
// DEC5F8_RSTAGE (A/B): the producer's pieces through registers instead of LDS-DMA -- buffer_load_dwordx4 to VGPRs
// under GEMM1's MFMAs, ds_write_b128 into the free slot after them (same ring, same timing, another mechanism);
// 2: all 12 pieces of the (ug, hq) pair on the producer that way, none on the consumer
#ifndef DEC5F8_RSTAGE
#define DEC5F8_RSTAGE 0
#endif
#ifndef DEC5F8_CRSTAGE
#define DEC5F8_CRSTAGE 0
#endif

template <bool WITH_O>
__global__ void __launch_bounds__(512) k_dec5_f8(const float* __restrict__ U, int64_t ldu,
                                                 const unsigned char* __restrict__ T8, const int* __restrict__ e_exp,
                                                 const float* __restrict__ e_maxnorm, int64_t nb, int64_t N,
                                                 int splits, int64_t tiles_per_split, Out out) {
  using namespace f8;
  constexpr int DW = D / 2;      // GEMM2: dims owned by one consumer
  constexpr int DB = DW / 32;    // GEMM2 d-blocks (12)
  constexpr int KS = D / 64;     // GEMM1 k-steps (12)
  constexpr int PW = 12;         // 1-KiB LDS-DMA pieces per (ug, hq) per tile
  constexpr int PB = DEC5F8_RSTAGE == 2 ? 0 : DEC5F8_DMA_B;
  constexpr int PA = PW - PB;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* pbuf = lds + NS * TB8;                                    // [2 par][4 producers][PBY]
  float* xmax = reinterpret_cast<float*>(lds + NS * TB8 + 2 * 4 * PBY);    // [4 producers][64]
  float* xm = xmax + 4 * 64;                                              // [2 ug][l 32 | m 32]

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int role = w >> 2, q = w & 3;
  const int ug = q & 1, hq = q >> 1;
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * 64 + ug * 32;
  // tile indices in 32 bits (N < 2^31, checked by the host) and wave-uniform in SGPRs
  const int ntiles = __builtin_amdgcn_readfirstlane((int)((N + TI - 1) / TI));
  const int t_beg = __builtin_amdgcn_readfirstlane((int)(split * tiles_per_split));
  const int t_end = __builtin_amdgcn_readfirstlane((int)min((int64_t)ntiles, (int64_t)t_beg + tiles_per_split));
  const int ke = *e_exp;  // scalars before any LDS-DMA is in flight
  const int sa = 127 - ke;

  // LDS-DMA: a plain copy of the tile, piece p = q * 12 + i at byte p * 1 KiB of tile and slot
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(T8), (short)0, ntiles * TB8, 0x00020000);
  const int voff = lane * 16;
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(q * PW * 1024);
  auto issue_piece = [&](uint32_t soff, int slot_i, int i, bool fresh) {
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB8 + i * 1024);
    const uint32_t so = soff + (uint32_t)((q * PW + i) * 1024);
    if (fresh)
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb), "v"(voff), "s"(rsrc), "s"(so) : "memory");
    else
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb), "v"(voff), "s"(rsrc), "s"(so) : "memory");
  };
  auto tile_soff = [&](int t) { return (uint32_t)__builtin_amdgcn_readfirstlane(t * TB8); };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto p_slot = [&](int par, int pq) { return pbuf + (par * 4 + pq) * PBY; };
  if ((DEC5F8_PRIO == 1 && role == 1) || (DEC5F8_PRIO == 2 && role == 0)) __builtin_amdgcn_s_setprio(1);

  if (role == 0) {
    // ------------------------------------------------------------------ producer ---
    const float emax = *e_maxnorm;
    // u over all of D: lane (col, h) holds u[64 ks + 32 h + j], j < 32, as e4m3 of u 2^ku (ku from the row)
    const float* urow = U + min(u0 + col, nb - 1) * ldu + 32 * h;
    float amax = 0.f, usq = 0.f;
#pragma unroll 8
    for (int q4 = 0; q4 < D / 8; ++q4) {
      const float4 a = *reinterpret_cast<const float4*>(urow + 64 * (q4 >> 3) + 4 * (q4 & 7));
      amax = fmaxf(amax, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
      usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
    }
    amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
    usq += __shfl_xor(usq, 32, 64);
    int eu = 0;
    (void)frexpf(amax, &eu);
    const int ku = amax > 0.f ? min(127, 8 - eu) : 0;
    const int sbu = 127 - ku;
    const float qu = ldexpf(1.f, ku);
    // re-read the row for the packing pass: without this the loads of the first pass are kept live (CSE),
    // 384 floats a lane, and spill
    // (each k-step's address depends on the previous k-step's packed words, so the compiler cannot hoist all 96
    // loads of this pass ahead of the packing: 384 floats a lane would spill)
    i32x8 uf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const float* up = urow + 64 * ks;
      if (ks > 0) asm volatile("" : "+v"(up) : "v"(uf[ks - 1]));
#pragma unroll
      for (int q4 = 0; q4 < 8; ++q4) {
        const float4 a = *reinterpret_cast<const float4*>(up + 4 * q4);
        uf[ks][q4] = pack4(a.x * qu, a.y * qu, a.z * qu, a.w * qu);
      }
    }
    const float bound = sqrtf(usq) * emax * 1.02f;
    // GEMM1 A operand (k-step ks): item row 32 hq + col, chunks 4 ks + 2 h + {0, 1}
    const int swc = sw(col);  // sw depends on the low 4 bits of the row only
    const int rowA = (32 * hq + col) * D;
    auto rdA = [&](const unsigned char* buf, int ks) {
      const int ch = 4 * ks + 2 * h;
      const unsigned char* row = buf + rowA;
      const uint4 x = *reinterpret_cast<const uint4*>(row + 16 * (ch ^ swc));
      const uint4 y = *reinterpret_cast<const uint4*>(row + 16 * ((ch + 1) ^ swc));
      i32x8 r;
      r[0] = (int)x.x; r[1] = (int)x.y; r[2] = (int)x.z; r[3] = (int)x.w;
      r[4] = (int)y.x; r[5] = (int)y.y; r[6] = (int)y.z; r[7] = (int)y.w;
      return r;
    };
    auto gemm1 = [&](const unsigned char* buf, f32x16& sv, auto&& fill) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = 0.f;
      constexpr int AH = DEC5F8_G1_AHEAD;
      i32x8 ra[AH];
#pragma unroll
      for (int j = 0; j < AH; ++j) ra[j] = rdA(buf, j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const i32x8 c = ra[ks % AH];
        if (!(DEC5F8_ABL & 8) && ks + AH < KS) ra[ks % AH] = rdA(buf, ks + AH);
        if (!(DEC5F8_ABL & 32)) sv = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c, uf[ks], sv, 0, 0, 0, sa, 0, sbu);
        else sv[0] += (float)(c[0] ^ uf[ks][0]);
        fill(ks);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // own half of tile t: items past N -> -inf; the half's max over its 32 items (every lane of a column)
    auto half_max = [&](int t, f32x16& sv) {
      if (t == ntiles - 1 && (N % TI) != 0) {
        const int lim = (int)(N - (int64_t)t * TI) - 4 * h - 32 * hq;
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : sv[r];
      }
      const float a0 = fmaxf(fmaxf(sv[0], sv[1]), sv[2]), a1 = fmaxf(fmaxf(sv[3], sv[4]), sv[5]);
      const float a2 = fmaxf(fmaxf(sv[6], sv[7]), sv[8]), a3 = fmaxf(fmaxf(sv[9], sv[10]), sv[11]);
      const float a4 = fmaxf(fmaxf(sv[12], sv[13]), fmaxf(sv[14], sv[15]));
      const float mx = fmaxf(fmaxf(fmaxf(a0, a1), a2), fmaxf(a3, a4));
      const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      return fmaxf(__uint_as_float(s2[0]), __uint_as_float(s2[1]));
    };
    float m = 0.f, mL = 0.f, lsum = 0.f;
    auto tile_exp = [&](float mh) { return max(-119, min(127, (int)ceilf(__builtin_fmaf(mh, kLog2e, -mL)) - 8)); };
    // the 16 exponentials of the half, their sum, the packed e4m3 P half and its exponent -> LDS parity par
    auto p_out = [&](const f32x16& sv, float mh, int par) {
      const int e = tile_exp(mh);
      const float cE = mL + (float)e;
      float qsum = 0.f;
      int pk[4];
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        float qv[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (j4 * 2 + (b >> 1) < DEC5_EXPPOLY8) {  // A/B: the pair (b, b + 1) on the packed polynomial
            if ((b & 1) == 0) {
              const f32x2 y = exp2_pk(f32x2{__builtin_fmaf(sv[4 * j4 + b], kLog2e, -cE),
                                            __builtin_fmaf(sv[4 * j4 + b + 1], kLog2e, -cE)});
              qv[b] = y[0];
              qv[b + 1] = y[1];
              qsum += qv[b];
              qsum += qv[b + 1];
            }
            continue;
          }
          qv[b] = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[4 * j4 + b], kLog2e, -cE));
          qsum += qv[b];
        }
        pk[j4] = pack4(qv[0], qv[1], qv[2], qv[3]);
      }
      lsum += ldexpf(qsum, e);
      reinterpret_cast<int4*>(p_slot(par, q))[lane] = make_int4(pk[0], pk[1], pk[2], pk[3]);
      reinterpret_cast<int*>(p_slot(par, q) + 1024)[lane] = e;
    };
    f32x16 s_nx;
#if DEC5F8_RSTAGE
    uint4 stg[PA];
    auto rs_load = [&](uint32_t soff, int i) {
      stg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, (int)(soff + (uint32_t)((q * PW + i) * 1024)), 0));
    };
    auto rs_write = [&](int slot_i) {
#pragma unroll
      for (int i = 0; i < PA; ++i)
        *reinterpret_cast<uint4*>(lds + slot_i * TB8 + (q * PW + i) * 1024 + lane * 16) = stg[i];
    };
#endif
    if (t_beg < t_end) {
      for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg), 0, i, i == 0);
      if (t_beg + 1 < t_end)
        for (int i = 0; i < PA; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
      wait_vmcnt<0>();
    }
    barrier();  // [P0] tiles t_beg (and t_beg + 1) landed (consumers' pieces too)
    float mh = 0.f;
    if (t_beg < t_end) {
      gemm1(lds, s_nx, [](int) {});
      mh = half_max(t_beg, s_nx);
      if (lane < 32) xmax[q * 64 + lane] = mh;
    }
    barrier();  // [PX] the first tile's half maxima of both producers of the user group
    if (t_beg < t_end) {
      m = fmaxf(fmaxf(mh, xmax[(q ^ 2) * 64 + col]), bound - kOffsetSpan);
      mL = m * kLog2e;
      p_out(s_nx, mh, 0);  // P(t_beg) -> parity 0
    }
    barrier();  // [P1]
    for (int t = t_beg; t < t_end; ++t) {
      const int li = t - t_beg;
      const int nxt = (li + 1) % NS, s_dma = (li + 2) % NS, par = li & 1;
      if (!(DEC5F8_ABL & (1 | 128))) wait_vmcnt<0>();
      if (!(DEC5F8_ABL & 2)) barrier();  // [L] tile t + 1 landed, P(t) published, GEMM2(t - 1) done
      if (t + 1 < t_end) {
        // branch-free DMA: past the split the pieces land in the free slot s_dma (tiles past N read as 0)
        const uint32_t soff_dma = tile_soff(t + 2);
#if DEC5F8_RSTAGE
        gemm1(lds + nxt * TB8, s_nx, [&](int ks) {
          if (ks < PA) rs_load(soff_dma, ks);
        });
        rs_write(s_dma);
#else
        gemm1(lds + nxt * TB8, s_nx, [&](int ks) {
          if (!(DEC5F8_ABL & 1) && ks < PA) issue_piece(soff_dma, s_dma, ks, ks == 0);
        });
#endif
        mh = half_max(t + 1, s_nx);
        if (!(DEC5F8_ABL & 4)) p_out(s_nx, mh, par ^ 1);
        else lsum += (s_nx[0] > 1e30f) ? 0.f : 1.f;  // keeps GEMM1 live, l >= 1: no user flagged
      }
    }
    wait_vmcnt<0>();
    const float lw = lsum + __shfl_xor(lsum, 32, 64);  // both lane halves of the column
    barrier();  // [E0]
    if (lane < 32) xmax[q * 64 + lane] = lw;
    barrier();  // [E1]
    if (hq == 0 && lane < 32) {  // l = l(half 0) + l(half 1), in that order; m
      xm[ug * 64 + lane] = lw + xmax[(q ^ 2) * 64 + lane];
      xm[ug * 64 + 32 + lane] = m;
    }
    barrier();  // [E2]
    return;
  }

  // -------------------------------------------------------------------- consumer ---
  const bool wave_active = u0 < nb;
  const int dbase = hq * DW;
  // GEMM2 A operand (d-block db of this wave's D half): four transposed reads c of items item_of(h, 8 c + qq)
  // = it0 + 16 c, which share the chunk swizzle sw(it0); chunk ch = 2 x + g1 (x = dbase / 32 + db) sits at
  // 16 (ch ^ sw) = loff[x & 7] - row part + 256 (x >> 3): eight lane offsets, the rest immediates
  const int g1 = (lane >> 4) & 1, qq = (lane & 15) >> 1, pp = lane & 1;
  const int it0 = item_of(h, qq);
  const int tsw = sw(it0);
  int loff[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) loff[k] = it0 * D + 8 * pp + 16 * ((2 * k + g1) ^ tsw);
  auto rdB = [&](const unsigned char* buf, int db) {
    i32x8 r;
    const int x = dbase / 32 + db;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
          (__attribute__((address_space(3))) i32x2*)(void*)(buf + loff[x & 7] + 256 * (x >> 3) + 16 * D * c));
      r[2 * c] = v[0];
      r[2 * c + 1] = v[1];
    }
    return r;
  };
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  auto gemm2 = [&](const unsigned char* buf, const i32x8& pf, int sbp, auto&& fill) {
    if constexpr (WITH_O) {
      constexpr int AH2 = 2;
      i32x8 a[AH2];
#pragma unroll
      for (int j = 0; j < AH2; ++j) a[j] = rdB(buf, j);
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        const i32x8 c = a[db % AH2];
        if (!(DEC5F8_ABL & 16) && db + AH2 < DB) a[db % AH2] = rdB(buf, db + AH2);
        if (!(DEC5F8_ABL & 64)) o[db] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c, pf, o[db], 0, 0, 0, sa, 0, sbp);
        else o[db][0] += (float)(c[0] ^ pf[0]);
        fill(db);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int db = 0; db < DB; ++db) fill(db);
    }
  };
  if constexpr (PB > 0) {
    if (t_beg < t_end) {
      for (int i = PA; i < PW; ++i) issue_piece(tile_soff(t_beg), 0, i, i == PA);
      if (t_beg + 1 < t_end)
        for (int i = PA; i < PW; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
      wait_vmcnt<0>();
    }
  }
#if DEC5F8_CRSTAGE
  // DEC5F8_CRSTAGE=1 (A/B; bf16: DEC5_CRSTAGE): the consumer's PB pieces through registers -- buffer_load_dwordx4 in
  // GEMM2(t)'s first gaps (tile t + 2), ds_write_b128 into the same image bytes before the next barrier
  uint4 cst[PB > 0 ? PB : 1];
  auto c_load = [&](uint32_t soff, int k) {
    cst[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rsrc, voff, (int)(soff + (uint32_t)((q * PW + PA + k) * 1024)), 0));
  };
  auto c_write = [&](int slot_i) {
#pragma unroll
    for (int k = 0; k < PB; ++k)
      *reinterpret_cast<uint4*>(lds + slot_i * TB8 + (q * PW + PA + k) * 1024 + lane * 16) = cst[k];
  };
#endif
  barrier();  // [P0]
  barrier();  // [PX]
  barrier();  // [P1]
  const int pq0 = ug, pq1 = ug + 2;  // the producers of this user group: item halves 0 and 1
  for (int t = t_beg; t < t_end; ++t) {
    const int li = t - t_beg;
    const int cur = li % NS, s_dma = (li + 2) % NS, par = li & 1;
    if constexpr (PB > 0) if (!(DEC5F8_ABL & (1 | 128))) wait_vmcnt<0>();
#if DEC5F8_CRSTAGE
    if (li >= 1 && t + 1 < t_end) c_write((li + 1) % NS);  // tile t + 1, loaded in the previous iteration
#endif
    if (!(DEC5F8_ABL & 2)) barrier();  // [L]
    // P(t): k-block 0 = item half 0 (elements 0..15), k-block 1 = half 1; lane half h supplies k-block h's scale
    const int4 y0 = reinterpret_cast<const int4*>(p_slot(par, pq0))[lane];
    const int4 y1 = reinterpret_cast<const int4*>(p_slot(par, pq1))[lane];
    const int eh = reinterpret_cast<const int*>(p_slot(par, h ? pq1 : pq0) + 1024)[lane];
    i32x8 pf;
    pf[0] = y0.x; pf[1] = y0.y; pf[2] = y0.z; pf[3] = y0.w;
    pf[4] = y1.x; pf[5] = y1.y; pf[6] = y1.z; pf[7] = y1.w;
    const int sbp = 127 + eh;
    const uint32_t soff_dma = tile_soff(t + 2);  // branch-free, as the producers'
    gemm2(lds + cur * TB8, pf, sbp, [&](int db) {
#if DEC5F8_CRSTAGE
      if constexpr (PB > 0)
        if (db < PB) c_load(soff_dma, db);
#else
      if constexpr (PB > 0)
        if (!(DEC5F8_ABL & 1) && db < PB) issue_piece(soff_dma, s_dma, PA + db, db == 0);
#endif
    });
  }
  if constexpr (PB > 0) wait_vmcnt<0>();
  barrier();  // [E0]
  barrier();  // [E1]
  barrier();  // [E2] producers' (l, m) published
  const int64_t user = u0 + col;
  if (!wave_active || t_beg >= t_end || user >= nb) return;
  const float ltot = xm[ug * 64 + col], mu = xm[ug * 64 + 32 + col];
  const int64_t row = out.direct ? user : (int64_t)split * nb + user;
  if (h == 0 && hq == 0) {
    out.flag[row] = !(ltot >= kMinL);
    if (out.direct) out.lse[user] = mu + logf(ltot);
    else { out.m[row] = mu; out.l[row] = ltot; }
  }
  if (WITH_O) {
    const float sc = out.direct ? 1.0f / ltot : 1.0f;
#pragma unroll
    for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(out.O + row * D + dd) =
            make_float4(o[d][4 * g4] * sc, o[d][4 * g4 + 1] * sc, o[d][4 * g4 + 2] * sc, o[d][4 * g4 + 3] * sc);
      }
  }
}

}  // namespace dec5


// Launch of the fp8 version-5 sweep (d = 768, 64 users per block, 64-item tiles, block b's split = b % splits)
int dec5_f8_launch(bool with_o, const float* U, int64_t ldu, const unsigned char* T8, const int* ke,
                   const float* enorm, int64_t nb, int64_t N, int splits, int64_t tiles_per_split, int64_t blocks,
                   int* flag, float* m, float* l, float* O, float* lse, int direct, hipStream_t st) {
  using namespace dec5;
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5_f8<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 f8::LDS_BYTES));
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5_f8<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 f8::LDS_BYTES));
    attr_set = true;
  }
  Out o{flag, m, l, O, lse, direct};
  if (with_o)
    k_dec5_f8<true><<<(unsigned)blocks, 512, f8::LDS_BYTES, st>>>(U, ldu, T8, ke, enorm, nb, N, splits,
                                                                   tiles_per_split, o);
  else
    k_dec5_f8<false><<<(unsigned)blocks, 512, f8::LDS_BYTES, st>>>(U, ldu, T8, ke, enorm, nb, N, splits,
                                                                    tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec5_f8");
  return HVAE_OK;
}

// Launch of the version-5 sweep (d = 768, 64 users per block, blocks = user blocks x splits, block b's
// split = b % splits): called by hvae_decoder.hip's dispatch with its plan and outputs.
int dec5_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                int splits, int64_t tiles_per_split, int64_t blocks, int* flag, float* m, float* l, float* O,
                float* lse, int direct, hipStream_t st) {
  using namespace dec5;
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5_bf16<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 LDS_BYTES));
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5_bf16<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 LDS_BYTES));
    attr_set = true;
  }
  Out o{flag, m, l, O, lse, direct};
  if (with_o)
    k_dec5_bf16<true><<<(unsigned)blocks, 512, LDS_BYTES, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N, splits,
                                                                tiles_per_split, o);
  else
    k_dec5_bf16<false><<<(unsigned)blocks, 512, LDS_BYTES, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N, splits,
                                                                 tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec5_bf16");
  return HVAE_OK;
}

}  // namespace hvae

#if DEC5_TIMING
extern "C" int hvae_dec5_timing_fetch(unsigned long long* out) {  // [2048 waves][8], timing builds only
  HVAE_HIP(hipDeviceSynchronize());
  HVAE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(hvae::dec5::dec5_tm), sizeof(hvae::dec5::dec5_tm)));
  return HVAE_OK;
}
#endif
