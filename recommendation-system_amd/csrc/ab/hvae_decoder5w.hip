// hvae_decoder5w.hip -- k_dec5w_bf16, version 5's producer / consumer split at d = 384 with 128 users per block:
// measured slower than version 2 at d = 384, so it is compiled only into the A/B library
// (make lib-ab; HVAE_DEC_V5W=1 selects it).
#if !HVAE_AB
#error "hvae_decoder5w.hip is part of the A/B library only (make lib-ab)"
#endif
#include <algorithm>
#include <array>

#include "../hvae_common.h"
#include "../hvae_dec5_shared.h"

namespace hvae {
namespace dec5 {

// ============================================================================ bf16, d = 384, 128 users ---
// k_dec5w_bf16: version 5's producer / consumer split at d = 384 with 128 users per block (Syn-1M, configs[2]).
// At d = 384 a user's U is 48 VGPRs and its O 96, so a block can hold four 32-user groups: producer q (role 0)
// = user group q, U over all of D (96 VGPRs), GEMM1 of tile t + 1 for both item halves (48 16x16x32 MFMAs, two A
// reads per k-step, each serving both 16-user halves), the 16 exponentials of its users and their P rows ->
// LDS; consumer q + 4 (role 1) = O of user group q over all of D (192 VGPRs), GEMM2 of tile t (24 32x32x16
// MFMAs). A 32-item tile is 24 KiB (version 2's image; 24 LDS-DMA pieces, three per wave), so the ring holds
// NS5W = 5 tiles and the pieces of tile t + 4 are issued in iteration t, three iterations before GEMM1 reads
// them: the fill latency that bounds the d = 768 sweep is hidden here, and 128 users per tile halve the E stream
// per flop against 64. One barrier per tile:
//   [barrier: tile t + 1 landed, P(t) published, GEMM2(t - 1) done]
//   all waves: pieces of t + 4 into the slot GEMM2(t - 1) freed (issued unconditionally: past the split they
//   fill that free slot, past N they read 0, so every wave's vmcnt arithmetic is the same each iteration)
//   producers: GEMM1(t + 1) | softmax | P(t + 1) out        consumers: GEMM2(t) from slot t % NS5W and P(t)
#ifndef NS5W
#define NS5W 5
#endif
namespace w384 {
constexpr int D384 = 384;
constexpr int TB384 = (D384 / 128) * 8192;  // 24 KiB
constexpr int PPW = TB384 / 1024 / 8;    // LDS-DMA pieces per wave per tile (3)
constexpr int LDS_BYTES = NS5W * TB384 + 2 * 4 * 32 * PST + 4 * 64 * 4;
static_assert(LDS_BYTES <= 160 * 1024, "k_dec5w_bf16 LDS");
static_assert(NS5W >= 3, "ring depth");
}  // namespace w384

template <bool WITH_O>
__global__ void __launch_bounds__(512) k_dec5w_bf16(const float* __restrict__ U, int64_t ldu,
                                                    const bf16_t* __restrict__ E, const float* __restrict__ e_maxnorm,
                                                    int64_t nb, int64_t N, int splits, int64_t tiles_per_split,
                                                    Out out) {
  using w384::D384;
  using w384::TB384;
  using w384::PPW;
  constexpr int DB = D384 / 32;    // GEMM2 d-blocks (12)
  constexpr int KS = D384 / 32;    // GEMM1 k-steps (12)
  constexpr int AHD = NS5W - 1;  // tiles of DMA ahead of GEMM2
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* pbuf = lds + NS5W * TB384;                                    // [2 parity][4 ug][32 users][PST]
  float* xm = reinterpret_cast<float*>(lds + NS5W * TB384 + 2 * 4 * 32 * PST);  // [4 ug][l 32 | m 32]

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int c16 = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int role = w >> 2, ug = w & 3;
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * 128 + ug * 32;
  // tile indices in 32 bits (N < 2^31, checked by the host) and wave-uniform
  const int ntiles = __builtin_amdgcn_readfirstlane((int)((N + kTI - 1) / kTI));
  const int t_beg = __builtin_amdgcn_readfirstlane((int)(split * tiles_per_split));
  const int t_end = __builtin_amdgcn_readfirstlane((int)min((int64_t)ntiles, (int64_t)t_beg + tiles_per_split));

  // LDS-DMA into version 2's image: wave w issues pieces 3 w .. 3 w + 2 of every tile
  int vlane[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int row = 8 * pb + ((lane >> 2) & 7);
    vlane[pb] = ((lane >> 2) & 7) * (D384 * 2) + 64 * (lane >> 5) + 16 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(E), (short)0, (int)(N * D384 * 2), 0x00020000);
  const uint32_t ring0 = lds_addr(lds);
  auto issue_piece = [&](int t, int slot_i, int i, bool fresh) {
    const int p = w * PPW + i;
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB384 + p * 1024);
    const uint32_t so = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)t * (uint32_t)(kTI * D384 * 2))) +
                        (uint32_t)(8 * ((p >> 1) & 3) * (D384 * 2) + 256 * (p >> 3) + 128 * (p & 1));
    const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
    if (fresh)
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb), "v"(vo), "s"(rsrc), "s"(so) : "memory");
    else
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb), "v"(vo), "s"(rsrc), "s"(so) : "memory");
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto p_row = [&](int par, int uu) { return pbuf + ((par * 4 + ug) * 32 + uu) * PST; };
  // prologue: tiles t_beg .. t_beg + AHD - 1 into slots 0 .. AHD - 1 (issued whatever the split's length, as
  // in the loop), then tiles t_beg and t_beg + 1 landed
  if (t_beg < t_end) {
    for (int j = 0; j < AHD; ++j)
      for (int i = 0; i < PPW; ++i) issue_piece(t_beg + j, j, i, i == 0 && j == 0);
    wait_vmcnt<(AHD - 2) * PPW>();
  }
  barrier();  // [P0]

  if (role == 0) {
    // ------------------------------------------------------------------ producer ---
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
    const int gi = dec5_rowblk(g);  // MFMA rows 4 g .. 4 g + 3 hold items 4 gi .. 4 gi + 3 of each half
    int laneA[2];
#pragma unroll
    for (int ih = 0; ih < 2; ++ih) {
      const int r1 = 16 * ih + 4 * dec5_rowblk(c16 >> 2) + (c16 & 3);
      laneA[ih] = ((r1 >> 3) << 11) + ((r1 & 7) << 6) + ((g ^ ((r1 >> 2) & 3)) << 4);
    }
    // GEMM1 of one tile: S^T[32 items][32 users], s[ih][uh]; its pieces of tile td at k-steps 0, 1, 2
    auto gemm1 = [&](const unsigned char* buf, f32x4 (&s)[2][2], int td, int sd, bool dma) {
#pragma unroll
      for (int ih = 0; ih < 2; ++ih)
#pragma unroll
        for (int uh = 0; uh < 2; ++uh)
#pragma unroll
          for (int r = 0; r < 4; ++r) s[ih][uh][r] = 0.f;
      auto rdA = [&](int ih, int ks) {
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(buf + laneA[ih] + ((ks >> 2) << 13) +
                                                                         ((ks & 3) << 9)));
      };
      bf16x8 a[2][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) { a[j][0] = rdA(0, j); a[j][1] = rdA(1, j); }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 c0 = a[ks & 1][0], c1 = a[ks & 1][1];
        if (ks + 2 < KS) { a[ks & 1][0] = rdA(0, ks + 2); a[ks & 1][1] = rdA(1, ks + 2); }
        s[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c0, uf[0][ks], s[0][0], 0, 0, 0);
        s[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c0, uf[1][ks], s[0][1], 0, 0, 0);
        s[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c1, uf[0][ks], s[1][0], 0, 0, 0);
        s[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c1, uf[1][ks], s[1][1], 0, 0, 0);
        if (dma && ks < PPW) issue_piece(td, sd, ks, ks == 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    float m[2] = {0.f, 0.f}, mL[2] = {0.f, 0.f}, lsum[2] = {0.f, 0.f};
    f32x4 s_nx[2][2];
    auto mask_tail = [&](int t) {
      if (t == ntiles - 1 && (N % kTI) != 0) {
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          const int lim = (int)(N - (int64_t)t * kTI) - 16 * ih - 4 * gi;
#pragma unroll
          for (int uh = 0; uh < 2; ++uh)
#pragma unroll
            for (int r = 0; r < 4; ++r) s_nx[ih][uh][r] = r >= lim ? -INFINITY : s_nx[ih][uh][r];
        }
      }
    };
    auto p_out = [&](int par) {  // 16 exponentials (4 items x 2 halves x 2 users), sums, packed P pieces -> LDS
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        unsigned char* prow = p_row(par, 16 * uh + c16);
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          float pv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[ih][uh][r], kLog2e, -mL[uh]));
            lsum[uh] += pv[r];
          }
          *reinterpret_cast<uint2*>(prow + 2 * (16 * ih + 8 * (gi & 1) + 4 * (gi >> 1))) =
              make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
        }
      }
    };
    if (t_beg < t_end) {
      // first tile: its max sets each user's fixed offset m (version 2's rule)
      gemm1(lds, s_nx, 0, 0, false);
      mask_tail(t_beg);
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        float mx = fmaxf(fmaxf(fmaxf(s_nx[0][uh][0], s_nx[0][uh][1]), fmaxf(s_nx[0][uh][2], s_nx[0][uh][3])),
                         fmaxf(fmaxf(s_nx[1][uh][0], s_nx[1][uh][1]), fmaxf(s_nx[1][uh][2], s_nx[1][uh][3])));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        m[uh] = fmaxf(mx, bound[uh] - kOffsetSpan);
        mL[uh] = m[uh] * kLog2e;
      }
      p_out(0);  // P(t_beg) -> parity 0
    }
    barrier();  // [P1]
    for (int t = t_beg; t < t_end; ++t) {
      const int li = t - t_beg;
      wait_vmcnt<(AHD - 2) * PPW>();  // this wave's pieces of tile t + 1 landed
      barrier();  // [L] tile t + 1 landed, P(t) published, GEMM2(t - 1) done
      if (t + 1 < t_end) {
        gemm1(lds + ((li + 1) % NS5W) * TB384, s_nx, t + AHD, (li + AHD) % NS5W, true);
        mask_tail(t + 1);
        p_out((li & 1) ^ 1);
      } else {
        for (int i = 0; i < PPW; ++i) issue_piece(t + AHD, (li + AHD) % NS5W, i, i == 0);
      }
    }
    wait_vmcnt<0>();
#pragma unroll
    for (int uh = 0; uh < 2; ++uh) {
      lsum[uh] += __shfl_xor(lsum[uh], 16, 64);  // over the 4 lanes g of the user
      lsum[uh] += __shfl_xor(lsum[uh], 32, 64);
    }
    barrier();  // [E0]
    if (g == 0) {
#pragma unroll
      for (int uh = 0; uh < 2; ++uh) {
        xm[ug * 64 + 16 * uh + c16] = lsum[uh];
        xm[ug * 64 + 32 + 16 * uh + c16] = m[uh];
      }
    }
    barrier();  // [E1]
    return;
  }

  // -------------------------------------------------------------------- consumer ---
  // GEMM2 (version 3's reads): O^T[D384][32 users] += E^T P^T over k-steps 0 (items 0..15) and 1 (16..31)
  const int g1 = (lane >> 4) & 1, qq = (lane >> 2) & 3, pp = lane & 3;
  auto dboff = [](int db) { return ((db >> 2) << 13) + ((db & 3) << 9); };
  const int laneT0 = ((4 * h + qq) << 6) + (((2 * g1 + (pp >> 1)) ^ ((0 + h) & 3)) << 4) + 8 * (pp & 1);
  const int laneT1 = ((4 * h + qq) << 6) + (((2 * g1 + (pp >> 1)) ^ ((2 + h) & 3)) << 4) + 8 * (pp & 1);
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  auto rdT = [&](const unsigned char* buf, int i) {
    const int kh = i / DB, db = i % DB;
    const unsigned char* tt = buf + (kh << 12);
    auto* p0 = (__attribute__((address_space(3))) s16x4*)(void*)(tt + laneT0 + dboff(db));
    auto* p1 = (__attribute__((address_space(3))) s16x4*)(void*)(tt + laneT1 + (1 << 11) + dboff(db));
    return std::array<s16x4, 2>{__builtin_amdgcn_ds_read_tr16_b64_v4i16(p0), __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1)};
  };
  barrier();  // [P1]
  for (int t = t_beg; t < t_end; ++t) {
    const int li = t - t_beg;
    wait_vmcnt<(AHD - 2) * PPW>();
    barrier();  // [L]
    // P(t) in GEMM2's B layout: user col, positions 8 h .. 8 h + 7 of k-steps 0 and 1
    const uint4 pf0 = *reinterpret_cast<const uint4*>(p_row(li & 1, col) + 16 * h);
    const uint4 pf1 = *reinterpret_cast<const uint4*>(p_row(li & 1, col) + 32 + 16 * h);
    const unsigned char* buf = lds + (li % NS5W) * TB384;
    const int td = t + AHD, sd = (li + AHD) % NS5W;
    if constexpr (WITH_O) {
      constexpr int BH = 2;
      std::array<s16x4, 2> n[BH];
#pragma unroll
      for (int j = 0; j < BH; ++j) n[j] = rdT(buf, j);
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) {
        const std::array<s16x4, 2> c = n[i % BH];
        if (i + BH < 2 * DB) n[i % BH] = rdT(buf, i + BH);
        const s16x8 a = {c[0][0], c[0][1], c[0][2], c[0][3], c[1][0], c[1][1], c[1][2], c[1][3]};
        o[i % DB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                           __builtin_bit_cast(bf16x8, i < DB ? pf0 : pf1), o[i % DB],
                                                           0, 0, 0);
        if (i < PPW) issue_piece(td, sd, i, i == 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      for (int i = 0; i < PPW; ++i) issue_piece(td, sd, i, i == 0);
    }
  }
  wait_vmcnt<0>();
  barrier();  // [E0]
  barrier();  // [E1] producers' (l, m) published
  const int64_t user = u0 + col;
  if (u0 >= nb || t_beg >= t_end || user >= nb) return;
  const float ltot = xm[ug * 64 + col], mu = xm[ug * 64 + 32 + col];
  const int64_t row = out.direct ? user : (int64_t)split * nb + user;
  if (h == 0) {
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
        const int dd = 32 * d + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(out.O + row * D384 + dd) =
            make_float4(o[d][4 * g4] * sc, o[d][4 * g4 + 1] * sc, o[d][4 * g4 + 2] * sc, o[d][4 * g4 + 3] * sc);
      }
  }
}

}  // namespace dec5

// Launch of the d = 384 version-5 sweep with 128 users per block (block b's split = b % splits)
int dec5w_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                 int splits, int64_t tiles_per_split, int64_t blocks, int* flag, float* m, float* l, float* O,
                 float* lse, int direct, hipStream_t st) {
  using namespace dec5;
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5w_bf16<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 w384::LDS_BYTES));
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec5w_bf16<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 w384::LDS_BYTES));
    attr_set = true;
  }
  Out o{flag, m, l, O, lse, direct};
  if (with_o)
    k_dec5w_bf16<true><<<(unsigned)blocks, 512, w384::LDS_BYTES, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N, splits,
                                                                       tiles_per_split, o);
  else
    k_dec5w_bf16<false><<<(unsigned)blocks, 512, w384::LDS_BYTES, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N,
                                                                        splits, tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec5w_bf16");
  return HVAE_OK;
}

}  // namespace hvae
