// hvae_decoder.hip -- the frozen-embedding decoder fused with the multinomial
// loss and its backward (K7, K8, K10 of SURVEY §2.1).
//
// Reference: HybridVAE.decode (src/ml/model.py:181-200) computes the full
// [B, N] scores u E^T; vae_loss_function (src/ml/model.py:281) takes
// log_softmax over items; autograd then forms d(u) = dS E. Because E is a
// frozen buffer (model.py:72-73) only d(u) is needed, and
//   d(u_b) = (1/B) (n_b * sum_i softmax(s_b)_i E_i - sum_{i in row b} x_bi E_i)
// so the dense part is exactly the output of an attention forward with
// Q = U, K = V = E. One streaming pass over E produces lse_b and
// O_b = softmax(s_b) E: 4 * B * N * D FLOPs, scores never leave registers.
//
// Layout / schedule (bf16 kernel, D <= 384):
//   * 4 waves x 32 users per workgroup; U fragments of the wave's 32 users
//     stay in VGPRs for the whole sweep; the O accumulator (D x 32 fp32)
//     too (192 VGPRs at D = 384) -> one wave per SIMD;
//   * items stream through LDS in tiles of 32 rows, double buffered,
//     register-staged; the LDS image is cut into 128-column segments of
//     [32 rows][256 B] with the chunk XOR swizzle (row&3)<<2 | (row>>2)&3,
//     which makes both the row reads of GEMM1 (ds_read_b128) and the
//     transposed reads of GEMM2 (ds_read_b64_tr_b16) bank-conflict free;
//   * "swapped" GEMM1 S^T = E_tile U^T puts one user per lane column, so the
//     per-user max/sum are in-lane + one lane^32 exchange, and the S^T
//     accumulator is directly the B operand of GEMM2 O^T += E_tile^T P^T
//     (k order permuted to the accumulator's row order);
//   * online softmax with a deferred rescale (only when a user's max grows
//     by more than kThr);
//   * the item axis is split over workgroups (flash-decoding); splits are a
//     multiple of 8 so all user blocks of one split share an XCD (blocks b
//     and b+8 share one), keeping the split's E slice L2-resident; a merge
//     kernel combines the (m, l, O) partials.
#include <algorithm>
#include <array>
#include <type_traits>

#include "hvae_common.h"
#include "hvae_dec_shared.h"

namespace hvae {



// ------------------------------------------------------- bf16, version 2 ---
// One row-major E image per tile (no transposed copy): GEMM1 reads its rows with
// ds_read_b128, GEMM2 reads its columns with ds_read_b64_tr_b16 (T10). E tiles
// arrive by LDS-DMA issued from inline asm (buffer_load_dwordx4 ... lds): the
// compiler does not see those writes, so it neither drains them before the
// transposed reads nor recomputes their addresses -- each lane's source offsets
// are fixed for the kernel, the tile base is a scalar soffset, and rows past N
// read 0 through the buffer's bounds check.
//
// Software pipeline, one barrier per tile: the softmax of tile t (VALU) is
// interleaved with GEMM1 of tile t+1 (MFMA), then GEMM2 of tile t.
//
// DS = 1: 4 waves x 32 users, each over all D (D <= 384: U 96 + O 192 VGPRs).
// DS = 2: waves (ug, dh) = (w & 1, w >> 1): 2 user groups x 2 halves of D, each
// wave's GEMM1 sums over its half and the two halves' partial S^T tiles are added
// through LDS (double-buffered by tile parity); both waves of a user group run the
// softmax, each accumulates O for its half of D. Serves D = 768 (U 96 + O 192 per
// wave) and small batches (64 users per block keeps all 4 waves busy).

template <int D, int DS, int NW, bool WITH_O>
__global__ void __launch_bounds__(64 * NW) k_dec2_bf16(const float* __restrict__ U, int64_t ldu,
                                                   const bf16_t* __restrict__ E, const float* __restrict__ e_maxnorm,
                                                   int64_t nb, int64_t N, int splits, int64_t tiles_per_split,
                                                   DecOut out) {
  constexpr int DW = D / DS;            // dims owned by one wave
  constexpr int KS = DW / 16;           // GEMM1 k-steps
  constexpr int DB = DW / 32;           // GEMM2 d-blocks
  constexpr int CH = D / 8;             // 16-B chunks per E row
  constexpr int NSEG = (D + 127) / 128;
  constexpr int TB = d2_tile_bytes<D, DS>();
  constexpr int PW = NSEG * 8 / NW;     // 1-KiB LDS-DMA pieces per wave per tile
  constexpr int NS = d2_stages<D, DS, NW>();
  constexpr int UPB = 32 * NW / DS;
  constexpr int HALF = NW / 2;          // DS = 2: partner wave = w ^ HALF
  constexpr bool kSpread = DS == 2 && NS >= 3;  // LDS-DMA pieces issued between GEMM1's MFMA pairs
  static_assert(NW == 4 || (NW == 8 && DS == 2), "8-wave blocks split D");
  static_assert(DW % 32 == 0 && KS % 2 == 0, "D / DS must be a multiple of 32");
  static_assert(NS >= 2, "LDS ring too small");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  constexpr int XB = d2_xbufs<D>();
  float* xbuf = reinterpret_cast<float*>(lds + NS * TB);                        // [XB][NW w][4 r4][64 lane][4]

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ug = DS == 1 ? w : (w % HALF), dh = DS == 1 ? 0 : (w / HALF);
  const int split = blockIdx.x % splits;
  const int64_t ub = blockIdx.x / splits;
  const int64_t u0 = ub * UPB + ug * 32;
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kBfTI - 1) / kBfTI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const int dbase = dh * DW;
  const float emax = *e_maxnorm;  // before any LDS-DMA is in flight (the compiler's wait would drain them)

  // U fragments (B operand of GEMM1): lane holds U[user][dbase + 16 ks + 8 h + j]
  uint4 uf[KS];
  float usq = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (user < nb) {
      a = *reinterpret_cast<const float4*>(U + user * ldu + dbase + 16 * ks + 8 * h);
      b = *reinterpret_cast<const float4*>(U + user * ldu + dbase + 16 * ks + 8 * h + 4);
    }
    usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
    uf[ks] = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y),
                        pack_bf16x2(b.z, b.w));
  }
  if constexpr (DS == 2) {  // |u| over the partner's half too (the score bound needs the whole row)
    const int obase = (1 - dh) * DW;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (user < nb) {
        const float4 a = *reinterpret_cast<const float4*>(U + user * ldu + obase + 16 * ks + 8 * h);
        const float4 b = *reinterpret_cast<const float4*>(U + user * ldu + obase + 16 * ks + 8 * h + 4);
        usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
      }
    }
  }
  usq += __shfl_xor(usq, 32, 64);

  // LDS-DMA source offsets of this lane's pieces (tile-relative) and the buffer
  // resource over bf16 E [N][D] (bounds = N D 2 bytes: tail rows read 0)
  int voff[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int o_b = (w * PW + i) * 1024 + lane * 16;  // inverse of d2_off
    const int seg = o_b >> 13, rem = o_b & 8191;
    const int row = ((rem >> 11) << 3) + ((rem >> 6) & 7);
    const int ch = (((rem >> 9) & 3) << 2) + (((rem >> 4) & 3) ^ ((row >> 2) & 3));
    const int gc = seg * 16 + ch;
    voff[i] = row * (D * 2) + (gc < CH ? gc : 0) * 16;
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(E), (short)0, (int)(N * D * 2), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(w * PW * 1024);
  // pieces [i0, i1) of this wave's share of tile t into ring slot slot_i
  auto issue_range = [&](int64_t t, int slot_i, int i0, int i1) {
    const uint32_t soff = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)(kBfTI * D * 2)));
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
#pragma unroll
    for (int i = i0; i < i1; ++i)
      if (i == i0)  // soff may be fresh from v_readfirstlane: 5 wait states before a buffer op reads it
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff[i]), "s"(rsrc), "s"(soff) : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff[i]), "s"(rsrc), "s"(soff) : "memory");
  };
  auto issue = [&](int64_t t, int slot_i) { issue_range(t, slot_i, 0, PW); };
  auto lds_fence = [] { asm volatile("" ::: "memory"); };

  // GEMM2 operand addressing (T10): group g16 = lane >> 4 reads 4 item rows x 16 d columns;
  // lane 4q + p of the group addresses row q, columns 4p..4p+3
  const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  // lane parts of d2_off for the GEMM1 row reads (by ks parity) and the transposed reads (by j)
  const int c4 = dbase / 32;  // chunk group of this wave's first column (dbase / 8 / 4)
  const int laneA0 = ((col >> 3) << 11) + ((col & 7) << 6) + (((0 + h) ^ ((col >> 2) & 3)) << 4);
  const int laneA1 = ((col >> 3) << 11) + ((col & 7) << 6) + (((2 + h) ^ ((col >> 2) & 3)) << 4);
  const int laneT0 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((0 + h) & 3)) << 4) + 8 * (pp & 1);
  const int laneT1 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((2 + h) & 3)) << 4) + 8 * (pp & 1);

  // GEMM1 partial over this wave's dims: S^T[32 items][32 users] = E_tile U^T. A operands are read
  // two k-groups ahead; fill(g) places other work (the previous tile's softmax) after the g-th MFMA
  // pair, in the shadow of the MFMA pipe (sched_barrier pins the interleave).
  auto gemm1 = [&](const unsigned char* buf, auto&& fill) {
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    // d2_off(col, c0 + 2 ks + h) = laneA[ks & 1] + (wave-uniform chunk-group term) + immediate
    const unsigned char* b0 = buf + laneA0;
    const unsigned char* b1 = buf + laneA1;
    auto rdA = [&](int ks) {
      const int grp = c4 + (ks >> 1);
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(((ks & 1) ? b1 : b0) + ((grp >> 2) << 13) +
                                                                         ((grp & 3) << 9)));
    };
    constexpr int AH = DEC2_G1_AHEAD;  // k-groups of A operands in flight
    bf16x8 a[2 * AH];
#pragma unroll
    for (int j = 0; j < 2 * AH; ++j)
      if (j < KS) a[j] = rdA(j);
#pragma unroll
    for (int g = 0; g < KS / 2; ++g) {
      const bf16x8 c0 = a[(2 * g) % (2 * AH)], c1 = a[(2 * g + 1) % (2 * AH)];
      if (2 * g + 2 * AH < KS) {
        a[(2 * g) % (2 * AH)] = rdA(2 * g + 2 * AH);
        a[(2 * g + 1) % (2 * AH)] = rdA(2 * g + 2 * AH + 1);
      }
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, __builtin_bit_cast(bf16x8, uf[2 * g]), s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, __builtin_bit_cast(bf16x8, uf[2 * g + 1]), s, 0, 0, 0);
      fill(g);
      __builtin_amdgcn_sched_barrier(0);
    }
    return s;
  };
  // DS = 2: this wave's partial S^T of a tile <-> its partner's, [r4][lane] float4 rows
  auto xput = [&](int par, const f32x16& s) {
    float* xb = xbuf + (((par % XB) * NW + w) * 4) * 256;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4)
      *reinterpret_cast<float4*>(xb + r4 * 256 + lane * 4) = make_float4(s[4 * r4], s[4 * r4 + 1], s[4 * r4 + 2],
                                                                         s[4 * r4 + 3]);
  };
  auto xadd = [&](int par, f32x16& s) {
    const float* xb = xbuf + (((par % XB) * NW + (w ^ HALF)) * 4) * 256;
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4) {
      const float4 v = *reinterpret_cast<const float4*>(xb + r4 * 256 + lane * 4);
      s[4 * r4] += v.x; s[4 * r4 + 1] += v.y; s[4 * r4 + 2] += v.z; s[4 * r4 + 3] += v.w;
    }
  };

  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m = 0.f, mL = 0.f, lsum = 0.f;
  f32x16 s_cur;
#pragma unroll
  for (int r = 0; r < 16; ++r) s_cur[r] = 0.f;

  int cur = 0;
  // GEMM2: O^T[DW][32 users] += E_tile^T P^T; A operands by transposed reads, two d-blocks ahead
  auto gemm2 = [&](const bf16x8 (&pf)[2]) {
    if constexpr (WITH_O) {
      const unsigned char* buf = lds + cur * TB;
      // d2_off(16 s2 + 8 j + 4 h + q, c0 + 4 db + 2 g1 + pp / 2) + 8 (pp & 1) = laneT[j] + uniform + immediate
      const unsigned char* t0 = buf + laneT0;
      const unsigned char* t1 = buf + laneT1;
      auto rdT = [&](int db, int row) {  // row = 16 s2 + 8 j + (4 h + q): pass 16 s2 + 8 j
        const int j = (row >> 3) & 1, grp = c4 + db;
        auto* p = (__attribute__((address_space(3))) s16x4*)(void*)((j ? t1 : t0) + ((row >> 3) << 11) +
                                                                     ((grp >> 2) << 13) + ((grp & 3) << 9));
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16(p);
      };
      constexpr int BH = DEC2_G2_AHEAD;  // d-blocks of A operands in flight
      s16x4 n[BH][4];
#pragma unroll
      for (int j = 0; j < BH; ++j)
        if (j < DB) {
          n[j][0] = rdT(j, 0); n[j][1] = rdT(j, 8);
          n[j][2] = rdT(j, 16); n[j][3] = rdT(j, 24);
        }
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        const int jb = db % BH;
        const s16x4 c00 = n[jb][0], c01 = n[jb][1], c10 = n[jb][2], c11 = n[jb][3];
        if (db + BH < DB) {
          n[jb][0] = rdT(db + BH, 0); n[jb][1] = rdT(db + BH, 8);
          n[jb][2] = rdT(db + BH, 16); n[jb][3] = rdT(db + BH, 24);
        }
        const s16x8 a0 = {c00[0], c00[1], c00[2], c00[3], c01[0], c01[1], c01[2], c01[3]};
        const s16x8 a1 = {c10[0], c10[1], c10[2], c10[3], c11[0], c11[1], c11[2], c11[3]};
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a0), pf[0], o[db], 0, 0, 0);
        o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a1), pf[1], o[db], 0, 0, 0);
      }
    }
  };

  constexpr int PRE = NS == 2 ? 2 : NS - 1;  // tiles in flight before the loop
  if (t_beg < t_end) {
#pragma unroll
    for (int i = 0; i < PRE; ++i) issue(min(t_beg + i, t_end - 1), i);
    wait_vmcnt<(PRE - 1) * PW>();
  }
  lds_fence();
  __builtin_amdgcn_s_barrier();
  lds_fence();
  float bound = 0.f;
  if (t_beg < t_end && wave_active) {
    s_cur = gemm1(lds, [](int) {});
    if (DS == 2 && DEC2_ABL != 4) xput((int)(t_beg & 1), s_cur);
  }
  bound = sqrtf(usq) * emax * 1.02f;

  for (int64_t t = t_beg; t < t_end; ++t) {
    const bool more = t + 1 < t_end;
    if (DEC2_ABL == 1 || DEC2_ABL == 2) {
    } else if (NS >= 3) wait_vmcnt<(NS >= 3 ? NS - 3 : 0) * PW>();
    else wait_vmcnt<0>();
    lds_fence();
    __builtin_amdgcn_s_barrier();
    lds_fence();
    const int nxt = cur == NS - 1 ? 0 : cur + 1;
    // NS >= 3: tile t + NS - 1 goes into the slot every wave finished with (GEMM2(t - 1), before the
    // barrier above). DS = 2 spreads its LDS-DMA pieces over GEMM1(t + 1)'s MFMA pairs (below), where
    // their issue cost hides behind the MFMA pipe (d = 768: 2.82 -> 2.71 ms); DS = 1 issues them in one
    // burst here (spread over GEMM1's row reads they cost more, 586 -> 611 us at Syn-1M; over GEMM2's
    // transposed reads, 580 -> 610 us; after GEMM2's issue, 589 -> 597 us).
    const int64_t t_dma = min(t + NS - 1, t_end - 1);
    const int s_dma = cur == 0 ? NS - 1 : cur - 1;
    if (DEC2_ABL != 1 && NS >= 3 && (!kSpread || !wave_active)) issue(t_dma, s_dma);  // idle waves load too
    if constexpr (DS == 2 && XB == 1 && DEC2_ABL != 4) {  // single exchange buffer: everyone has read S(t) before S(t+1) lands
      if (wave_active) xadd((int)(t & 1), s_cur);
      lds_fence();
      __builtin_amdgcn_s_barrier();
      lds_fence();
    }
    if (wave_active) {
      if (DS == 2 && XB == 2 && DEC2_ABL != 4) xadd((int)(t & 1), s_cur);
      if (t == ntiles - 1 && (N % kBfTI) != 0) {  // rows past N (read as 0) leave the softmax
        const int lim = (int)(N - t * kBfTI) - 4 * h;  // rows of this lane's half at or past it are tail
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s_cur[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : s_cur[r];
      }
      if (t == t_beg) {
        // Fixed per-user offset, set once per split: m >= bound - kOffsetSpan keeps every
        // p = exp(s - m) <= e^60 (no rescale of O ever); m >= first-tile max keeps the
        // large terms normal. A split whose sum ends below e^-60 is flagged for exact
        // recompute (its max term may have lost precision).
        float mx = s_cur[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s_cur[r]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        m = fmaxf(mx, bound - kOffsetSpan);
        mL = m * kLog2e;
      }
      // softmax of tile t (rows spread over GEMM1(t+1)'s MFMA pairs)
      float pv[16];
      uint32_t pk[8];
      auto smax_rows = [&](int r0, int r1) {
#pragma unroll
        for (int r = r0; r < r1; ++r) {
          pv[r] = DEC2_ABL == 3 ? __builtin_fmaf(s_cur[r], kLog2e, -mL)
                                : __builtin_amdgcn_exp2f(__builtin_fmaf(s_cur[r], kLog2e, -mL));
          lsum += pv[r];
          if (r & 1) pk[r >> 1] = pack_bf16x2(pv[r - 1], pv[r]);
        }
      };
      // One code path for every tile: the last tile of a split also runs a GEMM1 (over a stale ring slot,
      // result unused), so that the softmax stays spread over the MFMA pairs instead of being hoisted
      // (with its 16 live exponent arguments) into a block shared with a separate last-tile path.
      constexpr int NG = KS / 2;
      f32x16 s_nx = gemm1(lds + nxt * TB, [&](int g) {
        smax_rows(16 * g / NG, 16 * (g + 1) / NG);
        if (DEC2_ABL != 1 && kSpread && PW * g / NG < PW * (g + 1) / NG)
          issue_range(t_dma, s_dma, PW * g / NG, PW * (g + 1) / NG);
      });
      if (DS == 2 && more && DEC2_ABL != 4) xput((int)((t + 1) & 1), s_nx);
      bf16x8 pf[2];
      pf[0] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
      pf[1] = __builtin_bit_cast(bf16x8, make_uint4(pk[4], pk[5], pk[6], pk[7]));
      gemm2(pf);
      s_cur = s_nx;
    }
    if (NS == 2) {  // the slot of tile t is free once every wave is past GEMM2(t)
      lds_fence();
      __builtin_amdgcn_s_barrier();
      lds_fence();
      if (t + 2 < t_end) issue(t + 2, cur);
    }
    cur = nxt;
  }
  if (DEC2_ABL == 2) wait_vmcnt<0>();

  if (!wave_active) return;
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  if (user >= nb) return;
  if (h == 0 && dh == 0) {
    const int f = !(ltot >= kMinL);
    out.flag[out.direct ? user : (int64_t)split * nb + user] = f;
  }
  if (out.direct) {
    const float inv = 1.0f / ltot;
    if (h == 0 && dh == 0) out.lse[user] = m + logf(ltot);
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + user * D + dd) =
              make_float4(o[d][4 * g4] * inv, o[d][4 * g4 + 1] * inv, o[d][4 * g4 + 2] * inv, o[d][4 * g4 + 3] * inv);
        }
    }
  } else {
    const int64_t pi = (int64_t)split * nb + user;
    if (h == 0 && dh == 0) { out.m[pi] = m; out.l[pi] = ltot; }
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + pi * D + dd) =
              make_float4(o[d][4 * g4], o[d][4 * g4 + 1], o[d][4 * g4 + 2], o[d][4 * g4 + 3]);
        }
    }
  }
}


// ------------------------------------------------------------------- fp8 ---
// The same sweep on the block-scaled fp8 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, OCP e4m3 operands,
// twice the bf16 rate; BASELINE configs[4]). Both products carry exact power-of-two scales:
//   GEMM1 S^T = E_tile U^T: E8 = E 2^ke (one exponent for the whole matrix, from max|E|), u8 = u 2^ku
//     (one exponent per user, from max|u_b|); the MFMA's scale operands undo both, so S^T is fp32 scores
//     of the quantised operands.
//   GEMM2 O^T += E_tile^T P^T: P is block floating point, q = p 2^-e with one exponent e per user and
//     64-item tile (max q in (128, 256]), passed as that user's B scale; p itself never needs a range.
// Scale semantics (scripts/probe_fp8_mfma.hip on MI355X): element j of lane half h belongs to k-block
// j >> 4, whose scale lane (row | column) + 32 (j >> 4) supplies; the decoder gives both lanes of a row or
// column the same exponent, so it depends only on A and B sharing the (h, j) -> k slot map.
// One row-major e4m3 image per 64-item tile (GEMM2's K), 16-B chunks XOR-swizzled by item (f8_sw): GEMM1
// reads its A operand by rows (ds_read_b128), GEMM2 by columns with ds_read_b64_tr_b8 (lane 2q + p of a
// 16-lane group addresses row q, bytes 8p..8p+7; lane i receives column i, row q in byte q:
// scripts/probe_tr8.hip). Both kinds of read are bank-conflict free for D = 128, 256, 384, 768. The
// LDS-DMA is a plain copy of the tile.
// DS = 1 (D <= 384): 4 waves x 32 users, each over all D (U 48 + O 192 registers); the softmax of tile t
// is spread over GEMM1(t+1)'s MFMAs, as in k_dec2_bf16. DS = 2 (D = 768): waves (ug, dh) = (w & 1, w >> 1)
// split D in halves; partial S^T tiles are added through LDS; two 48-KiB tile slots, the next tile's
// LDS-DMA overlapping the whole current tile (GEMM1, exchange, softmax, GEMM2 in sequence).

template <int D, int DS, bool WITH_O>
__global__ void __launch_bounds__(256) k_dec_fp8(const float* __restrict__ U, int64_t ldu,
                                                 const unsigned char* __restrict__ T8, const int* __restrict__ e_exp,
                                                 const float* __restrict__ e_maxnorm, int64_t nb, int64_t N,
                                                 int splits, int64_t tiles_per_split, DecOut out) {
  constexpr int DW = D / DS;             // dims owned by one wave
  constexpr int KS = DW / 64;            // GEMM1 k-steps
  constexpr int DB = DW / 32;            // GEMM2 d-blocks
  constexpr int TB = f8_tile_bytes<D>();
  constexpr int PW = TB / 4096;          // 1-KiB LDS-DMA pieces per wave per tile
  constexpr int NS = f8_stages<D>();
  constexpr int UPB = 128 / DS;          // users per block
  static_assert(D % 64 == 0 && (DS == 1 ? (D <= 384 && NS >= 3) : (D == 768 && NS == (F8_DS2_RING ? 3 : 2))),
                "fp8 decoder shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ug = DS == 1 ? w : (w & 1), dh = DS == 1 ? 0 : (w >> 1);
  const int dbase = dh * DW;
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * UPB + ug * 32;
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kF8TI - 1) / kF8TI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const float emax = *e_maxnorm;  // scalars before any LDS-DMA is in flight
  const int ke = *e_exp;
  const int sa = 127 - ke;        // A scale (E8 = E 2^ke)

  // U: lane (col, h) holds u[dbase + 64 ks + 32 h + j], j < 32, as e4m3 of u 2^ku (ku from the whole row).
  // Lanes past nb read the last user's row (no per-load branches); their columns are never stored.
  const float* urow = U + min(user, nb - 1) * ldu + 32 * h;
  float amax = 0.f, usq = 0.f;
#pragma unroll 8
  for (int q4 = 0; q4 < D / 8; ++q4) {  // this lane half's 32-column groups of the whole row
    const float4 a = *reinterpret_cast<const float4*>(urow + 64 * (q4 >> 3) + 4 * (q4 & 7));
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(a.x), fabsf(a.y)), fmaxf(fabsf(a.z), fabsf(a.w))));
    usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
  }
  amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
  usq += __shfl_xor(usq, 32, 64);
  int eu = 0;
  (void)frexpf(amax, &eu);                               // amax = m 2^eu, m in [0.5, 1)
  const int ku = amax > 0.f ? min(127, 8 - eu) : 0;      // max |u 2^ku| <= 256 (e4m3 max 448)
  const int sbu = 127 - ku;
  const float qu = ldexpf(1.f, ku);
  i32x8 uf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int q4 = 0; q4 < 8; ++q4) {
      const float4 a = *reinterpret_cast<const float4*>(urow + dbase + 64 * ks + 4 * q4);
      uf[ks][q4] = pack_fp8x4(a.x * qu, a.y * qu, a.z * qu, a.w * qu);
    }
    __builtin_amdgcn_sched_barrier(0);  // one k-step's loads in flight at a time (registers)
  }

  // LDS-DMA: tile bytes [(w PW + i) KiB, +1 KiB) into the same place of the ring slot
  // (one VGPR: the piece index moves the scalar soffset and M0, not the lane offset)
  const int voff = w * PW * 1024 + lane * 16;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(T8), (short)0, (int)(ntiles * TB), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(w * PW * 1024);
  auto issue_range = [&](int64_t t, int slot_i, int i0, int i1) {
    const uint32_t soff = (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)TB));
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
#pragma unroll
    for (int i = i0; i < i1; ++i)
      if (i == i0)  // soff may be fresh from v_readfirstlane: 5 wait states before a buffer op reads it
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff), "s"(rsrc), "s"(soff + (uint32_t)(i * 1024))
                     : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff), "s"(rsrc), "s"(soff + (uint32_t)(i * 1024))
                     : "memory");
  };
  auto issue = [&](int64_t t, int slot_i) { issue_range(t, slot_i, 0, PW); };
  auto lds_fence = [] { asm volatile("" ::: "memory"); };
  auto barrier = [&] {
    lds_fence();
    __builtin_amdgcn_s_barrier();
    lds_fence();
  };

  // GEMM1 A operand (ks, half): item row 32 half + col, chunks 4 (ks0 + ks) + 2 h + {0, 1}
  // GEMM2 A operand (d-block db): four transposed reads, read c = items f8_item_of(h, 8 c + q) (q = 0..7)
  // The swizzle only permutes chunks within periods of PC chunks, so DS = 1 keeps each lane's in-period
  // offsets in registers (8 + 16, or 16 + 32 for PC = 16) and every read is base + offset + immediate;
  // the D split (register-bound) recomputes them per read.
  constexpr int PC = D % 256 == 0 ? 16 : 8;  // swizzle period in chunks
  constexpr int NA = PC / 4, NB = PC / 2;
  const int swc = f8_sw(D, col);
  const int g1 = (lane >> 4) & 1, qq = (lane & 15) >> 1, pp = lane & 1;
  int trow[4], tsw[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int it = f8_item_of(h, 8 * c + qq);
    trow[c] = it * D + 8 * pp;
    tsw[c] = f8_sw(D, it);
  }
  int offA[DS == 1 ? 2 : 1][DS == 1 ? NA : 1][2], offB[4][DS == 1 ? NB : 1];
  if constexpr (DS == 1) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int k = 0; k < NA; ++k)
#pragma unroll
        for (int part = 0; part < 2; ++part)
          offA[hf][k][part] = (32 * hf + col) * D + 16 * ((4 * k + 2 * h + part) ^ swc);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < NB; ++k) offB[c][k] = trow[c] + 16 * ((2 * k + g1) ^ tsw[c]);
  }
  auto rdA = [&](const unsigned char* buf, int ks, int half) {
    uint4 x, y;
    if constexpr (DS == 1) {
      const unsigned char* b = buf + 16 * PC * (ks / NA);
      x = *reinterpret_cast<const uint4*>(b + offA[half][ks % NA][0]);
      y = *reinterpret_cast<const uint4*>(b + offA[half][ks % NA][1]);
    } else {
      const int ch = 4 * (dbase / 64 + ks) + 2 * h;
      const unsigned char* row = buf + (32 * half + col) * D;
      x = *reinterpret_cast<const uint4*>(row + 16 * (ch ^ swc));
      y = *reinterpret_cast<const uint4*>(row + 16 * ((ch + 1) ^ swc));
    }
    i32x8 r;
    r[0] = (int)x.x; r[1] = (int)x.y; r[2] = (int)x.z; r[3] = (int)x.w;
    r[4] = (int)y.x; r[5] = (int)y.y; r[6] = (int)y.z; r[7] = (int)y.w;
    return r;
  };
  auto rdB = [&](const unsigned char* buf, int db) {
    i32x8 r;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const unsigned char* a;
      if constexpr (DS == 1) {
        a = buf + 16 * PC * (db / NB) + offB[c][db % NB];
      } else {
        const int ch = 2 * (dbase / 32 + db) + g1;
        a = buf + trow[c] + 16 * (ch ^ tsw[c]);
      }
      const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) i32x2*)(void*)a);
      r[2 * c] = v[0];
      r[2 * c + 1] = v[1];
    }
    return r;
  };
  // GEMM1 (this wave's dims): S^T of items 0-31 (s0) and 32-63 (s1) of the tile
  auto gemm1 = [&](const unsigned char* buf, f32x16& s0, f32x16& s1, auto&& fill) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
    // A operands of G1A k-steps in flight (DS = 1; the D split has no registers for a second)
    constexpr int G1A = DS == 1 ? F8_G1_AHEAD : 1;
    i32x8 ra0[G1A], ra1[G1A];
#pragma unroll
    for (int j = 0; j < G1A; ++j)
      if (j < KS) { ra0[j] = rdA(buf, j, 0); ra1[j] = rdA(buf, j, 1); }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const i32x8 c0 = ra0[ks % G1A], c1 = ra1[ks % G1A];
      if (ks + G1A < KS) { ra0[ks % G1A] = rdA(buf, ks + G1A, 0); ra1[ks % G1A] = rdA(buf, ks + G1A, 1); }
      s0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c0, uf[ks], s0, 0, 0, 0, sa, 0, sbu);
      s1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c1, uf[ks], s1, 0, 0, 0, sa, 0, sbu);
      fill(ks);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  // GEMM2 A operands in flight: DS = 1 keeps F8_G2_AHEAD d-blocks of transposed reads ahead (the D split has
  // no registers for more than one). Measured at Syn-1M shape: 1, 2, 3, 4 ahead = 363, 359, 361, 359 us, so the
  // operand latency is not what bounds the sweep (scripts/gpu_dec8_ab.sh)
  constexpr int AH2 = DS == 1 ? F8_G2_AHEAD : F8_DS2_AHEAD;
  auto gemm2 = [&](const unsigned char* buf, const i32x8& pf, int sbp, auto&& after) {
    if constexpr (WITH_O) {
      i32x8 a[AH2];
#pragma unroll
      for (int j = 0; j < AH2; ++j)
        if (j < DB) a[j] = rdB(buf, j);
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        const i32x8 c = a[db % AH2];
        if (db + AH2 < DB) a[db % AH2] = rdB(buf, db + AH2);
        o[db] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c, pf, o[db], 0, 0, 0, sa, 0, sbp);
        after(db);
      }
    }
  };

  float m = 0.f, mL = 0.f, lsum = 0.f;
  const float bound = sqrtf(usq) * emax * 1.02f;
  // per tile: mask items past N (read as 0), the fixed per-split offset on the first tile, the tile's
  // P exponent e (q = exp2(s log2e - mL - e) <= 2^8); returns e
  auto tile_prep = [&](int64_t t, f32x16& c0, f32x16& c1) {
    if (t == ntiles - 1 && (N % kF8TI) != 0) {
      const int lim = (int)(N - t * kF8TI) - 4 * h;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int it = (r & 3) + 8 * (r >> 2);
        c0[r] = it >= lim ? -INFINITY : c0[r];
        c1[r] = it + 32 >= lim ? -INFINITY : c1[r];
      }
    }
    // tree of v_max3 (depth 4 instead of a 31-long chain), then the other lane half through
    // v_permlane32_swap (a VALU op; __shfl_xor is an LDS round trip): r[0] / r[1] = the value of lane
    // (l & 31) / (l & 31) + 32, so their max is the column's in every lane
    float t3[11];
#pragma unroll
    for (int i = 0; i < 5; ++i) t3[i] = fmaxf(fmaxf(c0[3 * i], c0[3 * i + 1]), c0[3 * i + 2]);
#pragma unroll
    for (int i = 0; i < 5; ++i) t3[5 + i] = fmaxf(fmaxf(c1[3 * i], c1[3 * i + 1]), c1[3 * i + 2]);
    t3[10] = fmaxf(c0[15], c1[15]);
    const float u0 = fmaxf(fmaxf(t3[0], t3[1]), t3[2]), u1 = fmaxf(fmaxf(t3[3], t3[4]), t3[5]);
    const float u2 = fmaxf(fmaxf(t3[6], t3[7]), t3[8]), u3 = fmaxf(t3[9], t3[10]);
    float mx = fmaxf(fmaxf(u0, u1), fmaxf(u2, u3));
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    if (t == t_beg) {  // as k_dec2_bf16: p = exp(s - m) <= e^60, never rescaled; flagged if l ends tiny
      m = fmaxf(mx, bound - kOffsetSpan);
      mL = m * kLog2e;
    }
    return max(-119, min(127, (int)ceilf(__builtin_fmaf(mx, kLog2e, -mL)) - 8));
  };

  if constexpr (DS == 1) {
    f32x16 c0, c1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { c0[r] = 0.f; c1[r] = 0.f; }
    constexpr int PRE = NS - 1;  // tiles in flight before the loop
    if (t_beg < t_end) {
#pragma unroll
      for (int i = 0; i < PRE; ++i) issue(min(t_beg + i, t_end - 1), i);
      wait_vmcnt<(PRE - 1) * PW>();
    }
    barrier();
    if (t_beg < t_end && wave_active) gemm1(lds, c0, c1, [](int) {});
    int cur = 0;
    for (int64_t t = t_beg; t < t_end; ++t) {
      wait_vmcnt<(NS - 3) * PW>();  // tile t + 1 has landed
      barrier();
      const int nxt = cur == NS - 1 ? 0 : cur + 1;
      // tile t + NS - 1 into the slot of tile t - 1 (every wave finished its GEMM2 before the barrier):
      // in one burst here, or (F8_SPREAD) its pieces spread over GEMM2(t)'s MFMAs (Syn-1M shape: 334 us burst,
      // 349 us spread)
      const int64_t t_dma = min(t + NS - 1, t_end - 1);
      const int s_dma = cur == 0 ? NS - 1 : cur - 1;
      constexpr bool spread = F8_SPREAD && WITH_O;
      if (!spread || !wave_active) issue(t_dma, s_dma);
      if (wave_active) {
        int e = 0;
        float cE = 0.f;
        float qv[32];
        int pk[8];
        float qsum = 0.f;
        auto smax = [&](int j0, int j1) {
#pragma unroll
          for (int j = j0; j < j1; ++j) {
            const float s = j < 16 ? c0[j & 15] : c1[j & 15];
            qv[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(s, kLog2e, -cE));
            qsum += qv[j];
            if ((j & 3) == 3) pk[j >> 2] = pack_fp8x4(qv[j - 3], qv[j - 2], qv[j - 1], qv[j]);
          }
        };
        f32x16 n0, n1;
        // tile t's max and exponent under GEMM1(t+1)'s first MFMA pair, its exponentials under the others
        gemm1(lds + nxt * TB, n0, n1, [&](int g) {
          if (g == 0) {
            e = tile_prep(t, c0, c1);
            cE = mL + (float)e;
          } else {
            smax(4 * ((8 * (g - 1)) / (KS - 1)), 4 * ((8 * g) / (KS - 1)));
          }
        });
        lsum += ldexpf(qsum, e);
        i32x8 pf;
#pragma unroll
        for (int i = 0; i < 8; ++i) pf[i] = pk[i];
        gemm2(lds + cur * TB, pf, 127 + e, [&](int db) {
          if constexpr (spread)
            if (PW * db / DB < PW * (db + 1) / DB) issue_range(t_dma, s_dma, PW * db / DB, PW * (db + 1) / DB);
        });
        c0 = n0;
        c1 = n1;
      }
      cur = nxt;
    }
  } else if constexpr (F8_DS2_RING) {
    // DS = 2, 3-slot ring: wave dh owns the softmax of items 32 dh .. 32 dh + 31. Per tile: the partial S^T of
    // the partner's item half crosses through LDS (4 KiB per wave), the wave completes its own half, runs its
    // 16 exponentials under GEMM1(t+1)'s MFMAs, and the packed P half and its block exponent cross back
    // through the same buffer (the MFMA takes block b's scale from lane column + 32 b) before GEMM2(t).
    // Three 48 KiB slots + 4 x 4 KiB exchange = 160 KiB.
    float* xmine = reinterpret_cast<float*>(lds + NS * TB + w * 4096);
    const float* xpart = reinterpret_cast<const float*>(lds + NS * TB + (w ^ 2) * 4096);
    auto half_of = [&](const f32x16& a0, const f32x16& a1) -> const f32x16& { return dh == 0 ? a0 : a1; };
    auto put16 = [&](const f32x16& sv) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4)
        *reinterpret_cast<float4*>(xmine + r4 * 256 + lane * 4) =
            make_float4(sv[4 * r4], sv[4 * r4 + 1], sv[4 * r4 + 2], sv[4 * r4 + 3]);
    };
    // own half's full S^T = d-half 0 partial + d-half 1 partial (the same order in both waves' halves)
    auto complete = [&](const f32x16& own, f32x16& sm) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 y = *reinterpret_cast<const float4*>(xpart + r4 * 256 + lane * 4);
        const float yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) sm[4 * r4 + k] = dh == 0 ? own[4 * r4 + k] + yv[k] : yv[k] + own[4 * r4 + k];
      }
    };
    auto half_max = [&](int64_t t, f32x16& sm) {
      if (t == ntiles - 1 && (N % kF8TI) != 0) {
        const int lim = (int)(N - t * kF8TI) - 4 * h - 32 * dh;
#pragma unroll
        for (int r = 0; r < 16; ++r) sm[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : sm[r];
      }
      const float a0 = fmaxf(fmaxf(sm[0], sm[1]), sm[2]), a1 = fmaxf(fmaxf(sm[3], sm[4]), sm[5]);
      const float a2 = fmaxf(fmaxf(sm[6], sm[7]), sm[8]), a3 = fmaxf(fmaxf(sm[9], sm[10]), sm[11]);
      const float a4 = fmaxf(fmaxf(sm[12], sm[13]), fmaxf(sm[14], sm[15]));
      float mx = fmaxf(fmaxf(fmaxf(a0, a1), a2), fmaxf(a3, a4));
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    };
    f32x16 c0, c1;  // this wave's partial S^T of the current tile (both item halves)
#pragma unroll
    for (int r = 0; r < 16; ++r) { c0[r] = 0.f; c1[r] = 0.f; }
    constexpr int PRE = NS - 1;
    if (t_beg < t_end) {
#pragma unroll
      for (int i = 0; i < PRE; ++i) issue(min(t_beg + i, t_end - 1), i);
      wait_vmcnt<(PRE - 1) * PW>();
    }
    barrier();
    if (t_beg < t_end && wave_active) gemm1(lds, c0, c1, [](int) {});
    int cur = 0;
    for (int64_t t = t_beg; t < t_end; ++t) {
      wait_vmcnt<(NS - 3) * PW>();  // tile t + 1 has landed
      barrier();                    // B1: iteration t - 1 is over everywhere (slot t - 1, exchange buffer)
      const int nxt = cur == NS - 1 ? 0 : cur + 1;
      issue(min(t + NS - 1, t_end - 1), cur == 0 ? NS - 1 : cur - 1);
      if (wave_active) put16(half_of(c1, c0));  // the partner's item half of my D-half partial
      barrier();                                // B2
      f32x16 sm;
      float mh = 0.f;
      if (wave_active) {
        complete(half_of(c0, c1), sm);
        mh = half_max(t, sm);
      }
      if (t == t_beg) {  // the pair's common offset from the first tile's max over both halves
        barrier();
        if (wave_active) xmine[lane] = mh;
        barrier();
        if (wave_active) {
          m = fmaxf(fmaxf(mh, xpart[lane]), bound - kOffsetSpan);
          mL = m * kLog2e;
        }
      }
      int e = 0;
      int pk[4];
      f32x16 n0, n1;
      if (wave_active) {
        e = max(-119, min(127, (int)ceilf(__builtin_fmaf(mh, kLog2e, -mL)) - 8));
        const float cE = mL + (float)e;
        float qv[16];
        float qsum = 0.f;
        gemm1(lds + nxt * TB, n0, n1, [&](int g) {
#pragma unroll
          for (int j = 4 * ((4 * g) / KS); j < 4 * ((4 * g + 4) / KS); ++j) {
            qv[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(sm[j], kLog2e, -cE));
            qsum += qv[j];
            if ((j & 3) == 3) pk[j >> 2] = pack_fp8x4(qv[j - 3], qv[j - 2], qv[j - 1], qv[j]);
          }
        });
        lsum += ldexpf(qsum, e);
      }
      barrier();  // B3: the partner has read my partial
      if (wave_active) {
        reinterpret_cast<int4*>(xmine)[lane] = make_int4(pk[0], pk[1], pk[2], pk[3]);
        reinterpret_cast<int*>(xmine)[256 + lane] = e;
      }
      barrier();  // B4
      if (wave_active) {
        const int4 y = reinterpret_cast<const int4*>(xpart)[lane];
        const int ey = reinterpret_cast<const int*>(xpart)[256 + lane];
        i32x8 pf;
        if (dh == 0) {
          pf[0] = pk[0]; pf[1] = pk[1]; pf[2] = pk[2]; pf[3] = pk[3];
          pf[4] = y.x; pf[5] = y.y; pf[6] = y.z; pf[7] = y.w;
        } else {
          pf[0] = y.x; pf[1] = y.y; pf[2] = y.z; pf[3] = y.w;
          pf[4] = pk[0]; pf[5] = pk[1]; pf[6] = pk[2]; pf[7] = pk[3];
        }
        gemm2(lds + cur * TB, pf, 127 + (h == dh ? e : ey), [](int) {});  // lane half h: block h's scale
        c0 = n0;
        c1 = n1;
      }
      cur = nxt;
    }
    // the user's l = l(items 0-31) + l(items 32-63), the same sum in both waves
    const float lw = lsum + __shfl_xor(lsum, 32, 64);
    barrier();
    if (wave_active) xmine[lane] = lw;
    barrier();
    if (wave_active) lsum = dh == 0 ? lw + xpart[lane] : xpart[lane] + lw;
  } else {
    // DS = 2, two slots: tile t + 1's LDS-DMA runs under all of tile t
    float* xbuf = reinterpret_cast<float*>(lds + NS * TB);  // [4 w][2 s][64 lane][16]
    auto xput = [&](const f32x16& s0, const f32x16& s1) {
      float* xb = xbuf + w * 2048;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        *reinterpret_cast<float4*>(xb + r4 * 256 + lane * 4) = make_float4(s0[4 * r4], s0[4 * r4 + 1], s0[4 * r4 + 2],
                                                                           s0[4 * r4 + 3]);
        *reinterpret_cast<float4*>(xb + 1024 + r4 * 256 + lane * 4) =
            make_float4(s1[4 * r4], s1[4 * r4 + 1], s1[4 * r4 + 2], s1[4 * r4 + 3]);
      }
    };
    auto xadd = [&](f32x16& s0, f32x16& s1) {
      const float* xb = xbuf + (w ^ 2) * 2048;
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const float4 v = *reinterpret_cast<const float4*>(xb + r4 * 256 + lane * 4);
        const float4 u = *reinterpret_cast<const float4*>(xb + 1024 + r4 * 256 + lane * 4);
        s0[4 * r4] += v.x; s0[4 * r4 + 1] += v.y; s0[4 * r4 + 2] += v.z; s0[4 * r4 + 3] += v.w;
        s1[4 * r4] += u.x; s1[4 * r4 + 1] += u.y; s1[4 * r4 + 2] += u.z; s1[4 * r4 + 3] += u.w;
      }
    };
    if (t_beg < t_end) {
      issue(t_beg, 0);
      issue(min(t_beg + 1, t_end - 1), 1);
    }
    int cur = 0;
    for (int64_t t = t_beg; t < t_end; ++t) {
      wait_vmcnt<PW>();  // tile t has landed (t + 1 may be in flight)
      barrier();
      f32x16 c0, c1;
      if (wave_active) {
        gemm1(lds + cur * TB, c0, c1, [](int) {});
        xput(c0, c1);
      }
      barrier();
      if (wave_active) {
        xadd(c0, c1);
        const int e = tile_prep(t, c0, c1);
        const float cE = mL + (float)e;
        i32x8 pf;
        float qsum = 0.f;
#pragma unroll
        for (int j4 = 0; j4 < 8; ++j4) {
          float q[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int j = 4 * j4 + b;
            q[b] = __builtin_amdgcn_exp2f(__builtin_fmaf(j < 16 ? c0[j & 15] : c1[j & 15], kLog2e, -cE));
            qsum += q[b];
          }
          pf[j4] = pack_fp8x4(q[0], q[1], q[2], q[3]);
        }
        lsum += ldexpf(qsum, e);
        gemm2(lds + cur * TB, pf, 127 + e, [](int) {});
      }
      barrier();  // slot cur and the exchange buffer are free
      issue(min(t + 2, t_end - 1), cur);
      cur ^= 1;
    }
  }

  if (!wave_active) return;
  const float ltot = (DS == 2 && F8_DS2_RING) ? lsum : lsum + __shfl_xor(lsum, 32, 64);
  if (user >= nb) return;
  if (h == 0 && dh == 0) out.flag[out.direct ? user : (int64_t)split * nb + user] = !(ltot >= kMinL);
  if (out.direct) {
    const float inv = 1.0f / ltot;
    if (h == 0 && dh == 0) out.lse[user] = m + logf(ltot);
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + user * D + dd) =
              make_float4(o[d][4 * g4] * inv, o[d][4 * g4 + 1] * inv, o[d][4 * g4 + 2] * inv, o[d][4 * g4 + 3] * inv);
        }
    }
  } else {
    const int64_t pi = (int64_t)split * nb + user;
    if (h == 0 && dh == 0) { out.m[pi] = m; out.l[pi] = ltot; }
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = dbase + 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + pi * D + dd) =
              make_float4(o[d][4 * g4], o[d][4 * g4 + 1], o[d][4 * g4 + 2], o[d][4 * g4 + 3]);
        }
    }
  }
}


// ------------------------------------------------------------------- f32 ---
// Same algorithm on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 sums):
// 4 waves x 16 users, 16-item tiles, LDS rows padded to D+2 floats
// (conflict-free GEMM1 reads, 2-way on half of the GEMM2 reads).
constexpr int kF32TI = 16;
constexpr int kF32UsersPerWave = 16;
constexpr int kF32UsersPerBlock = 64;

template <int D>
constexpr int f32_tile_bytes() { return kF32TI * (D + 2) * 4; }

template <int D, bool WITH_O>
__global__ void __launch_bounds__(256) k_dec_f32(const float* __restrict__ U, int64_t ldu,
                                                 const float* __restrict__ E, int64_t nb, int64_t N,
                                                 int splits, int64_t tiles_per_split, DecOut out) {
  static_assert(D % 16 == 0, "D must be a multiple of 16");
  constexpr int KS = D / 4;
  constexpr int DB = D / 16;
  constexpr int LD = D + 2;
  constexpr int TF = kF32TI * LD;           // floats per tile buffer
  constexpr int Q4 = D / 4;                 // float4 per row
  constexpr int LPT = (kF32TI * Q4 + 255) / 256;
  extern __shared__ __attribute__((aligned(16))) float ldsf[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, q = lane >> 4, c16 = lane & 15;
  const int split = blockIdx.x % splits;
  const int64_t ub = blockIdx.x / splits;
  const int64_t u0 = ub * kF32UsersPerBlock + w * kF32UsersPerWave;
  const int64_t user = u0 + c16;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kF32TI - 1) / kF32TI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);

  float uf[KS];  // B operand of GEMM1: U[user][4 ks + q]
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) uf[ks] = (user < nb) ? U[user * ldu + 4 * ks + q] : 0.f;

  f32x4 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, lsum = 0.f;

  float4 stage[LPT];
  auto gload = [&](int64_t t) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      const int row = c / Q4, c4 = c % Q4;
      const int64_t item = t * kF32TI + row;
      stage[i] = (c < kF32TI * Q4 && item < N) ? *reinterpret_cast<const float4*>(E + item * D + 4 * c4)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto lstore = [&](float* buf) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = tid + 256 * i;
      if (c < kF32TI * Q4) {
        const int row = c / Q4, c4 = c % Q4;
        float* dst = buf + row * LD + 4 * c4;  // LD is even: 8-B aligned pairs
        dst[0] = stage[i].x; dst[1] = stage[i].y; dst[2] = stage[i].z; dst[3] = stage[i].w;
      }
    }
  };

  if (t_beg < t_end) {
    gload(t_beg);
    lstore(ldsf);
    __syncthreads();
  }
  int cur = 0;
  for (int64_t t = t_beg; t < t_end; ++t) {
    const bool more = t + 1 < t_end;
    if (more) gload(t + 1);
    const float* buf = ldsf + cur * TF;
    if (wave_active) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        s = __builtin_amdgcn_mfma_f32_16x16x4f32(buf[c16 * LD + 4 * ks + q], uf[ks], s, 0, 0, 0);
      // S^T: row = item 4q + r, col = user c16
      const int64_t ib = t * kF32TI + 4 * q;
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (ib + r >= N) s[r] = -INFINITY;
        mx = fmaxf(mx, s[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (__any(mx > m + kThr)) {
        const float mn = fmaxf(m, mx);
        const float alpha = __expf(m - mn);
        lsum *= alpha;
        if (WITH_O) {
#pragma unroll
          for (int d = 0; d < (WITH_O ? DB : 1); ++d) o[d] *= alpha;
        }
        m = mn;
      }
      float p[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = __expf(s[r] - m);
        lsum += p[r];
      }
      if (WITH_O) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int d = 0; d < (WITH_O ? DB : 1); ++d)
            o[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(buf[(4 * q + r) * LD + 16 * d + c16], p[r], o[d], 0, 0, 0);
      }
    }
    if (more) lstore(ldsf + (cur ^ 1) * TF);
    __syncthreads();
    cur ^= 1;
  }

  if (!wave_active) return;
  float ltot = lsum + __shfl_xor(lsum, 16, 64);
  ltot += __shfl_xor(ltot, 32, 64);
  if (user >= nb) return;
  // O^T block d: lane holds d-rows 16 d + 4 q + r for user c16
  if (out.direct) {
    const float inv = 1.0f / ltot;
    if (q == 0) out.lse[user] = m + logf(ltot);
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
        *reinterpret_cast<float4*>(out.O + user * D + 16 * d + 4 * q) =
            make_float4(o[d][0] * inv, o[d][1] * inv, o[d][2] * inv, o[d][3] * inv);
    }
  } else {
    const int64_t pi = (int64_t)split * nb + user;
    if (q == 0) { out.m[pi] = m; out.l[pi] = ltot; }
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
        *reinterpret_cast<float4*>(out.O + pi * D + 16 * d + 4 * q) = make_float4(o[d][0], o[d][1], o[d][2], o[d][3]);
    }
  }
}

// Combine the per-split (m, l, O) partials: one block per user; the split
// weights exp(m_s - M) live in LDS, threads run over D (coalesced rows).
constexpr int kMaxSplits = 4096;

__device__ float exact_user(int64_t b, const float* __restrict__ U, int64_t ldu, const bf16_t* __restrict__ E,
                            int64_t N, int64_t D, float (&o)[4], float* red, float* pbuf);

// Per-user finalisation of the streaming decoder, one 256-thread block per user:
//   1. combine the per-split (m, l, O) partials (or take the single-split result),
//   2. recompute exactly if a split flagged the user (bf16 fixed-offset underflow),
//   3. if a CSR batch is given, the sparse half of the loss and of d(u):
//        recon_rows[b] = n_b lse_b - u_b . (sum_j x_bj E_j)
//        dU[b]         = scale (n_b O_b - sum_j x_bj E_j)          (fp32 E)
// Thread t owns d = t + 256 k (D <= 1024) throughout, so O never round-trips
// through memory between the steps.
struct FinArgs {
  const float* pm; const float* pl; const float* pO;  // partial mode (splits > 1)
  const int* flag;                                    // [splits][nb] / [nb] or NULL
  int splits;
  const float* lse_in; const float* O_in;             // direct mode (splits == 1)
  const float* U; int64_t ldu; const bf16_t* Ebf;     // exact fixup inputs (bf16 path)
  const float* E32; int64_t N; int64_t D; int64_t nb;
  const int64_t* row_ptr; const int32_t* col_idx; const float* vals;
  const int32_t* rows; const int64_t* rows_offset;    // CSR batch (nullable row_ptr => no sparse terms)
  float scale;
  float* lse_out; float* O_out; float* recon_rows; float* dU;
  const float* kl_rows; float beta; const float* beta_dev; float* loss3; double* accum3;  // fused loss (optional)
  unsigned* ticket;
  // version-6 partials (hvae_dec6.h): user b's slots are dec6_slot_of(.., b / v6_upb, i), rows slot * v6_upb + b % v6_upb
  int v6_upb, v6_nub, v6_S, v6_main, v6_P;
};

#ifndef FIN_EB_V4
#define FIN_EB_V4 8  // 16-B form: 8 entries x 16 B in flight per thread (59 VGPRs, 7 waves per SIMD) beat 16 (99, 4): Syn-1M shape 33.5 -> 27.9 us, Syn-10M 45.5 -> 39.8 (profiles/r05_finalize_eb_ab.jsonl)
#endif
constexpr int kFinEB = 16;  // CSR entries per batch of the finalize's sparse-term loads

// GRP: the merge of many split partials (> 8) by split groups (memory-level parallelism at small
// batches); otherwise one thread per column walks the splits in order (fewer registers, more blocks
// per CU at large batches). V4 (every row operand 16-B aligned, as the host checks): thread t owns the four
// columns 4 t .. 4 t + 3 and moves them as one 16-B load / store (the scalar form's thread owns t + 256 k and
// issues four times the load instructions for the same bytes: 2.2-3.1 TB/s, profiles/pmc_syn1m.json)
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void f4_fma(float4& acc, float w, const float4& v) {
  acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
}
template <bool GRP, bool V4>
__global__ void __launch_bounds__(256) k_dec_finalize(FinArgs a) {
  constexpr int EB = V4 ? FIN_EB_V4 : kFinEB;  // CSR entries per batch of the sparse-term loads
  __shared__ float wsh[kMaxSplits];
  __shared__ __attribute__((aligned(16))) float obuf[V4 ? 1024 : 4];  // exact fixup's columns -> V4 layout
  __shared__ __attribute__((aligned(16))) float opart[GRP ? 8 * 1024 : 4];  // per-split-group O sums
  __shared__ float red[4];
  __shared__ float pbuf[256];
  __shared__ int any_flag;
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t D = a.D;
  // the batch row's CSR entries: located and the first EB fetched now, under the merge's loads
  int64_t sp_beg = 0, sp_end = 0;
  int sp_j[EB];
  float sp_x[EB];
  if (a.row_ptr) {
    const int64_t r = batch_row(a.rows, a.rows_offset, b);
    sp_beg = a.row_ptr[r];
    sp_end = a.row_ptr[r + 1];
  }
#pragma unroll
  for (int u = 0; u < EB; ++u) {
    const int64_t e = sp_beg + u;
    sp_j[u] = e < sp_end ? a.col_idx[e] : 0;
    sp_x[u] = e < sp_end ? a.vals[e] : 0.f;
  }
  if (tid == 0) any_flag = 0;
  __syncthreads();
  float lse_b;
  float o[4] = {0.f, 0.f, 0.f, 0.f};
  int nsp = a.splits;
#if HVAE_AB  // version 6's slot rows (A/B library only)
  const int v6u = a.v6_upb ? (int)(b / a.v6_upb) : 0;
  const int64_t v6j = a.v6_upb ? b % a.v6_upb : 0;
  if (a.v6_upb) nsp = dec6_nslots(a.v6_nub, a.v6_S, a.v6_main, a.v6_P, v6u);
  auto prow = [&](int s) -> int64_t {  // partial row of user b's s-th split / slot
    return a.v6_upb ? (int64_t)dec6_slot_of(a.v6_nub, a.v6_S, a.v6_main, a.v6_P, v6u, s) * a.v6_upb + v6j
                    : (int64_t)s * a.nb + b;
  };
#else
  auto prow = [&](int s) -> int64_t { return (int64_t)s * a.nb + b; };  // partial row of user b's s-th split
#endif
  if (a.splits > 1 || a.v6_upb) {
    float M = -INFINITY;
    int fl = 0;
    for (int s = tid; s < nsp; s += 256) {
      const int64_t r = prow(s);
      M = fmaxf(M, a.pm[r]);
      if (a.flag) fl |= a.flag[r];
    }
    if (fl) any_flag = 1;
    M = wave_max(M);
    if ((tid & 63) == 0) red[tid >> 6] = M;
    __syncthreads();
    M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float L = 0.f;
    for (int s = tid; s < nsp; s += 256) {
      const int64_t r = prow(s);
      const float ms = a.pm[r];
      const float wv = (ms == -INFINITY) ? 0.f : __expf(ms - M);
      wsh[s] = wv;
      L += wv * a.pl[r];
    }
    L = block_sum<256>(L, red);  // its barriers also publish wsh and any_flag
    lse_b = M + logf(L);
    const float inv = 1.0f / L;
    if (V4 && a.pO && !GRP) {  // sum_s w_s O_s in split order, 8 splits' 16-B loads in flight
      const bool act = 4 * tid < D;
      float4 acc4 = make_float4(0.f, 0.f, 0.f, 0.f);
      int s0 = 0;
      for (; s0 + 8 <= nsp; s0 += 8) {
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act ? ld4(a.pO + prow(s0 + j) * D + 4 * tid) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f4_fma(acc4, wsh[s0 + j], v[j]);
      }
      for (; s0 < nsp; ++s0)
        if (act) f4_fma(acc4, wsh[s0], ld4(a.pO + prow(s0) * D + 4 * tid));
      o[0] = acc4.x * inv; o[1] = acc4.y * inv; o[2] = acc4.z * inv; o[3] = acc4.w * inv;
    }
    if (!V4 && a.pO && !GRP) {
      // sum_s w_s O_s in split order; loads batched 8 splits x 4 columns deep so that
      // they are in flight together (a one-at-a-time chain is HBM-latency bound)
      const int nk = (int)min<int64_t>(4, (D - tid + 255) / 256);
      const float* base = a.pO + tid;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      int s0 = 0;
      for (; s0 + 8 <= nsp; s0 += 8) {
        float v[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float* rp = base + prow(s0 + j) * D;
#pragma unroll
          for (int k = 0; k < 4; ++k) v[j][k] = k < nk ? rp[256 * k] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] += wsh[s0 + j] * v[j][k];
      }
      for (; s0 < nsp; ++s0) {
        const float* rp = base + prow(s0) * D;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < nk) acc[k] += wsh[s0] * rp[256 * k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = acc[k] * inv;
    }
    if constexpr (GRP) if (a.pO) {
      // sum_s w_s O_s (many splits): 8 split groups x 32 float4-column lanes, thread (sg, cq) sums splits sg, sg + 8, ...
      // over float4 columns cq + 32 i, 4 splits' loads in flight together (one HBM latency per 32 splits
      // instead of a chain); the 8 group sums are then added in group order through LDS (deterministic)
      constexpr int SG = 8;
      const int sg = tid >> 5, cq = tid & 31;
      const int nq = (int)(D >> 2);
      float4 acc4[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int s0 = sg; s0 < nsp; s0 += SG * 4) {
        float4 v[4][8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sj = s0 + SG * j;
          const float4* row = reinterpret_cast<const float4*>(a.pO + (sj < nsp ? prow(sj) : 0) * D);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int q = cq + 32 * i;
            v[j][i] = (sj < nsp && q < nq) ? row[q] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sj = s0 + SG * j;
          const float wv = sj < nsp ? wsh[sj] : 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc4[i].x += wv * v[j][i].x; acc4[i].y += wv * v[j][i].y;
            acc4[i].z += wv * v[j][i].z; acc4[i].w += wv * v[j][i].w;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int q = cq + 32 * i;
        if (q < nq) reinterpret_cast<float4*>(opart + sg * 1024)[q] = acc4[i];
      }
      __syncthreads();
      if constexpr (V4) {
        if (4 * tid < D) {
          float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int g = 0; g < SG; ++g) {
            const float4 v = reinterpret_cast<const float4*>(opart + g * 1024)[tid];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
          }
          o[0] = t.x * inv; o[1] = t.y * inv; o[2] = t.z * inv; o[3] = t.w * inv;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t d = tid + 256 * k;
          float t = 0.f;
          if (d < D) {
#pragma unroll
            for (int g = 0; g < SG; ++g) t += opart[g * 1024 + d];
          }
          o[k] = t * inv;
        }
      }
    }
  } else {
    if (a.flag && a.flag[b]) any_flag = 1;
    lse_b = a.lse_in[b];
    if (a.O_in) {
      if constexpr (V4) {
        if (4 * tid < D) {
          const float4 v = ld4(a.O_in + b * D + 4 * tid);
          o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t d = tid + 256 * k;
          if (d < D) o[k] = a.O_in[b * D + d];
        }
      }
    }
    __syncthreads();
  }
  if (any_flag) {  // rare, block-uniform
    lse_b = exact_user(b, a.U, a.ldu, a.Ebf, a.N, D, o, red, pbuf);  // columns tid + 256 k
    if constexpr (V4) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (tid + 256 * k < D) obuf[tid + 256 * k] = o[k];
      __syncthreads();
      if (4 * tid < D) {
        const float4 v = reinterpret_cast<const float4*>(obuf)[tid];
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
      }
    }
  }
  if (tid == 0) a.lse_out[b] = lse_b;
  if (a.O_out) {
    if constexpr (V4) {
      if (4 * tid < D) *reinterpret_cast<float4*>(a.O_out + b * D + 4 * tid) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t d = tid + 256 * k;
        if (d < D) a.O_out[b * D + d] = o[k];
      }
    }
  }
  if (!a.row_ptr) return;
  // ---- sparse terms against the fp32 E, in ascending entry order; entries EB at a time with all their
  // E loads in flight together (the first chunk's indices were fetched before the merge)
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float n = 0.f;
  for (int64_t e0 = sp_beg; e0 < sp_end; e0 += EB) {
    if (e0 != sp_beg) {
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int64_t e = e0 + u;
        sp_j[u] = e < sp_end ? a.col_idx[e] : 0;
        sp_x[u] = e < sp_end ? a.vals[e] : 0.f;
      }
    }
    float ev[EB][4];
    if constexpr (V4) {
      const bool act = 4 * tid < D;
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const float4 v = (e0 + u < sp_end && act) ? ld4(a.E32 + (int64_t)sp_j[u] * D + 4 * tid)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        ev[u][0] = v.x; ev[u][1] = v.y; ev[u][2] = v.z; ev[u][3] = v.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < EB; ++u)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int64_t d = tid + 256 * k;
          ev[u][k] = (e0 + u < sp_end && d < D) ? a.E32[(int64_t)sp_j[u] * D + d] : 0.f;
        }
    }
#pragma unroll
    for (int u = 0; u < EB; ++u) {
      if (e0 + u >= sp_end) break;
      n += sp_x[u];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += sp_x[u] * ev[u][k];
    }
  }
  float dot = 0.f;
  if constexpr (V4) {
    if (4 * tid < D) {
      const float4 uu = ld4(a.U + b * a.ldu + 4 * tid);
      dot = uu.x * acc[0] + uu.y * acc[1] + uu.z * acc[2] + uu.w * acc[3];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t d = tid + 256 * k;
      if (d < D) dot += a.U[b * a.ldu + d] * acc[k];
    }
  }
  dot = block_sum<256>(dot, red);
  if (a.recon_rows && tid == 0) {
    if (a.loss3) st_shared_f(&a.recon_rows[b], n * lse_b - dot);
    else a.recon_rows[b] = n * lse_b - dot;
  }
  if (a.dU) {
    if constexpr (V4) {
      if (4 * tid < D)
        *reinterpret_cast<float4*>(a.dU + b * D + 4 * tid) =
            make_float4(a.scale * (n * o[0] - acc[0]), a.scale * (n * o[1] - acc[1]), a.scale * (n * o[2] - acc[2]),
                        a.scale * (n * o[3] - acc[3]));
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t d = tid + 256 * k;
        if (d < D) a.dU[b * D + d] = a.scale * (n * o[k] - acc[k]);
      }
    }
  }
  if (a.loss3 && last_block_arrives(a.ticket, gridDim.x))
    loss_block_reduce(a.recon_rows, true, a.kl_rows, a.nb, a.beta_dev ? *a.beta_dev : a.beta, a.loss3, a.accum3);
}

// Exact recompute of one user flagged by k_dec_bf16 (its max score sits more
// than kUnderflowSpan below the fixed offset: only possible for |u| in the
// hundreds). Two passes in fp32 over the bf16 E by one 256-thread block.
// Returns lse; o[k] = O[b, threadIdx.x + 256 k].
__device__ float exact_user(int64_t b, const float* __restrict__ U, int64_t ldu, const bf16_t* __restrict__ E,
                            int64_t N, int64_t D, float (&o)[4], float* red, float* pbuf) {
  const float* u = U + b * ldu;
  auto score = [&](int64_t i) {
    float s = 0.f;
    for (int64_t d = 0; d < D; ++d) s += u[d] * bf2f(E[i * D + d]);
    return s;
  };
  float mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < N; i += 256) mx = fmaxf(mx, score(i));
  mx = wave_max(mx);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float l = 0.f;
  float oacc[4] = {0.f, 0.f, 0.f, 0.f};  // thread owns d = threadIdx.x + 256 k (D <= 1024)
  for (int64_t i0 = 0; i0 < N; i0 += 256) {
    const int64_t i = i0 + threadIdx.x;
    const float pv = (i < N) ? expf(score(i) - mx) : 0.f;
    pbuf[threadIdx.x] = pv;
    l += pv;
    __syncthreads();
    const int64_t cnt = min((int64_t)256, N - i0);
    for (int64_t j = 0; j < cnt; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t d = threadIdx.x + 256 * k;
        if (d < D) oacc[k] += pbuf[j] * bf2f(E[(i0 + j) * D + d]);
      }
    __syncthreads();
  }
  l = block_sum<256>(l, red);
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = oacc[k] / l;
  return mx + logf(l);
}

// bf16 decoder image: E rounded to bf16 [N][D], then the tile-transposed Et (tail items 0)
__global__ void __launch_bounds__(256) k_build_image(const float* __restrict__ E32, int64_t N, int64_t D,
                                                     bf16_t* __restrict__ Ebf, bf16_t* __restrict__ Et,
                                                     int64_t ntiles) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N * D; i += stride) Ebf[i] = f2bf(E32[i]);
  const int64_t tot = ntiles * D * kBfTI;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += stride) {
    const int64_t t = i / (D * kBfTI), r = i % (D * kBfTI);
    const int64_t d = r / kBfTI, pos = r % kBfTI;
    const int64_t item = t * kBfTI + et_item_of_pos((int)pos);
    Et[i] = item < N ? f2bf(E32[item * D + d]) : (bf16_t)0;
  }
}

// e4m3 tiles of the fp8 image: per 64-item tile, rows of D bytes with 16-B chunks swizzled by f8_off;
// E8 = e4m3(E 2^ke), ke from max |E|; items past N are 0. One thread per 4 bytes (4 consecutive d).
__global__ void __launch_bounds__(256) k_build_f8(const float* __restrict__ E32, int64_t N, int64_t D, int64_t ntiles,
                                                  const unsigned* __restrict__ amax_bits, unsigned char* __restrict__ T8,
                                                  int* __restrict__ ke_out) {
  const float amax = __uint_as_float(*amax_bits);
  int ea = 0;
  (void)frexpf(amax, &ea);
  const int ke = amax > 0.f ? min(127, 8 - ea) : 0;  // max |E 2^ke| <= 256
  if (blockIdx.x == 0 && threadIdx.x == 0) *ke_out = ke;
  const float qs = ldexpf(1.f, ke);
  const int64_t words = ntiles * kF8TI * D / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const int64_t item = (i * 4) / D;  // global item; d = 4 consecutive columns
    const int d = (int)((i * 4) % D);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (item < N) v = *reinterpret_cast<const float4*>(E32 + item * D + d);
    const int64_t t = item / kF8TI;
    const int it = (int)(item % kF8TI);
    unsigned char* dst = T8 + t * kF8TI * D + f8_off((int)D, it, d >> 4) + (d & 15);
    *reinterpret_cast<int*>(dst) = pack_fp8x4(v.x * qs, v.y * qs, v.z * qs, v.w * qs);
  }
}

__global__ void __launch_bounds__(256) k_abs_max(const float* __restrict__ x, int64_t n, unsigned* __restrict__ out_bits) {
  float best = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    best = fmaxf(best, fabsf(x[i]));
  best = wave_max(best);
  if ((threadIdx.x & 63) == 0) atomicMax(out_bits, __float_as_uint(best));
}

// max_i ||E_i||_2 over an fp32 or bf16 [N, D] matrix (score bound of the bf16 path).
__global__ void __launch_bounds__(256) k_row_norm_max(int dtype, const void* __restrict__ E, int64_t N, int64_t D,
                                                      unsigned* __restrict__ out_bits) {
  const int lane = threadIdx.x & 63;
  float best = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < N; i += (int64_t)gridDim.x * 4) {
    float s = 0.f;
    for (int64_t d = lane; d < D; d += 64) {
      const float v = dtype == HVAE_BF16 ? bf2f(((const bf16_t*)E)[i * D + d]) : ((const float*)E)[i * D + d];
      s += v * v;
    }
    best = fmaxf(best, sqrtf(wave_sum(s)));
  }
  if (lane == 0) atomicMax(out_bits, __float_as_uint(best));  // non-negative floats order as uints
}


// A/B switches (environment, read at plan time) exist only in variant builds (-DHVAE_AB=1, scripts/build_ab.sh);
// the product library runs one sweep per (dtype, D): bf16 version 2 at D <= 384, version 5 at D = 768, the fp8
// ring, the fp32 sweep.
#if HVAE_AB
static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

// HVAE_DEC_V1=1 selects the version-1 bf16 sweep (transposed image copy), HVAE_DEC_SPLITS=k forces k item splits
static bool dec_use_v1() {
  static const int v = env_int("HVAE_DEC_V1", 0);
  return v != 0;
}
static int dec_forced_splits() { return env_int("HVAE_DEC_SPLITS", 0); }

static int dec_forced_ds() {
  static const int v = env_int("HVAE_DEC_DS", 0);
  return v;
}

static int dec_forced_nw() {
  static const int v = env_int("HVAE_DEC_NW", 0);
  return v;
}
#else
static bool dec_use_v1() { return false; }
static int dec_forced_splits() { return 0; }
static int dec_forced_ds() { return 0; }
static int dec_forced_nw() { return 0; }
static int env_int(const char*, int dflt) { return dflt; }
#endif

static bool v2_supported(int64_t D) { return D == 64 || D == 128 || D == 256 || D == 384 || D == 768; }
// HVAE_DEC_V3=0 keeps the version-2 sweep at D = 768 (A/B; read at every plan, so a test can switch it)
static bool v3_supported(int64_t D) { return D == 768 && env_int("HVAE_DEC_V3", 1) != 0; }
// HVAE_DEC_V4=0 keeps version 3 at D = 768 (A/B; read at every plan)
static bool v4_supported(int64_t D) { return D == 768 && env_int("HVAE_DEC_V4", 1) != 0; }
// HVAE_DEC_V4_384=1 runs version 4 with 8 waves at D = 384 (large batches) instead of version 2's DS = 1 sweep
static bool v4_384(int64_t D, int64_t nb) { return D == 384 && nb > 64 && env_int("HVAE_DEC_V4_384", 0) != 0; }
// version 5 (hvae_decoder5.hip: producer / consumer waves, two per SIMD) runs the bf16 sweep at D = 768 since
// both use the conflict-free GEMM1 row map (2.5 % under version 4 at the Syn-10M shard); HVAE_DEC_V5=0 runs
// version 4 (A/B; read at every plan)
static bool v5_supported(int64_t D) { return D == 768 && env_int("HVAE_DEC_V5", 1) != 0; }
int dec5_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                int splits, int64_t tiles_per_split, int64_t blocks, int* flag, float* m, float* l, float* O,
                float* lse, int direct, hipStream_t st);
int dec5w_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                 int splits, int64_t tiles_per_split, int64_t blocks, int* flag, float* m, float* l, float* O,
                 float* lse, int direct, hipStream_t st);
// HVAE_DEC_V5W=1 (A/B build) runs the d = 384 bf16 sweep of large batches as version 5's producer / consumer split
// with 128 users per block (k_dec5w_bf16). It passes the decoder parity tests but measured slower than version 2's
// DS = 1 sweep at Syn-1M (579-645 vs 520-531 us, profiles/r03_dec5w_vs_v2_syn1m.jsonl), so version 2 stays
static bool v5w_supported(int64_t D) { return D == 384 && env_int("HVAE_DEC_V5W", 0) != 0; }
int dec5_f8_launch(bool with_o, const float* U, int64_t ldu, const unsigned char* T8, const int* ke,
                   const float* enorm, int64_t nb, int64_t N, int splits, int64_t tiles_per_split, int64_t blocks,
                   int* flag, float* m, float* l, float* O, float* lse, int direct, hipStream_t st);

static void dec_set_splits(DecPlan& p, int64_t tiles, int64_t s) {
  s = std::max<int64_t>(1, std::min<int64_t>(s, std::min<int64_t>(tiles, kMaxSplits)));
  p.tiles_per_split = std::max<int64_t>(1, cdiv(tiles, s));  // N = 0: one empty split
  p.splits = (int)cdiv(tiles, p.tiles_per_split);
}

static DecPlan dec_plan(int dtype, int64_t nb, int64_t N, int64_t D) {
  DecPlan p{};
  if (dtype == HVAE_FP8) {  // k_dec_fp8: 128 users per block (64 with the D split), 64-item tiles
    p.ds = D > 384 ? 2 : 1;
    p.upb = 128 / p.ds;
    const int64_t nub = cdiv(nb, p.upb), tiles = cdiv(N, kF8TI);
    int64_t s = cdiv(256, std::max<int64_t>(1, nub));  // nb = 0: a workspace query
    s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / 2));
    s = std::min<int64_t>(s, std::max<int64_t>(1, N / std::max<int64_t>(1, 2 * nb)));
    if (s >= 8) s = s / 8 * 8;
    if (dec_forced_splits() > 0) s = dec_forced_splits();
    dec_set_splits(p, tiles, s);
    if (p.splits >= 8 && p.splits % 8 && dec_forced_splits() <= 0) dec_set_splits(p, tiles, (int64_t)p.splits / 8 * 8);
    p.blocks = nub * p.splits;
    return p;
  }
  const bool bf = dtype == HVAE_BF16;
  p.v2 = bf && !dec_use_v1() && v2_supported(D);
  p.v3 = p.v2 && v3_supported(D);
  p.v4 = (p.v3 && v4_supported(D)) || (p.v2 && v4_384(D, nb));
  p.v5 = p.v4 && v5_supported(D);  // same users per block (64), splits and partial layout as version 4
#if HVAE_AB  // HVAE_DEC_V6=1: version 6 (ab/hvae_decoder6.hip, 96 users per E tile) above 64 users
  p.v6 = p.v5 && D == 768 && env_int("HVAE_DEC_V6", 0) != 0 && dec6_plan(nb, N, p.p6);
#else
  p.v6 = 0;
#endif
  p.ds = p.v2 && (D > 384 || nb <= 64) ? 2 : 1;
  if (p.v2 && D <= 384 && (dec_forced_ds() == 1 || dec_forced_ds() == 2)) p.ds = dec_forced_ds();
  p.nw = p.v2 && p.ds == 2 && nb > 64 && D <= 384 ? 8 : 4;
  if (p.v2 && p.ds == 2 && D <= 384 && (dec_forced_nw() == 4 || dec_forced_nw() == 8)) p.nw = dec_forced_nw();
  p.upb = bf ? (p.v4 && D == 384 ? 128 : (p.v3 || p.v5) ? 64 : p.v2 ? 32 * p.nw / p.ds : kBfUsersPerBlock)
             : kF32UsersPerBlock;
  const int64_t ti = bf ? kBfTI : kF32TI;
  const int64_t target = bf ? 256 : 512;
  const int64_t nub = cdiv(nb, p.upb), tiles = cdiv(N, ti);
  int64_t s = cdiv(target, std::max<int64_t>(1, nub));
  s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / 2));
  // each split writes nb (D + 2) floats of partials: keep them below ~2x the E bytes it streams
  s = std::min<int64_t>(s, std::max<int64_t>(1, (bf ? N : 2 * N) / std::max<int64_t>(1, 2 * nb)));
  if (s >= 8) s = s / 8 * 8;
  if (dec_forced_splits() > 0) s = dec_forced_splits();
  dec_set_splits(p, tiles, s);
  if (p.splits >= 8 && p.splits % 8 && dec_forced_splits() <= 0) {  // keep "split shares an XCD" when possible
    const int64_t s8 = (int64_t)p.splits / 8 * 8;
    dec_set_splits(p, tiles, s8);
  }
  p.blocks = nub * p.splits;
  p.lds = 0;
  return p;
}

// workspace: flags [splits * nb] | partials (m, l, O) [splits * nb * (D + 2)] (splits > 1) | O scratch [nb * D]
static size_t dec_flag_bytes(int splits, int64_t nb) {
  return (size_t)cdiv((int64_t)splits * nb * sizeof(int), 256) * 256;
}
static size_t dec_ws_bytes(int splits, int64_t nb, int64_t D) {
  return dec_flag_bytes(splits, nb) + (splits > 1 ? (size_t)splits * nb * (D + 2) * sizeof(float) : 0) +
         (size_t)nb * D * sizeof(float);
}


template <int D, int DS, int NW, bool WO>
static int launch_bf16_v2_nw(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                             const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int lds = d2_lds_bytes<D, DS, NW>();
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec2_bf16<D, DS, NW, WO>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  k_dec2_bf16<D, DS, NW, WO><<<(unsigned)p.blocks, 64 * NW, lds, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N,
                                                                       p.splits, p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec2_bf16");
  return HVAE_OK;
}

template <int D, int DS, bool WO>
static int launch_bf16_v2(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                          const DecPlan& p, DecOut o, hipStream_t st) {
  if constexpr (DS == 2 && d2_stages<D, 2, 8>() >= 3) {
    if (p.nw == 8) return launch_bf16_v2_nw<D, 2, 8, WO>(U, ldu, E, enorm, nb, N, p, o, st);
  }
  return launch_bf16_v2_nw<D, DS, 4, WO>(U, ldu, E, enorm, nb, N, p, o, st);
}



template <int D, bool WO>
static int launch_fp8(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                      const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int DS = D > 384 ? 2 : 1;
  constexpr int lds = f8_stages<D>() * f8_tile_bytes<D>() + f8_xbytes<D>();
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec_fp8<D, DS, WO>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  const unsigned char* T8 = (const unsigned char*)E + f8_offset_bytes(N, D);
  const int* ke = (const int*)((const char*)E + f8_tail_offset(N, D));
  k_dec_fp8<D, DS, WO><<<(unsigned)p.blocks, 256, lds, st>>>(U, ldu, T8, ke, enorm, nb, N, p.splits, p.tiles_per_split,
                                                            o);
  HVAE_LAUNCH_CHECK("k_dec_fp8");
  return HVAE_OK;
}


template <int D, bool WO>
static int launch_f32(const float* U, int64_t ldu, const void* E, int64_t nb, int64_t N, const DecPlan& p,
                      DecOut o, hipStream_t st) {
  constexpr int lds = 2 * f32_tile_bytes<D>();
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec_f32<D, WO>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  k_dec_f32<D, WO><<<(unsigned)p.blocks, 256, lds, st>>>(U, ldu, (const float*)E, nb, N, p.splits,
                                                        p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec_f32");
  return HVAE_OK;
}

template <bool WO>
static int dispatch(int dtype, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb,
                    int64_t N, int64_t D, const DecPlan& p, DecOut o, hipStream_t st) {
  if (dtype == HVAE_FP8) {
    switch (D) {
      case 128: return launch_fp8<128, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 256: return launch_fp8<256, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 384: return launch_fp8<384, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 768:
#if HVAE_AB  // HVAE_DEC_F8V4=1 runs the version-4 structure, HVAE_DEC_F8V5=0 the D-split ring
        if (env_int("HVAE_DEC_F8V4", 0) != 0) return ab_dec_f8v4(WO, U, ldu, E, enorm, nb, N, p, o, st);
        if (env_int("HVAE_DEC_F8V5", 1) == 0) return launch_fp8<768, WO>(U, ldu, E, enorm, nb, N, p, o, st);
#endif
        return dec5_f8_launch(WO, U, ldu, (const unsigned char*)E + f8_offset_bytes(N, 768),
                              (const int*)((const char*)E + f8_tail_offset(N, 768)), enorm, nb, N, p.splits,
                              p.tiles_per_split, p.blocks, o.flag, o.m, o.l, o.O, o.lse, o.direct, st);
      default: break;
    }
#if HVAE_AB
  } else if (dtype == HVAE_BF16 && p.v2 && p.ds == 1 && !p.v4 && D == 384 && v5w_supported(D)) {
    return dec5w_launch(WO, U, ldu, E, enorm, nb, N, p.splits, p.tiles_per_split, p.blocks, o.flag, o.m, o.l, o.O,
                        o.lse, o.direct, st);
#endif
  } else if (dtype == HVAE_BF16 && p.v5 && D == 768) {
    return dec5_launch(WO, U, ldu, E, enorm, nb, N, p.splits, p.tiles_per_split, p.blocks, o.flag, o.m, o.l, o.O,
                       o.lse, o.direct, st);
#if HVAE_AB
  } else if (dtype == HVAE_BF16 && p.v4 && D == 768) {
    return ab_dec_v4(WO, 768, U, ldu, E, enorm, nb, N, p, o, st);
  } else if (dtype == HVAE_BF16 && p.v4 && D == 384) {
    return ab_dec_v4(WO, 384, U, ldu, E, enorm, nb, N, p, o, st);
  } else if (dtype == HVAE_BF16 && p.v3 && D == 768) {
    return ab_dec_v3(WO, U, ldu, E, enorm, nb, N, p, o, st);
#endif
  } else if (dtype == HVAE_BF16 && p.v2) {
    if (p.ds == 1) {
      switch (D) {
        case 64: return launch_bf16_v2<64, 1, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 128: return launch_bf16_v2<128, 1, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 256: return launch_bf16_v2<256, 1, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 384: return launch_bf16_v2<384, 1, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        default: break;
      }
    } else {
      switch (D) {
        case 64: return launch_bf16_v2<64, 2, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 128: return launch_bf16_v2<128, 2, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 256: return launch_bf16_v2<256, 2, WO>(U, ldu, E, enorm, nb, N, p, o, st);
        case 384: return launch_bf16_v2<384, 2, WO>(U, ldu, E, enorm, nb, N, p, o, st);
#if HVAE_AB
        case 768: return launch_bf16_v2<768, 2, WO>(U, ldu, E, enorm, nb, N, p, o, st);
#endif
        default: break;
      }
    }
#if HVAE_AB
  } else if (dtype == HVAE_BF16) {
    if (D == 64 || D == 128 || D == 256 || D == 384) return ab_dec_v1(WO, (int)D, U, ldu, E, enorm, nb, N, p, o, st);
#endif
  } else if (dtype != HVAE_BF16) {
    switch (D) {
      case 32: return launch_f32<32, WO>(U, ldu, E, nb, N, p, o, st);
      case 64: return launch_f32<64, WO>(U, ldu, E, nb, N, p, o, st);
      case 128: return launch_f32<128, WO>(U, ldu, E, nb, N, p, o, st);
      case 256: return launch_f32<256, WO>(U, ldu, E, nb, N, p, o, st);
      case 384: return launch_f32<384, WO>(U, ldu, E, nb, N, p, o, st);
      default: break;
    }
  }
  HVAE_FAIL(HVAE_ERR_UNSUPPORTED, "hvae_decoder_fwd: no %s kernel for D=%lld",
            dtype == HVAE_FP8 ? "fp8" : dtype == HVAE_BF16 ? "bf16" : "f32", (long long)D);
}

}  // namespace hvae

using namespace hvae;


extern "C" int hvae_decoder_supported(int dtype, int64_t D) {
  if (dtype == HVAE_BF16) return D == 64 || D == 128 || D == 256 || D == 384 || (D == 768 && !dec_use_v1());
  if (dtype == HVAE_F32) return D == 32 || D == 64 || D == 128 || D == 256 || D == 384;
  if (dtype == HVAE_FP8) return D == 128 || D == 256 || D == 384 || D == 768;
  return 0;
}

extern "C" int hvae_row_norm_max(int dtype, const void* E, int64_t N, int64_t D, float* out, void* stream) {
  HVAE_REQUIRE(E && out && N > 0 && D > 0 && (dtype == HVAE_F32 || dtype == HVAE_BF16),
               "hvae_row_norm_max: bad args");
  hipStream_t st = as_stream(stream);
  HVAE_HIP(hipMemsetAsync(out, 0, sizeof(float), st));
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(N, 4), 1024);
  k_row_norm_max<<<grid, 256, 0, st>>>(dtype, E, N, D, (unsigned*)out);
  HVAE_LAUNCH_CHECK("k_row_norm_max");
  return HVAE_OK;
}

extern "C" size_t hvae_decoder_image_bytes(int dtype, int64_t N, int64_t D) {
  if (dtype == HVAE_F32) return (size_t)N * D * sizeof(float);
  if (dtype == HVAE_FP8) return (size_t)f8_tail_offset(N, D) + 256;
  return (size_t)et_offset_bytes(N, D) + (size_t)cdiv(N, kBfTI) * D * kBfTI * sizeof(bf16_t);
}

extern "C" int hvae_decoder_image(int dtype, const float* E32, int64_t N, int64_t D, void* out, void* stream) {
  HVAE_REQUIRE(E32 && out && N > 0 && D > 0, "hvae_decoder_image: bad args");
  HVAE_REQUIRE(dtype == HVAE_BF16 || dtype == HVAE_F32 || dtype == HVAE_FP8, "hvae_decoder_image: bad dtype");
  hipStream_t st = as_stream(stream);
  if (dtype == HVAE_FP8) {
    HVAE_REQUIRE((D == 128 || D == 256 || D == 384 || D == 768) && N * D * 2 < (1ll << 31),
                 "hvae_decoder_image: fp8 needs D in {128, 256, 384, 768} and N D < 2^30");
    const int64_t ntiles = cdiv(N, kF8TI);
    unsigned* amax = (unsigned*)((char*)out + f8_tail_offset(N, D) + 128);  // scratch word of the tail
    HVAE_HIP(hipMemsetAsync(amax, 0, sizeof(unsigned), st));
    k_abs_max<<<(unsigned)std::min<int64_t>(cdiv(N * D, 256), 4096), 256, 0, st>>>(E32, N * D, amax);
    HVAE_LAUNCH_CHECK("k_abs_max");
    k_build_image<<<(unsigned)std::min<int64_t>(cdiv(N * D, 256), 8192), 256, 0, st>>>(E32, N, D, (bf16_t*)out,
                                                                                      nullptr, 0);
    HVAE_LAUNCH_CHECK("k_build_image");
    k_build_f8<<<(unsigned)std::min<int64_t>(cdiv(ntiles * 16 * D, 256), 8192), 256, 0, st>>>(
        E32, N, D, ntiles, amax, (unsigned char*)out + f8_offset_bytes(N, D), (int*)((char*)out + f8_tail_offset(N, D)));
    HVAE_LAUNCH_CHECK("k_build_f8");
    return HVAE_OK;
  }
  if (dtype == HVAE_F32) {
    HVAE_HIP(hipMemcpyAsync(out, E32, (size_t)N * D * sizeof(float), hipMemcpyDeviceToDevice, st));
    return HVAE_OK;
  }
  const int64_t ntiles = cdiv(N, kBfTI);
  bf16_t* Ebf = (bf16_t*)out;
  bf16_t* Et = (bf16_t*)((char*)out + et_offset_bytes(N, D));
  const unsigned grid = (unsigned)std::min<int64_t>(cdiv(ntiles * D * kBfTI, 256), 8192);
  k_build_image<<<grid, 256, 0, st>>>(E32, N, D, Ebf, Et, ntiles);
  HVAE_LAUNCH_CHECK("k_build_image");
  return HVAE_OK;
}

// version 6: flags | m | l | O over the slot rows [p6.slots][96], then the O scratch of the other layouts (the
// workspace also fits version 5's, the fallback when a caller's workspace is short)
static size_t dec6_ws_bytes(const Dec6Plan& q, int64_t nb, int64_t D) {
  const size_t rows = (size_t)q.slots * kDec6Users;
  return (size_t)cdiv((int64_t)(rows * sizeof(int)), 256) * 256 + rows * (2 + (size_t)D) * sizeof(float) +
         (size_t)nb * D * sizeof(float);
}
static size_t plan_ws_bytes(const DecPlan& p, int64_t nb, int64_t D) {
  const size_t base = dec_ws_bytes(p.splits, nb, D);
  return p.v6 ? std::max(base, dec6_ws_bytes(p.p6, nb, D)) : base;
}

extern "C" int64_t hvae_decoder_users_per_tile(int dtype, int64_t nb, int64_t N, int64_t D) {
  if (nb <= 0 || N <= 0 || D <= 0) return 0;
  const DecPlan p = dec_plan(dtype, nb, N, D);
  return p.v6 ? kDec6Users : std::min<int64_t>(p.upb, nb);
}

extern "C" size_t hvae_decoder_workspace(int dtype, int64_t nb, int64_t N, int64_t D) {
  const DecPlan p = dec_plan(dtype, nb, N, D);
  return plan_ws_bytes(p, nb, D);
}

static int decoder_finalize(FinArgs& a, const float* U, int64_t ldu, const void* E, const float* E32,
                            const hvae_csr_batch* x, int64_t nb, int64_t N, int64_t D, float scale, float* lse,
                            float* recon_rows, float* dU, const float* kl_rows, float beta, const float* beta_dev,
                            float* loss3, double* accum3, bool grouped, hipStream_t st);

// the finalize's 16-B column form: every row operand it reads or writes starts 16-B aligned
static bool fin_v4(const FinArgs& a) {
  auto al = [](const void* p) { return ((uintptr_t)p % 16) == 0; };
  return a.D % 4 == 0 && a.ldu % 4 == 0 && al(a.U) && al(a.pO) && al(a.O_in) && al(a.O_out) && al(a.E32) && al(a.dU);
}

// flash sweep + finalize; csr / recon_rows / dU optional
static int decoder_run(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                       const float* E32, const hvae_csr_batch* x, int64_t nb, int64_t N, int64_t D, float scale,
                       float* lse, float* O, float* recon_rows, float* dU, const float* kl_rows, float beta,
                       const float* beta_dev, float* loss3, double* accum3, void* ws, size_t ws_bytes,
                       hipStream_t st) {
  HVAE_REQUIRE(dtype == HVAE_BF16 || dtype == HVAE_F32 || dtype == HVAE_FP8, "hvae decoder: bad dtype");
  HVAE_REQUIRE(U && E && lse && N > 0 && D > 0 && ldu >= D, "hvae decoder: bad args");
  HVAE_REQUIRE(dtype == HVAE_F32 || e_maxnorm, "hvae decoder: bf16 / fp8 need e_maxnorm");
  HVAE_REQUIRE(D <= 1024, "hvae decoder: D > 1024 unsupported");
  HVAE_REQUIRE(ldu % 4 == 0 && ((uintptr_t)U % 16) == 0 && ((uintptr_t)E % 16) == 0 &&
                   (!O || ((uintptr_t)O % 16) == 0),
               "hvae decoder: U/E/O must be 16-B aligned with ldu %% 4 == 0");
  HVAE_REQUIRE(N < (1ll << 31), "hvae decoder: N too large");
  HVAE_REQUIRE(dtype == HVAE_F32 || N * D * 2 < (1ll << 31), "hvae decoder: bf16 / fp8 E image over 2 GiB");
  HVAE_REQUIRE(!x || (E32 && x->row_ptr && x->nb == nb && x->n_items == N), "hvae decoder: bad CSR batch");
  if (nb == 0) return HVAE_OK;
  DecPlan p = dec_plan(dtype, nb, N, D);
  if (!ws || ws_bytes < dec_ws_bytes(1, nb, D))
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae decoder: workspace %zu < %zu", ws_bytes, dec_ws_bytes(1, nb, D));
  if (p.splits > 1 && ws_bytes < dec_ws_bytes(p.splits, nb, D)) {  // fewer splits that fit
    int64_t fit = p.splits;
    while (fit > 1 && ws_bytes < dec_ws_bytes((int)fit, nb, D)) fit = fit * 3 / 4;
    const int64_t tiles = cdiv(N, dtype == HVAE_FP8 ? kF8TI : dtype == HVAE_BF16 ? kBfTI : kF32TI);
    dec_set_splits(p, tiles, fit);
    p.blocks = cdiv(nb, p.upb) * p.splits;
  }
  const bool bf = dtype != HVAE_F32;  // fixed-offset sweeps (bf16, fp8): flags, bf16 E for the exact fixup
  const bool want_o = O || dU;
  FinArgs a{};
#if HVAE_AB
  if (p.v6 && ws_bytes < dec6_ws_bytes(p.p6, nb, D)) p.v6 = 0;
  if (p.v6) {  // version 6: slot-row partials, merged per user by the finalize's slot map
    const Dec6Plan& q = p.p6;
    const size_t rows = (size_t)q.slots * kDec6Users;
    char* w6 = (char*)ws;
    int* flag6 = (int*)w6;
    w6 += (size_t)cdiv((int64_t)(rows * sizeof(int)), 256) * 256;
    float* pm = (float*)w6;
    float* pl = pm + rows;
    float* pO = pl + rows;
    int rc;
    {
      ProbeScope probe("decoder_sweep", st);
      rc = dec6_launch(want_o, U, ldu, E, e_maxnorm, nb, N, q, flag6, pm, pl, want_o ? pO : nullptr, st);
    }
    if (rc) return rc;
    a.splits = q.S;
    a.pm = pm; a.pl = pl; a.pO = want_o ? pO : nullptr;
    a.flag = flag6;
    a.v6_upb = kDec6Users; a.v6_nub = q.nub; a.v6_S = q.S; a.v6_main = q.main; a.v6_P = q.P;
    a.O_out = O;
    return decoder_finalize(a, U, ldu, E, E32, x, nb, N, D, scale, lse, recon_rows, dU, kl_rows, beta, beta_dev,
                            loss3, accum3, q.X > 0 || q.S > 8, st);
  }
#endif
  char* w = (char*)ws;
  DecOut o{};
  o.flag = (int*)w;
  w += dec_flag_bytes(p.splits, nb);
  float* o_scratch = nullptr;
  if (p.splits == 1) {
    o.direct = 1;
    o.lse = lse;
    o.O = O ? O : (want_o ? (float*)w : nullptr);
    o_scratch = o.O;
  } else {
    float* base = (float*)w;
    o.direct = 0;
    o.m = base;
    o.l = base + (size_t)p.splits * nb;
    o.O = base + (size_t)2 * p.splits * nb;
  }
  int rc;
  {
    ProbeScope probe("decoder_sweep", st);
    rc = want_o ? dispatch<true>(dtype, U, ldu, E, e_maxnorm, nb, N, D, p, o, st)
                  : dispatch<false>(dtype, U, ldu, E, e_maxnorm, nb, N, D, p, o, st);
  }
  if (rc) return rc;
  if (p.splits == 1 && !bf && !x) return HVAE_OK;  // fp32 single split: the sweep wrote lse / O already
  a.splits = p.splits;
  if (p.splits > 1) { a.pm = o.m; a.pl = o.l; a.pO = want_o ? o.O : nullptr; }
  else { a.lse_in = lse; a.O_in = o_scratch; }
  a.flag = bf ? o.flag : nullptr;
  a.O_out = O ? O : (p.splits == 1 ? o_scratch : nullptr);
  return decoder_finalize(a, U, ldu, E, E32, x, nb, N, D, scale, lse, recon_rows, dU, kl_rows, beta, beta_dev, loss3,
                          accum3, p.splits > 8, st);
}

// the finalize launch of decoder_run (a's partial / direct inputs and O_out set by the caller)
static int decoder_finalize(FinArgs& a, const float* U, int64_t ldu, const void* E, const float* E32,
                            const hvae_csr_batch* x, int64_t nb, int64_t N, int64_t D, float scale, float* lse,
                            float* recon_rows, float* dU, const float* kl_rows, float beta, const float* beta_dev,
                            float* loss3, double* accum3, bool grouped, hipStream_t st) {
  HVAE_REQUIRE(!loss3 || x, "hvae decoder: fused loss needs the batch");
  a.U = U; a.ldu = ldu; a.Ebf = (const bf16_t*)E;
  a.E32 = E32; a.N = N; a.D = D; a.nb = nb;
  if (x) {
    a.row_ptr = x->row_ptr; a.col_idx = x->col_idx; a.vals = x->vals; a.rows = x->rows;
    a.rows_offset = x->rows_offset;
  }
  a.scale = scale;
  a.lse_out = lse;
  a.recon_rows = recon_rows;
  a.dU = dU;
  if (loss3) {
    HVAE_REQUIRE(x && recon_rows && kl_rows, "hvae_decoder_train: fused loss needs recon_rows and kl_rows");
    a.kl_rows = kl_rows; a.beta = beta; a.beta_dev = beta_dev; a.loss3 = loss3; a.accum3 = accum3;
    if (!(a.ticket = ticket_slice())) return HVAE_ERR_HIP;
  }
  ProbeScope probe("decoder_finalize", st);
  const bool v4 = fin_v4(a);
  if (grouped) {
    if (v4) k_dec_finalize<true, true><<<(unsigned)nb, 256, 0, st>>>(a);
    else k_dec_finalize<true, false><<<(unsigned)nb, 256, 0, st>>>(a);
  } else {
    if (v4) k_dec_finalize<false, true><<<(unsigned)nb, 256, 0, st>>>(a);
    else k_dec_finalize<false, false><<<(unsigned)nb, 256, 0, st>>>(a);
  }
  HVAE_LAUNCH_CHECK("k_dec_finalize");
  return HVAE_OK;
}

extern "C" int hvae_decoder_fwd(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                                int64_t nb, int64_t N, int64_t D, float* lse, float* O, void* ws,
                                size_t ws_bytes, void* stream) {
  return decoder_run(dtype, U, ldu, E, e_maxnorm, nullptr, nullptr, nb, N, D, 0.f, lse, O, nullptr, nullptr,
                     nullptr, 0.f, nullptr, nullptr, nullptr, ws, ws_bytes, as_stream(stream));
}

extern "C" int hvae_decoder_train(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                                  const float* E32, const hvae_csr_batch* x, int64_t D, float grad_scale,
                                  float* lse, float* O, float* recon_rows, float* dU, const float* kl_rows,
                                  float beta, const float* beta_dev, float* loss3, double* accum3, void* ws,
                                  size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(x && recon_rows, "hvae_decoder_train: needs the CSR batch and recon_rows");
  return decoder_run(dtype, U, ldu, E, e_maxnorm, E32, x, x->nb, x->n_items, D, grad_scale, lse, O, recon_rows, dU,
                     kl_rows, beta, beta_dev, loss3, accum3, ws, ws_bytes, as_stream(stream));
}

extern "C" int hvae_decoder_bwd(const hvae_csr_batch* x, const float* U, int64_t ldu, const float* E32,
                                int64_t D, const float* lse, const float* O, float grad_scale,
                                float* recon_rows, float* dU, void* stream) {
  HVAE_REQUIRE(x && x->row_ptr && U && E32 && lse && recon_rows && D > 0 && D <= 1024 && ldu >= D,
               "hvae_decoder_bwd: bad args");
  HVAE_REQUIRE(!dU || O, "hvae_decoder_bwd: dU needs O");
  if (x->nb == 0) return HVAE_OK;
  FinArgs a{};
  a.splits = 1;
  a.lse_in = lse;
  a.O_in = O;
  a.U = U; a.ldu = ldu;
  a.E32 = E32; a.N = x->n_items; a.D = D; a.nb = x->nb;
  a.row_ptr = x->row_ptr; a.col_idx = x->col_idx; a.vals = x->vals; a.rows = x->rows;
  a.rows_offset = x->rows_offset;
  a.scale = grad_scale;
  a.lse_out = const_cast<float*>(lse);  // rewritten with the same value
  a.recon_rows = recon_rows;
  a.dU = dU;
  if (fin_v4(a)) k_dec_finalize<false, true><<<(unsigned)x->nb, 256, 0, as_stream(stream)>>>(a);
  else k_dec_finalize<false, false><<<(unsigned)x->nb, 256, 0, as_stream(stream)>>>(a);
  HVAE_LAUNCH_CHECK("k_dec_finalize");
  return HVAE_OK;
}
