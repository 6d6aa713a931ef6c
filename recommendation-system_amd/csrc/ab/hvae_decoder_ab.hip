// hvae_decoder_ab.hip -- the retired decoder sweeps, compiled only into the A/B library (make lib-ab ->
// build_var/libhvae_ab.so; never libhvae.so). hvae_decoder.hip's plan selects them from the environment
// (HVAE_DEC_V1 / V3 / V4 / V4_384 / F8V4) in that build; tests/ab_checks.py keeps their parity checks.
//   * version 1 (k_dec_bf16): the transposed-copy sweep, D <= 384;
//   * version 3 (k_dec3_bf16) and version 4 (k_dec4_bf16): the D = 768 sweeps version 5 replaced (4 also at 384);
//   * k_dec4_f8: the fp8 sweep with version 4's structure (it tied with the D-split ring).
// DESIGN.md 4.1 records the measurements that retired each.
#if !HVAE_AB
#error "hvae_decoder_ab.hip is part of the A/B library only (make lib-ab)"
#endif
#include <algorithm>
#include <array>
#include <type_traits>

#include "../hvae_common.h"
#include "../hvae_dec_shared.h"

namespace hvae {

template <int D, bool WITH_O>
__global__ void __launch_bounds__(256) k_dec_bf16(const float* __restrict__ U, int64_t ldu,
                                                  const bf16_t* __restrict__ E, const bf16_t* __restrict__ Et,
                                                  const float* __restrict__ e_maxnorm, int64_t nb,
                                                  int64_t N, int splits, int64_t tiles_per_split,
                                                  DecOut out) {
  static_assert(D % 32 == 0, "D must be a multiple of 32");
  constexpr int KS = D / 16;              // GEMM1 k-steps (even)
  constexpr int DB = D / 32;              // GEMM2 d-blocks
  constexpr int CH = D / 8;               // 16-B chunks per row
  constexpr int NSEG = (D + 127) / 128;
  constexpr int TB = bf_tile_bytes<D>();  // NSEG * 8 KiB
  constexpr int PIECES_E = NSEG * 2;          // 1-KiB LDS-DMA pieces per wave per E tile
  constexpr int PIECES_T = D / 64;            // ... per Et tile (D * 64 B over 4 waves)
  constexpr int PIECES_PER_WAVE = PIECES_E + PIECES_T;
  constexpr int TBT = bf_ttile_bytes<D>();
  constexpr int SB = TB + TBT;                // one ring stage: E tile | Et tile
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, col = lane & 31;
  const int split = blockIdx.x % splits;
  const int64_t ub = blockIdx.x / splits;
  const int64_t u0 = ub * kBfUsersPerBlock + w * kBfUsersPerWave;
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kBfTI - 1) / kBfTI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);

  // U fragments (B operand of GEMM1): lane holds U[user][16 ks + 8 h + j],
  // packed bf16 pairs (4 VGPRs per k-step).
  uint4 uf[KS];
  float usq = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (user < nb) {
      a = *reinterpret_cast<const float4*>(U + user * ldu + 16 * ks + 8 * h);
      b = *reinterpret_cast<const float4*>(U + user * ldu + 16 * ks + 8 * h + 4);
    }
    usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
    uf[ks] = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y),
                        pack_bf16x2(b.z, b.w));
  }
  usq += __shfl_xor(usq, 32, 64);
  // Upper bound of every score of this user (bf16 rounding margin included).
  const float bound = sqrtf(usq) * (*e_maxnorm) * 1.02f;

  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m = -INFINITY, lsum = 0.f, mtrue = -INFINITY;

  // E tile -> LDS by LDS-DMA (global_load_lds_dwordx4). The destination of a
  // wave-instruction is 1 KiB contiguous (base + 16 lane), so the XOR swizzle
  // is applied to the per-lane SOURCE: LDS slot -> (row, chunk) -> E address.
  // Tail rows (item >= N) re-read row N-1; their scores are masked to -inf.
  auto issue_tile = [&](int64_t t, unsigned char* buf) {
#pragma unroll
    for (int i = 0; i < PIECES_E; ++i) {
      const int piece = w * PIECES_E + i;
      const int o_b = piece * 1024 + lane * 16;  // byte offset in the tile image
      const int seg = o_b >> 13, row = (o_b >> 8) & 31, slot = (o_b >> 4) & 15;
      const int gc = seg * 16 + (slot ^ bf_swz(row));
      int64_t item = t * kBfTI + row;
      item = item < N ? item : N - 1;
      const bf16_t* src = E + item * D + (gc < CH ? gc : 0) * 8;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(buf + piece * 1024),
                                       16, 0, 0);
    }
    // Et tile: row d = 64 B = 4 chunks, physical chunk = logical ^ ((d >> 1) & 3) (8 lanes of a
    // ds_read_b128 phase then cover all 32 banks)
    const bf16_t* et = Et + t * (int64_t)D * kBfTI;
#pragma unroll
    for (int i = 0; i < PIECES_T; ++i) {
      const int piece = w * PIECES_T + i;
      const int o_b = piece * 1024 + lane * 16;
      const int d = o_b >> 6, pc = (o_b >> 4) & 3;
      const bf16_t* src = et + d * kBfTI + ((pc ^ ((d >> 1) & 3)) * 8);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(buf + TB + piece * 1024),
                                       16, 0, 0);
    }
  };

  // NS-deep ring: tiles t+1 .. t+NS-1 are in flight while tile t is consumed. One
  // barrier per tile: after it, tile t has landed for every wave (each waited for its
  // own LDS-DMA pieces with vmcnt) and every wave is done with tile t-1, whose slot
  // then takes tile t+NS-1.
  // Past the end of the range the ring re-reads the last tile into the free slot, so
  // that exactly NS-2 younger tiles are always in flight and the wait is one constant.
  constexpr int NS = bf_stages<D>();
  if (t_beg < t_end) {
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) issue_tile(min(t_beg + i, t_end - 1), lds + i * SB);
  }
  int cur = 0;
  for (int64_t t = t_beg; t < t_end; ++t) {
    wait_vmcnt<(NS - 2) * PIECES_PER_WAVE>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue_tile(min(t + NS - 1, t_end - 1), lds + (cur == 0 ? NS - 1 : cur - 1) * SB);
    const unsigned char* buf = lds + cur * SB;
    const unsigned char* bufT = buf + TB;
    if (wave_active) {
      // ---- GEMM1: S^T[32 items][32 users] = E_tile U^T, A reads one group ahead
      f32x16 s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
      auto rdA = [&](int ks) {
        return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(buf + bf_off(col, 2 * ks + h)));
      };
      bf16x8 an0 = rdA(0), an1 = rdA(1);
#pragma unroll
      for (int g = 0; g < KS / 2; ++g) {
        const bf16x8 ac0 = an0, ac1 = an1;
        if (g + 1 < KS / 2) { an0 = rdA(2 * g + 2); an1 = rdA(2 * g + 3); }
        __builtin_amdgcn_sched_barrier(0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac0, __builtin_bit_cast(bf16x8, uf[2 * g]), s, 0, 0, 0);
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac1, __builtin_bit_cast(bf16x8, uf[2 * g + 1]), s, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- mask the tail, online softmax with deferred rescale
      const int64_t ib = t * kBfTI + 4 * h;
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t item = ib + (r & 3) + 8 * (r >> 2);
        if (item >= N) s[r] = -INFINITY;
        mx = fmaxf(mx, s[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // Fixed per-user offset, set once: m >= bound - kOffsetSpan means every
      // later p = exp(s - m) <= e^kOffsetSpan (no overflow, so no rescale of
      // the AGPR-resident O accumulator is ever needed); m >= first-tile max
      // keeps the large terms normal. mtrue tracks the real max for the
      // underflow check done at the end (fixed up by k_dec_fixup).
      if (t == t_beg) m = fmaxf(mx, bound - kOffsetSpan);
      mtrue = fmaxf(mtrue, mx);
      float pv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        pv[r] = __expf(s[r] - m);
        lsum += pv[r];
      }
      bf16x8 pf[2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        pf[s2] = __builtin_bit_cast(bf16x8, make_uint4(pack_bf16x2(pv[8 * s2 + 0], pv[8 * s2 + 1]),
                                                       pack_bf16x2(pv[8 * s2 + 2], pv[8 * s2 + 3]),
                                                       pack_bf16x2(pv[8 * s2 + 4], pv[8 * s2 + 5]),
                                                       pack_bf16x2(pv[8 * s2 + 6], pv[8 * s2 + 7])));
      if (WITH_O) {
        // ---- GEMM2: O^T[D][32 users] += Et_tile P^T: lane (h, m) reads row d = 32 db + m,
        // logical chunk 2 s2 + h (the 8 items of k-block s2 it supplies), one ds_read_b128
        const int mrow = lane & 31;
        auto rdE = [&](int db, int s2) {
          const int d = 32 * db + mrow;
          return __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(bufT + d * 64 + (((2 * s2 + h) ^ ((d >> 1) & 3)) << 4)));
        };
        bf16x8 e0 = rdE(0, 0), e1 = rdE(0, 1);
#pragma unroll
        for (int db = 0; db < (WITH_O ? DB : 1); ++db) {
          const bf16x8 c0 = e0, c1 = e1;
          if (db + 1 < DB) { e0 = rdE(db + 1, 0); e1 = rdE(db + 1, 1); }
          __builtin_amdgcn_sched_barrier(0);
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, pf[0], o[db], 0, 0, 0);
          o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, pf[1], o[db], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    cur = cur == NS - 1 ? 0 : cur + 1;
  }

  if (!wave_active) return;
  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  if (user >= nb) return;
  // the max term itself may have lost precision: exact recompute (k_dec_fixup / k_dec_merge).
  // Written for every user every call, so the flags need no clearing pass.
  if (h == 0) {
    const int f = !(mtrue >= m - kUnderflowSpan && ltot > 0.f);
    out.flag[out.direct ? user : (int64_t)split * nb + user] = f;
  }
  if (out.direct) {
    const float inv = 1.0f / ltot;
    if (h == 0) out.lse[user] = m + logf(ltot);
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + user * D + dd) =
              make_float4(o[d][4 * g4] * inv, o[d][4 * g4 + 1] * inv, o[d][4 * g4 + 2] * inv, o[d][4 * g4 + 3] * inv);
        }
    }
  } else {
    const int64_t pi = (int64_t)split * nb + user;
    if (h == 0) { out.m[pi] = m; out.l[pi] = ltot; }
    if (WITH_O) {
#pragma unroll
      for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int dd = 32 * d + 8 * g4 + 4 * h;
          *reinterpret_cast<float4*>(out.O + pi * D + dd) =
              make_float4(o[d][4 * g4], o[d][4 * g4 + 1], o[d][4 * g4 + 2], o[d][4 * g4 + 3]);
        }
    }
  }
}


// ------------------------------------------------------- bf16, version 3 ---
// D = 768 (Syn-10M), the version-2 D split with the softmax owned by halves. Version 2 at D = 768 adds the
// pair's whole partial S^T tiles through LDS and both waves of a user group run the full softmax: its loop
// issues ~330 non-MFMA instructions per 48 MFMAs at one wave per SIMD, and MFMA is busy 40 % of the time
// (profiles/r02_pmc_dec2_d768.txt). Here wave (ug, dh) owns items 16 dh .. 16 dh + 15 of every tile:
//   * it sends the partner only the half of its partial S^T the partner owns (2 KiB), completes its own half
//     (8 values per lane), runs only those 8 exponentials (under GEMM1(t + 1)'s MFMAs) and sends its packed
//     P half back (1 KiB): P of the 32 items = [P half of dh = 0 | P half of dh = 1], the B operands of
//     GEMM2's two k-steps;
//   * GEMM2(t) first runs the k-step of its own P half (12 MFMAs) while the partner's half is read, then the
//     other (12 MFMAs), so no barrier is followed by an MFMA that waits on LDS.
// Two barriers per tile: A publishes tile t + 1 and the partial S^T halves of t + 1; B publishes P(t).
// The image, the LDS-DMA ring (three 48-KiB slots) and GEMM1 / GEMM2 operand reads are version 2's.
// timing ablations (A/B builds only, results invalid): 1 = no LDS-DMA / vmcnt waits in the loop,
// 2 = no barriers in the loop, 3 = both, 4 = no half-S / P exchange through LDS
#ifndef DEC3_ABL
#define DEC3_ABL 0
#endif
// where a tile's LDS-DMA pieces go: 0 = one per GEMM1 MFMA pair, 1 = one per two GEMM2 MFMAs,
// 2 = half in each
#ifndef DEC3_DMA
#define DEC3_DMA 0
#endif
// diagnostic build (DEC3_STAMPS=1): per-wave s_memtime phase sums of the main loop, read back with
// hvae_debug_dec3_stamps (never in a shipped build: the stamps' SMEM waits perturb the schedule)
#ifndef DEC3_STAMPS
#define DEC3_STAMPS 0
#endif
#if DEC3_STAMPS
__device__ unsigned long long g_dec3_stamps[4096][8];
#define DEC3_STAMP(i)                                         \
  do {                                                        \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    st_acc[i] += n_ - st_prev;                                \
    st_prev = n_;                                             \
  } while (0)
#else
#define DEC3_STAMP(i) do {} while (0)
#endif
#ifndef DEC3_DMA_PRE
#define DEC3_DMA_PRE 0  // (DEC3_DMA 0) pieces issued before GEMM1's first MFMA (0, 3, 6 = 11.07, 11.13, 11.19 ms)
#endif
#ifndef DEC3_G1_AHEAD
#define DEC3_G1_AHEAD 2  // GEMM1 A operand k-groups (MFMA pairs) in flight
#endif
#ifndef DEC3_G2_AHEAD
#define DEC3_G2_AHEAD 2  // GEMM2 A operand d-blocks in flight
#endif
#ifndef DEC3_SM_VGPR
#define DEC3_SM_VGPR 0
#endif
// barrier B: -1 = before GEMM2(t), k = after GEMM2's own-half MFMA min(k, D / 64 - 1); at the Syn-10M shard
// (10 launches x 2 rounds, profiles/r02_dec3_bb.jsonl): -1 11.00 ms, 4 10.88, 8 10.89, last (11) 10.74
#ifndef DEC3_BB
#define DEC3_BB 99
#endif
// GEMM2(t)'s first A reads: 0 = at its start, k = in GEMM1's MFMA pair NG - k (0: 11.00 ms, 1: 10.99 alone)
#ifndef DEC3_G2PRE
#define DEC3_G2PRE 1
#endif
__host__ __device__ constexpr int d3_lds_bytes(int D) { return 3 * ((D / 128) * 8192) + 4 * 2048 + 4 * 1024; }

template <int D, bool WITH_O>
__global__ void __launch_bounds__(256) k_dec3_bf16(const float* __restrict__ U, int64_t ldu,
                                                   const bf16_t* __restrict__ E, const float* __restrict__ e_maxnorm,
                                                   int64_t nb, int64_t N, int splits, int64_t tiles_per_split,
                                                   DecOut out) {
  constexpr int DW = D / 2;             // dims owned by one wave
  constexpr int KS = DW / 16;           // GEMM1 k-steps
  constexpr int NG = KS / 2;            // GEMM1 MFMA pairs
  constexpr int DB = DW / 32;           // GEMM2 d-blocks
  constexpr int NSEG = D / 128;
  constexpr int TB = NSEG * 8192;
  constexpr int PW = NSEG * 8 / 4;      // 1-KiB LDS-DMA pieces per wave per tile
  constexpr int NS = 3;
  constexpr int BBI = DEC3_BB < 0 ? -1 : (DEC3_BB < DB ? DEC3_BB : DB - 1);
  static_assert(D % 128 == 0 && KS % 2 == 0 && NG >= 12 && PW <= NG && d3_lds_bytes(D) <= 160 * 1024,
                "k_dec3_bf16 shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  float* xs = reinterpret_cast<float*>(lds + NS * TB);                 // [4 w][2 r4][64 lane][4]: partner halves
  uint32_t* xp = reinterpret_cast<uint32_t*>(lds + NS * TB + 4 * 2048);  // [4 w][64 lane][4]: packed P halves
  float* xm = reinterpret_cast<float*>(xp);                            // [4 w][32]: max / sum exchange (aliases xp)

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ug = w & 1, dh = w >> 1, pw = w ^ 2;  // partner wave: same users, other D half
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * 64 + ug * 32;
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kBfTI - 1) / kBfTI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const int dbase = dh * DW;
  const float emax = *e_maxnorm;  // before any LDS-DMA is in flight (the compiler's wait would drain them)

  // U fragments (B operand of GEMM1): lane holds U[user][dbase + 16 ks + 8 h + j]; |u| over the whole row
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
    uf[ks] = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y), pack_bf16x2(b.z, b.w));
    __builtin_amdgcn_sched_barrier(0);  // a few k-steps' loads in flight, not all 48 (register peak)
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (user < nb) {
      const float4 a = *reinterpret_cast<const float4*>(U + user * ldu + (DW - dbase) + 16 * ks + 8 * h);
      const float4 b = *reinterpret_cast<const float4*>(U + user * ldu + (DW - dbase) + 16 * ks + 8 * h + 4);
      usq += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  usq += __shfl_xor(usq, 32, 64);
  const float bound = sqrtf(usq) * emax * 1.02f;

  // LDS-DMA into version 2's image. Piece p (1 KiB) of a tile holds rows 8 ((p >> 1) & 3) + ((lane >> 2) & 7),
  // chunk group 2 (p & 1) + (lane >> 5) of segment p >> 3; the chunk XOR (row >> 2) & 3 depends on p only
  // through bit 1, so two lane offsets serve every piece and the rest of the source offset is scalar.
  int vlane[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int row = 8 * pb + ((lane >> 2) & 7);
    vlane[pb] = ((lane >> 2) & 7) * (D * 2) + 64 * (lane >> 5) + 16 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(E), (short)0, (int)(N * D * 2), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(w * PW * 1024);
  static_assert(PW % 2 == 0, "piece parity is compile-time");
  // pieces [i0, i1) of tile t into ring slot slot_i; soff = the tile's byte offset, wave-uniform (readfirstlane).
  // fresh: soff was just produced by v_readfirstlane (5 wait states before a buffer op reads it)
  auto issue_pieces = [&](uint32_t soff, int slot_i, int i0, int i1, bool fresh) {
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int p = w * PW + i;  // wave-uniform; bits 0 and 1 of p are those of i (PW is even)
      const uint32_t so = soff + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (i & 1));
      const int vo = vlane[(i >> 1) & 1];
      if (fresh && i == i0)
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
    }
  };
  auto tile_soff = [&](int64_t t) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)(kBfTI * D * 2)));
  };
  auto issue_range = [&](int64_t t, int slot_i, int i0, int i1) { issue_pieces(tile_soff(t), slot_i, i0, i1, true); };
  auto lds_fence = [] { asm volatile("" ::: "memory"); };
  auto barrier = [&] {  // this wave's LDS writes complete, then the workgroup barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    lds_fence();
  };

  // operand addressing (version 2): GEMM1 row reads by ks parity, GEMM2 transposed reads by j
  const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  static_assert((DW / 32) % 4 == 0, "a D half starts at a 128-column segment boundary");
  const int cseg = (dbase / 128) << 13;  // the wave's first segment (uniform), so every other term is immediate
  const int laneA0 = ((col >> 3) << 11) + ((col & 7) << 6) + (((0 + h) ^ ((col >> 2) & 3)) << 4);
  const int laneA1 = ((col >> 3) << 11) + ((col & 7) << 6) + (((2 + h) ^ ((col >> 2) & 3)) << 4);
  const int laneT0 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((0 + h) & 3)) << 4) + 8 * (pp & 1);
  const int laneT1 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((2 + h) & 3)) << 4) + 8 * (pp & 1);

  // GEMM1 partial over this wave's dims: S^T[32 items][32 users] = E_tile U^T; fill(g) after MFMA pair g
  auto gemm1 = [&](const unsigned char* buf, auto&& pre, auto&& fill) {
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    const unsigned char* b0 = buf + cseg + laneA0;
    const unsigned char* b1 = buf + cseg + laneA1;
    auto rdA = [&](int ks) {
      const int grp = ks >> 1;
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(((ks & 1) ? b1 : b0) + ((grp >> 2) << 13) +
                                                                         ((grp & 3) << 9)));
    };
    constexpr int AH = DEC3_G1_AHEAD;
    bf16x8 a[2 * AH];
#pragma unroll
    for (int j = 0; j < 2 * AH; ++j) a[j] = rdA(j);
    pre();  // under the first operand reads' latency
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
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
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  // GEMM2(t) over both k-steps (items 16 kh .. 16 kh + 15), own half first: O^T[DW][32 users] += E^T P^T.
  // MFMA i (0 .. 2 DB - 1) is k-step kh(i) = i < DB ? own : partner, d-block i % DB; the transposed A reads run
  // BH MFMAs ahead across the two halves, and the first BH (g2_pre) can go out before the loop (in GEMM1's
  // last gaps). pf_own is in registers; pf_par is read from LDS in fill(i) for some i < DB.
  constexpr int BH = DEC3_G2_AHEAD;
  auto rdT = [&](const unsigned char* buf, int kown, int i) {
    const int kh = i < DB ? kown : 1 - kown, db = i % DB;
    const unsigned char* t = buf + cseg + (kh << 12);
    auto* p0 = (__attribute__((address_space(3))) s16x4*)(void*)(t + laneT0 + ((db >> 2) << 13) + ((db & 3) << 9));
    auto* p1 = (__attribute__((address_space(3))) s16x4*)(void*)(t + laneT1 + (1 << 11) + ((db >> 2) << 13) +
                                                                 ((db & 3) << 9));
    return std::array<s16x4, 2>{__builtin_amdgcn_ds_read_tr16_b64_v4i16(p0), __builtin_amdgcn_ds_read_tr16_b64_v4i16(p1)};
  };
  auto g2_pre = [&](const unsigned char* buf, int kown, std::array<s16x4, 2> (&n)[BH]) {
#pragma unroll
    for (int j = 0; j < BH; ++j) n[j] = rdT(buf, kown, j);
  };
  auto gemm2 = [&](const unsigned char* buf, int kown, std::array<s16x4, 2> (&n)[BH], const bf16x8& pf_own,
                   const uint4& pf_par,
                   auto&& fill) {
    if constexpr (WITH_O) {
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) {
        const std::array<s16x4, 2> c = n[i % BH];
        if (i + BH < 2 * DB) n[i % BH] = rdT(buf, kown, i + BH);
        const s16x8 a = {c[0][0], c[0][1], c[0][2], c[0][3], c[1][0], c[1][1], c[1][2], c[1][3]};
        const bf16x8 pf = i < DB ? pf_own : __builtin_bit_cast(bf16x8, pf_par);
        o[i % DB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), pf, o[i % DB], 0, 0, 0);
        fill(i);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) fill(i);  // the exchange and any LDS-DMA placed in GEMM2 still run
    }
  };
  // this wave's half of a partial S^T tile: rows 8 dh .. 8 dh + 7 of the accumulator (items 16 dh ..);
  // the partner's half goes to LDS as [r4][lane] float4
  // (the halves are picked by value selects on the wave-uniform dh: a runtime index into the accumulator
  // vector -- which the compiler folds such a select into -- moves it through indexed-register mode)
  auto half_of = [&](const f32x16& s, int which, int r) {
    float a = s[r], b = s[8 + r];
    asm volatile("" : "+v"(a), "+v"(b));  // opaque: keeps the select from folding into an indexed extract
    return which ? b : a;
  };
  auto put_half = [&](const f32x16& s) {
    float* dst = xs + w * 512;
#pragma unroll
    for (int r4 = 0; r4 < 2; ++r4)
      *reinterpret_cast<float4*>(dst + r4 * 256 + lane * 4) =
          make_float4(half_of(s, 1 - dh, 4 * r4), half_of(s, 1 - dh, 4 * r4 + 1), half_of(s, 1 - dh, 4 * r4 + 2),
                      half_of(s, 1 - dh, 4 * r4 + 3));
  };

  float m = 0.f, mL = 0.f, lsum = 0.f;
  float sm[8];   // this wave's half of S^T(t): own partial, completed in GEMM1(t + 1)'s first gaps
  float4 y0 = make_float4(0.f, 0.f, 0.f, 0.f), y1 = y0;
#pragma unroll
  for (int r = 0; r < 8; ++r) sm[r] = 0.f;
  f32x16 s_nx;
#pragma unroll
  for (int r = 0; r < 16; ++r) s_nx[r] = 0.f;
  if (t_beg < t_end) {
    issue_range(t_beg, 0, 0, PW);
    issue_range(min(t_beg + 1, t_end - 1), 1, 0, PW);
    wait_vmcnt<PW>();
  }
  barrier();
  if (t_beg < t_end) {
    // first tile: whole S^T half, the pair's common fixed offset m from its max (version 2's rule), then the
    // partner halves are zeroed so that the loop's completion step is the same for every tile
    s_nx = gemm1(lds, [] {}, [](int) {});
    put_half(s_nx);
    barrier();
    float mh = -INFINITY;
    {
      const float* src = xs + pw * 512;
      y0 = *reinterpret_cast<const float4*>(src + lane * 4);
      y1 = *reinterpret_cast<const float4*>(src + 256 + lane * 4);
      const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
      for (int r = 0; r < 8; ++r) sm[r] = dh == 0 ? half_of(s_nx, dh, r) + yv[r] : yv[r] + half_of(s_nx, dh, r);
      if (t_beg == ntiles - 1 && (N % kBfTI) != 0) {
        const int lim = (int)(N - t_beg * kBfTI) - 4 * h - 16 * dh;
#pragma unroll
        for (int r = 0; r < 8; ++r) sm[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : sm[r];
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) mh = fmaxf(mh, sm[r]);
      mh = fmaxf(mh, __shfl_xor(mh, 32, 64));
      if (h == 0) xm[w * 32 + col] = mh;
    }
    barrier();
    {
      m = fmaxf(fmaxf(mh, xm[pw * 32 + col]), bound - kOffsetSpan);
      mL = m * kLog2e;
      float* dst = xs + w * 512;
      *reinterpret_cast<float4*>(dst + lane * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(dst + 256 + lane * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    barrier();  // the max exchange is read (xm aliases the P buffers) and the zeroed halves are published
  }

  // the loop is instantiated per D half (dh) so that every register pick of a half is static
#if DEC3_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_prev = __builtin_amdgcn_s_memtime();
#endif
  auto sweep = [&](auto dh_c) {
  constexpr int DHC = decltype(dh_c)::value;
  int cur = 0;
  for (int64_t t = t_beg; t < t_end; ++t) {
    DEC3_STAMP(0);  // [0] end of the previous iteration -> here
#if DEC3_SM_VGPR
#pragma unroll
    for (int r = 0; r < 8; ++r) asm volatile("" : "+v"(sm[r]));  // keep the loop-carried half in VGPRs
#endif
    // [A(t)]: tile t + 1 has landed; the partner's partial half of S^T(t) is published
    if (DEC3_ABL != 1 && DEC3_ABL != 3) wait_vmcnt<0>();
    DEC3_STAMP(1);  // [1] LDS-DMA wait
    if (DEC3_ABL != 2 && DEC3_ABL != 3) barrier();
    DEC3_STAMP(2);  // [2] barrier A
    const int nxt = cur == NS - 1 ? 0 : cur + 1;
    const int64_t t_dma = min(t + 2, t_end - 1);
    const int s_dma = cur == 0 ? NS - 1 : cur - 1;
    const uint32_t soff_dma = tile_soff(t_dma);  // well before the first piece reads it
    constexpr int P1 = DEC3_DMA == 0 ? PW : DEC3_DMA == 1 ? 0 : PW / 2;  // pieces under GEMM1, the rest GEMM2
    constexpr bool kDma = DEC3_ABL != 1 && DEC3_ABL != 3;
    {
      // every wave runs the same body (a wave past nb computes on zero rows): a branch around it splits the
      // loop-carried O accumulators between register classes
      // GEMM1(t + 1) (on a stale slot after the last tile: one code path, result unused); in its gaps: the
      // completion of S^T(t)'s own half, the tail mask, the 8 exponentials of tile t, the LDS-DMA of t + 2
      float pv[8];
      uint32_t pk[4];
      const bool tail = t == ntiles - 1 && (N % kBfTI) != 0;  // wave-uniform
      std::array<s16x4, 2> n2[BH];
      f32x16 s_new = gemm1(lds + nxt * TB, [&] {
        if (kDma && DEC3_DMA == 0) issue_pieces(soff_dma, s_dma, 0, DEC3_DMA_PRE, true);
      }, [&](int g) {
        if (g == 0 && DEC3_ABL != 4) {
          const float* src = xs + pw * 512;
          y0 = *reinterpret_cast<const float4*>(src + lane * 4);
          y1 = *reinterpret_cast<const float4*>(src + 256 + lane * 4);
        } else if (g == 1) {
          const float yv[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
          for (int r = 0; r < 8; ++r) sm[r] = DHC == 0 ? sm[r] + yv[r] : yv[r] + sm[r];
          if (__builtin_expect(tail, 0)) {  // rows past N (read as 0) leave the softmax
            const int lim = (int)(N - t * kBfTI) - 4 * h - 16 * dh;
#pragma unroll
            for (int r = 0; r < 8; ++r) sm[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : sm[r];
          }
        } else if (g >= 2 && g < 10) {
          const int r = g - 2;
          pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sm[r], kLog2e, -mL));
          lsum += pv[r];
          if (r & 1) pk[r >> 1] = pack_bf16x2(pv[r - 1], pv[r]);
        }
        constexpr int PRE = DEC3_DMA == 0 ? DEC3_DMA_PRE : 0;
        if (kDma && g < P1 - PRE) issue_pieces(soff_dma, s_dma, PRE + g, PRE + g + 1, PRE == 0 && g == 0);
        if (DEC3_G2PRE > 0 && g == NG - DEC3_G2PRE) g2_pre(lds + cur * TB, DHC, n2);  // GEMM2(t)'s first reads
      });
      DEC3_STAMP(3);  // [3] GEMM1 (+ softmax, DMA issue)
      // P(t) own half out; [B(t)] (before GEMM2, or after its own-half MFMA DEC3_BB); then the partner's
      // partial half of S^T(t + 1) out and the partner's P half in; GEMM2(t), own half first
      if (DEC3_ABL != 4) *reinterpret_cast<uint4*>(xp + (w * 64 + lane) * 4) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
      uint4 po = make_uint4(0u, 0u, 0u, 0u);
      auto exch_b = [&] {
        if (DEC3_ABL != 2 && DEC3_ABL != 3) barrier();
        if (DEC3_ABL != 4) {
          float* dst = xs + w * 512;  // the partner's half of the new partial (static registers)
#pragma unroll
          for (int r4 = 0; r4 < 2; ++r4) {
            const int r = 8 * (1 - DHC) + 4 * r4;
            *reinterpret_cast<float4*>(dst + r4 * 256 + lane * 4) =
                make_float4(s_new[r], s_new[r + 1], s_new[r + 2], s_new[r + 3]);
          }
          po = *reinterpret_cast<const uint4*>(xp + (pw * 64 + lane) * 4);
        }
      };
      if (BBI < 0) exch_b();
      DEC3_STAMP(4);  // [4] P out + barrier B
      if (DEC3_G2PRE == 0) g2_pre(lds + cur * TB, DHC, n2);
      const bf16x8 pown = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
      gemm2(lds + cur * TB, DHC, n2, pown, po, [&](int i) {
        if (BBI >= 0 && i == BBI) exch_b();
        if (kDma && P1 + i / 2 < PW && (i & 1) == 0) issue_pieces(soff_dma, s_dma, P1 + i / 2, P1 + i / 2 + 1, false);
        if (i == DB - 1) DEC3_STAMP(5);  // [5] half-S out + GEMM2 own half
      });
      DEC3_STAMP(6);  // [6] GEMM2 partner half
#pragma unroll
      for (int r = 0; r < 8; ++r) sm[r] = s_new[8 * DHC + r];
    }
    cur = nxt;
  }
  };
  if (dh == 0) sweep(std::integral_constant<int, 0>{});
  else sweep(std::integral_constant<int, 1>{});
#if DEC3_STAMPS
  if (lane == 0 && blockIdx.x * 4 + w < 4096) {
    st_acc[7] = (unsigned long long)(t_end > t_beg ? t_end - t_beg : 0);
    for (int i = 0; i < 8; ++i) g_dec3_stamps[blockIdx.x * 4 + w][i] = st_acc[i];
  }
#endif

  wait_vmcnt<0>();  // the last tile's LDS-DMA (a duplicate, never read) lands before the ring is released

  // l = (own items) + (partner's items), the same sum in both waves
  lsum += __shfl_xor(lsum, 32, 64);
  barrier();  // every wave is past its last read of the P buffers (xm aliases them)
  if (h == 0) xm[w * 32 + col] = lsum;
  barrier();
  if (!wave_active || t_beg >= t_end || user >= nb) return;
  const float lo = xm[pw * 32 + col];
  const float ltot = dh == 0 ? lsum + lo : lo + lsum;
  if (h == 0 && dh == 0) out.flag[out.direct ? user : (int64_t)split * nb + user] = !(ltot >= kMinL);
  const int64_t row = out.direct ? user : (int64_t)split * nb + user;
  if (h == 0 && dh == 0) {
    if (out.direct) out.lse[user] = m + logf(ltot);
    else { out.m[row] = m; out.l[row] = ltot; }
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

// ------------------------------------------------------------- version 4 ---
// D = 768, one barrier per tile and no partial-S exchange. Version 3 splits GEMM1 over D, so the pair's
// partial S^T halves cross LDS every tile (2 KiB each way) and a second barrier orders them. Here wave
// (ug, dh) computes S^T of ITS 16 items over all of D for its 32 users with v_mfma_f32_16x16x32_bf16
// (u over all of D in 192 VGPRs as the B operand; one E row read serves both 16-user halves), so its
// scores are complete and only P crosses LDS:
//   iteration t: [barrier: tile t + 1 landed, P(t) halves published] -> LDS-DMA of t + 2 into the slot
//   GEMM2(t - 1) freed -> GEMM1(t + 1) (48 MFMAs of 16 cycles) -> GEMM2(t) over both k-steps with P(t) read
//   back from LDS in the B layout (24 MFMAs of 32 cycles), the 8 exponentials of tile t + 1 in its gaps ->
//   P(t + 1) own half out (P double-buffered by tile parity).
// O (the wave's D half, 192 AGPRs), the LDS image, the DMA pieces, the GEMM2 reads and the fixed-offset /
// flag rules are version 3's; P is stored per user in GEMM2's k order (position 8 (q >> 2 & 1) + 4 (q >> 3)
// + (q & 3) for item q of a half), with an 80-B row stride so that the B-layout reads hit every bank once.
#ifndef DEC4_DMA
#define DEC4_DMA 0  // LDS-DMA pieces: 0 = in GEMM1's gaps, 1 = in GEMM2's, 2 = half in each
#endif
// timing ablations (A/B builds only, results invalid): 1 = no LDS-DMA / vmcnt waits in the loop,
// 2 = no barrier in the loop, 3 = no exponentials / P stores, 4 = LDS-DMA issued but never waited for in the loop
#ifndef DEC4_ABL
#define DEC4_ABL 0
#endif
#ifndef DEC4_G1_AHEAD
#define DEC4_G1_AHEAD 2  // GEMM1 A operand k-steps in flight
#endif
// NW waves per block = NW / 2 user groups x 2 D halves (NW = 8: two waves per SIMD, <= 256 registers each --
// d = 384, where u over all of D takes 96 VGPRs and O's half 96 AGPRs). A D half that is not a whole number of
// 128-column segments (d = 384) owns every other 32-column d-block instead (block 2 db + dh).
// GEMM1's MFMA row block b (rows 4 b .. 4 b + 3 of the 16x16x32 A operand, lanes c16 = 4 b ..) reads own-item
// block dec4_rowblk(b) = 0, 2, 3, 1 of the tile half. In the image's chunk XOR (d2_off) the natural order puts
// the two 4-row blocks of each ds_read_b128 lane group on the same banks (2-way: SQ_LDS_BANK_CONFLICT 0.33 of
// the sweep's LDS cycles); with this map every group's 16 lanes read 16 distinct 16-B bank slots.
#ifndef DEC4_ROWMAP
#define DEC4_ROWMAP 0x1320
#endif
__host__ __device__ constexpr int dec4_rowblk(int b) { return (DEC4_ROWMAP >> (4 * b)) & 3; }

__host__ __device__ constexpr int d4_lds_bytes(int D, int NW) {
  return 3 * ((D / 128) * 8192) + 2 * (NW / 2) * 32 * 80 + NW * 64 * 4;
}

template <int D, int NW, bool WITH_O>
__global__ void __launch_bounds__(64 * NW) k_dec4_bf16(const float* __restrict__ U, int64_t ldu,
                                                   const bf16_t* __restrict__ E, const float* __restrict__ e_maxnorm,
                                                   int64_t nb, int64_t N, int splits, int64_t tiles_per_split,
                                                   DecOut out) {
  constexpr int DW = D / 2;         // GEMM2: dims owned by one wave
  constexpr int DB = DW / 32;       // GEMM2 d-blocks
  constexpr int KS = D / 32;        // GEMM1 k-steps (16x16x32, all of D)
  constexpr int NSEG = D / 128;
  constexpr int TB = NSEG * 8192;
  constexpr int NUG = NW / 2;       // user groups per block
  constexpr int PW = NSEG * 8 / NW; // 1-KiB LDS-DMA pieces per wave per tile
  constexpr int NS = 3;
  constexpr int PST = 80;           // P row stride (bytes)
  constexpr bool SEGH = DW % 128 == 0;  // a D half is whole segments (else interleaved d-blocks)
  static_assert(D % 128 == 0 && (NSEG * 8) % NW == 0 && (NW == 4 || NW == 8) && d4_lds_bytes(D, NW) <= 160 * 1024,
                "k_dec4_bf16 shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* pbuf = lds + NS * TB;                                     // [2 parity][NUG ug][32 users][PST]
  float* xm = reinterpret_cast<float*>(lds + NS * TB + 2 * NUG * 32 * PST);  // [NW w][64]: max / sum exchange

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  // GEMM1 layout: users c16 + 16 nb; MFMA rows 4 g .. 4 g + 3 are own items 4 gi .. 4 gi + 3 (row map below)
  const int c16 = lane & 15, g = lane >> 4, gi = dec4_rowblk(g);
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ug = w & (NUG - 1), dh = w / NUG, pw = w ^ NUG;
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * (32 * NUG) + ug * 32;
  const int64_t user = u0 + col;  // GEMM2 / output layout
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kBfTI - 1) / kBfTI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const int dbase = dh * DW;
  const float emax = *e_maxnorm;  // before any LDS-DMA is in flight

  // u as GEMM1's B operand: lane holds U[u0 + c16 + 16 nb][32 ks + 8 g .. + 7]
  uint4 uf[KS][2];
  float usq[2] = {0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) {
      const int64_t uu = u0 + c16 + 16 * n2;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (uu < nb) {
        a = *reinterpret_cast<const float4*>(U + uu * ldu + 32 * ks + 8 * g);
        b = *reinterpret_cast<const float4*>(U + uu * ldu + 32 * ks + 8 * g + 4);
      }
      usq[n2] += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w) + (b.x * b.x + b.y * b.y) + (b.z * b.z + b.w * b.w);
      uf[ks][n2] = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w), pack_bf16x2(b.x, b.y),
                              pack_bf16x2(b.z, b.w));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  float bound[2];
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
    float v = usq[n2];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    bound[n2] = sqrtf(v) * emax * 1.02f;
  }

  // LDS-DMA into version 2's image (version 3's pieces)
  int vlane[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int row = 8 * pb + ((lane >> 2) & 7);
    vlane[pb] = ((lane >> 2) & 7) * (D * 2) + 64 * (lane >> 5) + 16 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(E), (short)0, (int)(N * D * 2), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(w * PW * 1024);
  auto issue_pieces = [&](uint32_t soff, int slot_i, int i0, int i1, bool fresh) {
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int p = w * PW + i;  // wave-uniform; its own bits (PW need not be a multiple of 4)
      const uint32_t so = soff + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (p & 1));
      const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
      if (fresh && i == i0)
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
    }
  };
  auto tile_soff = [&](int64_t t) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)(kBfTI * D * 2)));
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // GEMM1: S^T[16 own items][32 users] over all of D; A = image row 16 dh + 4 dec4_rowblk(c16 >> 2) + (c16 & 3),
  // chunk 4 ks + g
  const int r1 = 16 * dh + 4 * dec4_rowblk(c16 >> 2) + (c16 & 3);
  const int laneA = ((r1 >> 3) << 11) + ((r1 & 7) << 6) + ((g ^ ((r1 >> 2) & 3)) << 4);
  auto gemm1 = [&](const unsigned char* buf, f32x4 (&s)[2], auto&& fill) {
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[n2][r] = 0.f;
    const unsigned char* b0 = buf + laneA;
    auto rdA = [&](int ks) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(b0 + ((ks >> 2) << 13) + ((ks & 3) << 9)));
    };
    constexpr int AH = DEC4_G1_AHEAD;
    bf16x8 a[AH];
#pragma unroll
    for (int j = 0; j < AH; ++j) a[j] = rdA(j);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8 c = a[ks % AH];
      if (ks + AH < KS) a[ks % AH] = rdA(ks + AH);
      s[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, __builtin_bit_cast(bf16x8, uf[ks][0]), s[0], 0, 0, 0);
      s[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, __builtin_bit_cast(bf16x8, uf[ks][1]), s[1], 0, 0, 0);
      fill(ks);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" : "+v"(s[0]), "+v"(s[1]));  // S^T in VGPRs (the softmax reads it; O owns the AGPRs)
  };
  // GEMM2 (version 3's reads): O^T[DW][32 users] += E^T P^T over k-steps 0 (items 0..15) and 1 (16..31)
  const int g1 = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  // the wave's d-block db: global 32-column block dbase / 32 + db (SEGH) or 2 db + dh
  const int cseg = SEGH ? (dbase / 128) << 13 : dh << 9;
  auto dboff = [](int db) { return SEGH ? ((db >> 2) << 13) + ((db & 3) << 9) : ((db >> 1) << 13) + ((db & 1) << 10); };
  auto dcol = [&](int db) { return SEGH ? dbase + 32 * db : 32 * (2 * db + dh); };
  const int laneT0 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((0 + h) & 3)) << 4) + 8 * (pp & 1);
  const int laneT1 = ((4 * h + q) << 6) + (((2 * g1 + (pp >> 1)) ^ ((2 + h) & 3)) << 4) + 8 * (pp & 1);
  f32x16 o[WITH_O ? DB : 1];
#pragma unroll
  for (int d = 0; d < (WITH_O ? DB : 1); ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  constexpr int BH = 2;
  auto rdT = [&](const unsigned char* buf, int i) {
    const int kh = i / DB, db = i % DB;
    const unsigned char* t = buf + cseg + (kh << 12);
    auto* p0 = (__attribute__((address_space(3))) s16x4*)(void*)(t + laneT0 + dboff(db));
    auto* p1 = (__attribute__((address_space(3))) s16x4*)(void*)(t + laneT1 + (1 << 11) + dboff(db));
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
        if (i + BH < 2 * DB) n[i % BH] = rdT(buf, i + BH);
        const s16x8 a = {c[0][0], c[0][1], c[0][2], c[0][3], c[1][0], c[1][1], c[1][2], c[1][3]};
        o[i % DB] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                           __builtin_bit_cast(bf16x8, i < DB ? pf0 : pf1), o[i % DB],
                                                           0, 0, 0);
        fill(i);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2 * DB; ++i) fill(i);
    }
  };
  // P rows: pbuf[par][ug][user][PST]; own half at k-step dh; lane's items 4 g .. 4 g + 3 -> positions
  // 16 dh + 8 (gi & 1) + 4 (gi >> 1)
  auto p_row = [&](int par, int uu) { return pbuf + ((par * NUG + ug) * 32 + uu) * PST; };
  const int ppos = 2 * (16 * dh + 8 * (gi & 1) + 4 * (gi >> 1));

  float m[2] = {0.f, 0.f}, mL[2] = {0.f, 0.f}, lsum[2] = {0.f, 0.f};
  f32x4 s_nx[2];
  // tail: own items 16 dh + 4 g + i of tile t past N leave the softmax
  auto mask_tail = [&](f32x4 (&s)[2], int64_t t) {
    if (t == ntiles - 1 && (N % kBfTI) != 0) {
      const int lim = (int)(N - t * kBfTI) - 16 * dh - 4 * gi;
#pragma unroll
      for (int n2 = 0; n2 < 2; ++n2)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[n2][r] = r >= lim ? -INFINITY : s[n2][r];
    }
  };
  if (t_beg < t_end) {
    issue_pieces(tile_soff(t_beg), 0, 0, PW, true);
    issue_pieces(tile_soff(min(t_beg + 1, t_end - 1)), 1, 0, PW, true);
    wait_vmcnt<PW>();
  }
  barrier();
  if (t_beg < t_end) {
    // first tile: its max over both halves sets the pair's fixed offset m (version 2's rule)
    gemm1(lds, s_nx, [](int) {});
    mask_tail(s_nx, t_beg);
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) {
      float mx = fmaxf(fmaxf(s_nx[n2][0], s_nx[n2][1]), fmaxf(s_nx[n2][2], s_nx[n2][3]));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (g == 0) xm[w * 64 + c16 + 16 * n2] = mx;
      m[n2] = mx;
    }
    barrier();
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) {
      m[n2] = fmaxf(fmaxf(m[n2], xm[pw * 64 + c16 + 16 * n2]), bound[n2] - kOffsetSpan);
      mL[n2] = m[n2] * kLog2e;
    }
    // P(t_beg) own half -> parity 0
#pragma unroll
    for (int n2 = 0; n2 < 2; ++n2) {
      float pv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pv[r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[n2][r], kLog2e, -mL[n2]));
        lsum[n2] += pv[r];
      }
      *reinterpret_cast<uint2*>(p_row(0, c16 + 16 * n2) + ppos) =
          make_uint2(pack_bf16x2(pv[0], pv[1]), pack_bf16x2(pv[2], pv[3]));
    }
  }

  for (int64_t t = t_beg; t < t_end; ++t) {
    const int li = (int)(t - t_beg);
    const int cur = li % NS, nxt = (li + 1) % NS, s_dma = (li + 2) % NS, par = li & 1;
    // [t]: tile t + 1 has landed, P(t) halves are published (the xm reads of the prologue are done)
    if (DEC4_ABL != 1 && DEC4_ABL != 4) wait_vmcnt<0>();
    if (DEC4_ABL != 2) barrier();
    const int64_t t_dma = min(t + 2, t_end - 1);
    const uint32_t soff_dma = tile_soff(t_dma);
    // P(t) in GEMM2's B layout: user col, positions 8 h .. 8 h + 7 of k-steps 0 and 1
    const uint4 pf0 = *reinterpret_cast<const uint4*>(p_row(par, col) + 16 * h);
    const uint4 pf1 = *reinterpret_cast<const uint4*>(p_row(par, col) + 32 + 16 * h);
    // GEMM1(t + 1) (a stale slot after the last tile: one code path, result unused) with the DMA of t + 2
    gemm1(lds + nxt * TB, s_nx, [&](int ks) {
      constexpr int P1 = DEC4_DMA == 0 ? PW : DEC4_DMA == 1 ? 0 : PW / 2;  // pieces in GEMM1
      if (DEC4_ABL != 1 && (ks & 1) == 1 && ks / 2 < P1) issue_pieces(soff_dma, s_dma, ks / 2, ks / 2 + 1, ks == 1);
    });
    mask_tail(s_nx, t + 1);
    // GEMM2(t); the softmax of tile t + 1 in its gaps (after the last tile it runs on the unused GEMM1 result:
    // its l terms are weighted 0 and its P half is never read -- no branch, so nothing is sunk out of the gaps)
    const float lw = t + 1 < t_end ? 1.f : 0.f;
    float pv[8];
    uint32_t pk[4];
    gemm2(lds + cur * TB, pf0, pf1, [&](int i) {
      if (DEC4_ABL != 3 && i >= 1 && i <= 8) {
        const int e = i - 1, n2 = e >> 2, r = e & 3;
        pv[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[n2][r], kLog2e, -mL[n2]));
        lsum[n2] = __builtin_fmaf(pv[e], lw, lsum[n2]);
        if (r & 1) pk[e >> 1] = pack_bf16x2(pv[e - 1], pv[e]);
        if (e == 3 || e == 7)
          *reinterpret_cast<uint2*>(p_row(par ^ 1, c16 + 16 * n2) + ppos) = make_uint2(pk[2 * n2], pk[2 * n2 + 1]);
      }
      constexpr int P1 = DEC4_DMA == 0 ? PW : DEC4_DMA == 1 ? 0 : PW / 2;
      if (DEC4_ABL != 1 && (i & 1) == 0 && P1 + i / 2 < PW)
        issue_pieces(soff_dma, s_dma, P1 + i / 2, P1 + i / 2 + 1, P1 == 0 && i == 0);
    });
  }

  wait_vmcnt<0>();  // the last tile's LDS-DMA (a duplicate, never read) lands before the ring is released

  // l = own items (4 lanes g) + partner's items; then per user in the GEMM2 / output layout
#pragma unroll
  for (int n2 = 0; n2 < 2; ++n2) {
    lsum[n2] += __shfl_xor(lsum[n2], 16, 64);
    lsum[n2] += __shfl_xor(lsum[n2], 32, 64);
  }
  barrier();  // every wave is past its last read of xm
  if (g == 0) {
    xm[w * 64 + c16] = lsum[0];
    xm[w * 64 + c16 + 16] = lsum[1];
    xm[w * 64 + 32 + c16] = m[0];
    xm[w * 64 + 32 + c16 + 16] = m[1];
  }
  barrier();
  if (!wave_active || t_beg >= t_end || user >= nb) return;
  const float lown = xm[w * 64 + col], lo = xm[pw * 64 + col], mu = xm[w * 64 + 32 + col];
  const float ltot = dh == 0 ? lown + lo : lo + lown;
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
        const int dd = dcol(d) + 8 * g4 + 4 * h;
        *reinterpret_cast<float4*>(out.O + row * D + dd) =
            make_float4(o[d][4 * g4] * sc, o[d][4 * g4 + 1] * sc, o[d][4 * g4 + 2] * sc, o[d][4 * g4 + 3] * sc);
      }
  }
}


// fp8 at d = 768 with version 4's structure (k_dec4_f8): wave (ug, dh) computes the COMPLETE S^T of items
// 32 dh .. 32 dh + 31 of each 64-item tile over all of D (u over all of D as e4m3: 96 VGPRs, where the
// DS = 2 ring above holds a D half and exchanges partial scores), so only P crosses LDS: each wave writes its
// packed e4m3 half and that half's block exponent (the MFMA takes k-block b's scale from lane column + 32 b,
// so the halves keep their own exponents), double-buffered by tile parity, which leaves one barrier per tile:
//   [barrier: tile t + 1 landed, P(t) halves published, GEMM2(t - 1) done]
//   -> GEMM1(t + 1) (12 32x32x64 MFMAs, the LDS-DMA of tile t + 2 one piece per MFMA gap)
//   -> the own half's max and exponent -> GEMM2(t) (12 MFMAs over both item halves, the 16 exponentials of
//   tile t + 1 in its gaps) -> P(t + 1) half out.
// The image, the pieces, the GEMM2 transposed reads, the exponent rule and the fixed offset are k_dec_fp8's.
#ifndef F8V4_G1_AHEAD
#define F8V4_G1_AHEAD 2
#endif
constexpr int kF8v4PBytes = 1024 + 256;  // per wave and parity: P half (64 lanes x 16 B) + exponent (64 x 4 B)
constexpr int f8v4_lds_bytes() { return 3 * 64 * 768 + 2 * 4 * kF8v4PBytes + 4 * 256; }

template <bool WITH_O>
__global__ void __launch_bounds__(256) k_dec4_f8(const float* __restrict__ U, int64_t ldu,
                                                 const unsigned char* __restrict__ T8, const int* __restrict__ e_exp,
                                                 const float* __restrict__ e_maxnorm, int64_t nb, int64_t N,
                                                 int splits, int64_t tiles_per_split, DecOut out) {
  constexpr int D = 768;
  constexpr int DW = D / 2;        // GEMM2: dims owned by one wave
  constexpr int KS = D / 64;       // GEMM1 k-steps over all of D
  constexpr int DB = DW / 32;      // GEMM2 d-blocks
  constexpr int TB = f8_tile_bytes<D>();
  constexpr int PW = TB / 4096;    // 1-KiB LDS-DMA pieces per wave per tile (12)
  constexpr int NS = 3;
  static_assert(f8v4_lds_bytes() <= 160 * 1024, "k_dec4_f8 LDS");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  unsigned char* pbuf = lds + NS * TB;                                        // [2 par][4 w][kF8v4PBytes]
  float* xm = reinterpret_cast<float*>(lds + NS * TB + 2 * 4 * kF8v4PBytes);  // [4 w][64]

  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ug = w & 1, dh = w >> 1, pw = w ^ 2;
  const int dbase = dh * DW;
  const int split = blockIdx.x % splits;
  const int64_t u0 = (int64_t)(blockIdx.x / splits) * 64 + ug * 32;
  const int64_t user = u0 + col;
  const bool wave_active = u0 < nb;
  const int64_t ntiles = (N + kF8TI - 1) / kF8TI;
  const int64_t t_beg = (int64_t)split * tiles_per_split;
  const int64_t t_end = min(ntiles, t_beg + tiles_per_split);
  const float emax = *e_maxnorm;  // scalars before any LDS-DMA is in flight
  const int ke = *e_exp;
  const int sa = 127 - ke;

  // u over all of D: lane (col, h) holds u[64 ks + 32 h + j], j < 32, as e4m3 of u 2^ku (ku from the row)
  const float* urow = U + min(user, nb - 1) * ldu + 32 * h;
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
  i32x8 uf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int q4 = 0; q4 < 8; ++q4) {
      const float4 a = *reinterpret_cast<const float4*>(urow + 64 * ks + 4 * q4);
      uf[ks][q4] = pack_fp8x4(a.x * qu, a.y * qu, a.z * qu, a.w * qu);
    }
    __builtin_amdgcn_sched_barrier(0);
  }

  const int voff = w * PW * 1024 + lane * 16;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(T8), (short)0, (int)(ntiles * TB), 0x00020000);
  const uint32_t ring0 = lds_addr(lds) + (uint32_t)(w * PW * 1024);
  auto issue_piece = [&](uint32_t soff, int slot_i, int i, bool fresh) {
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
    if (fresh)
      asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff), "s"(rsrc), "s"(soff + (uint32_t)(i * 1024)) : "memory");
    else
      asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                   :: "s"(lb + (uint32_t)(i * 1024)), "v"(voff), "s"(rsrc), "s"(soff + (uint32_t)(i * 1024)) : "memory");
  };
  auto tile_soff = [&](int64_t t) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)(t * (int64_t)TB)); };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // GEMM1 A operand (k-step ks of all of D): item row 32 dh + col, chunks 4 ks + 2 h + {0, 1}
  const int swc = f8_sw(D, col);  // f8_sw depends on the low 4 bits of the row only
  const unsigned char* rowA_off = nullptr;
  const int rowA = (32 * dh + col) * D;
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
  (void)rowA_off;
  // GEMM2 A operand (d-block db of this wave's D half): four transposed reads of items f8_item_of(h, 8 c + qq)
  const int g1 = (lane >> 4) & 1, qq = (lane & 15) >> 1, pp = lane & 1;
  int trow[4], tsw[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int it = f8_item_of(h, 8 * c + qq);
    trow[c] = it * D + 8 * pp;
    tsw[c] = f8_sw(D, it);
  }
  auto rdB = [&](const unsigned char* buf, int db) {
    i32x8 r;
    const int ch = 2 * (dbase / 32 + db) + g1;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
          (__attribute__((address_space(3))) i32x2*)(void*)(buf + trow[c] + 16 * (ch ^ tsw[c])));
      r[2 * c] = v[0];
      r[2 * c + 1] = v[1];
    }
    return r;
  };
  auto gemm1 = [&](const unsigned char* buf, f32x16& sv, auto&& fill) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = 0.f;
    constexpr int AH = F8V4_G1_AHEAD;
    i32x8 ra[AH];
#pragma unroll
    for (int j = 0; j < AH; ++j) ra[j] = rdA(buf, j);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const i32x8 c = ra[ks % AH];
      if (ks + AH < KS) ra[ks % AH] = rdA(buf, ks + AH);
      sv = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c, uf[ks], sv, 0, 0, 0, sa, 0, sbu);
      fill(ks);
      __builtin_amdgcn_sched_barrier(0);
    }
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
        if (db + AH2 < DB) a[db % AH2] = rdB(buf, db + AH2);
        o[db] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(c, pf, o[db], 0, 0, 0, sa, 0, sbp);
        fill(db);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int db = 0; db < DB; ++db) fill(db);
    }
  };

  float m = 0.f, mL = 0.f, lsum = 0.f;
  const float bound = sqrtf(usq) * emax * 1.02f;
  // own half of tile t: items past N -> -inf; the half's max over its 32 items (every lane of a column)
  auto half_max = [&](int64_t t, f32x16& sv) {
    if (t == ntiles - 1 && (N % kF8TI) != 0) {
      const int lim = (int)(N - t * kF8TI) - 4 * h - 32 * dh;
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = ((r & 3) + 8 * (r >> 2) >= lim) ? -INFINITY : sv[r];
    }
    const float a0 = fmaxf(fmaxf(sv[0], sv[1]), sv[2]), a1 = fmaxf(fmaxf(sv[3], sv[4]), sv[5]);
    const float a2 = fmaxf(fmaxf(sv[6], sv[7]), sv[8]), a3 = fmaxf(fmaxf(sv[9], sv[10]), sv[11]);
    const float a4 = fmaxf(fmaxf(sv[12], sv[13]), fmaxf(sv[14], sv[15]));
    float mx = fmaxf(fmaxf(fmaxf(a0, a1), a2), fmaxf(a3, a4));
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
  };
  auto tile_exp = [&](float mh) { return max(-119, min(127, (int)ceilf(__builtin_fmaf(mh, kLog2e, -mL)) - 8)); };
  auto p_slot = [&](int par, int ww) { return pbuf + (par * 4 + ww) * kF8v4PBytes; };
  int pk[4] = {0, 0, 0, 0}, e_own = 0;  // this wave's P half of the current tile and its exponent
  auto p_publish = [&](int par) {
    reinterpret_cast<int4*>(p_slot(par, w))[lane] = make_int4(pk[0], pk[1], pk[2], pk[3]);
    reinterpret_cast<int*>(p_slot(par, w) + 1024)[lane] = e_own;
  };

  f32x16 s_nx;
  if (t_beg < t_end) {
    for (int i = 0; i < PW; ++i) issue_piece(tile_soff(t_beg), 0, i, i == 0);
    if (t_beg + 1 < t_end)
      for (int i = 0; i < PW; ++i) issue_piece(tile_soff(t_beg + 1), 1, i, false);
    wait_vmcnt<0>();
  }
  barrier();
  float mh = 0.f;
  if (t_beg < t_end) {
    gemm1(lds, s_nx, [](int) {});
    mh = half_max(t_beg, s_nx);
    if (lane < 32) xm[w * 64 + lane] = mh;
  }
  barrier();  // the pair's common offset from the first tile's max over both halves
  if (t_beg < t_end) {
    m = fmaxf(fmaxf(mh, xm[pw * 64 + col]), bound - kOffsetSpan);
    mL = m * kLog2e;
    e_own = tile_exp(mh);
    const float cE = mL + (float)e_own;
    float qsum = 0.f;
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      float q[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        q[b] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[4 * j4 + b], kLog2e, -cE));
        qsum += q[b];
      }
      pk[j4] = pack_fp8x4(q[0], q[1], q[2], q[3]);
    }
    lsum += ldexpf(qsum, e_own);
    p_publish(0);
  }
  for (int64_t t = t_beg; t < t_end; ++t) {
    const int li = (int)(t - t_beg);
    const int cur = li % NS, nxt = (li + 1) % NS, s_dma = (li + 2) % NS, par = li & 1;
    wait_vmcnt<0>();
    barrier();  // tile t + 1 landed, P(t) halves published, GEMM2(t - 1) done
    const int4 y = reinterpret_cast<const int4*>(p_slot(par, pw))[lane];
    const int ey = reinterpret_cast<const int*>(p_slot(par, pw) + 1024)[lane];
    i32x8 pf;
    if (dh == 0) {
      pf[0] = pk[0]; pf[1] = pk[1]; pf[2] = pk[2]; pf[3] = pk[3];
      pf[4] = y.x; pf[5] = y.y; pf[6] = y.z; pf[7] = y.w;
    } else {
      pf[0] = y.x; pf[1] = y.y; pf[2] = y.z; pf[3] = y.w;
      pf[4] = pk[0]; pf[5] = pk[1]; pf[6] = pk[2]; pf[7] = pk[3];
    }
    const int sbp = 127 + (h == dh ? e_own : ey);  // lane half h: k-block h's scale
    const bool more = t + 1 < t_end;
    if (more) {
      const bool dma = t + 2 < t_end;
      const uint32_t soff_dma = tile_soff(dma ? t + 2 : t);
      gemm1(lds + nxt * TB, s_nx, [&](int ks) {
        if (dma) issue_piece(soff_dma, s_dma, ks, ks == 0);
      });
      mh = half_max(t + 1, s_nx);
    }
    const int e_nx = more ? tile_exp(mh) : 0;
    const float cE = mL + (float)e_nx;
    float q[16];
    float qsum = 0.f;
    int pk_nx[4];
    gemm2(lds + cur * TB, pf, sbp, [&](int db) {
      if (more) {
#pragma unroll
        for (int j = (16 * db) / DB; j < (16 * (db + 1)) / DB; ++j) {
          q[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(s_nx[j], kLog2e, -cE));
          qsum += q[j];
          if ((j & 3) == 3) pk_nx[j >> 2] = pack_fp8x4(q[j - 3], q[j - 2], q[j - 1], q[j]);
        }
      }
    });
    if (more) {
      lsum += ldexpf(qsum, e_nx);
      pk[0] = pk_nx[0]; pk[1] = pk_nx[1]; pk[2] = pk_nx[2]; pk[3] = pk_nx[3];
      e_own = e_nx;
      p_publish(par ^ 1);
    }
  }
  wait_vmcnt<0>();
  // l = own half (both lane halves of the column) + the partner's half, in dh order
  const float lw = lsum + __shfl_xor(lsum, 32, 64);
  barrier();
  if (lane < 32) xm[w * 64 + lane] = lw;
  barrier();
  const float ltot = dh == 0 ? lw + xm[pw * 64 + col] : xm[pw * 64 + col] + lw;
  if (!wave_active || t_beg >= t_end || user >= nb) return;
  if (h == 0 && dh == 0) out.flag[out.direct ? user : (int64_t)split * nb + user] = !(ltot >= kMinL);
  const int64_t row = out.direct ? user : (int64_t)split * nb + user;
  if (h == 0 && dh == 0) {
    if (out.direct) out.lse[user] = m + logf(ltot);
    else { out.m[row] = m; out.l[row] = ltot; }
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


template <int D, bool WO>
static int launch_bf16(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                       const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int lds = bf_stages<D>() * (bf_tile_bytes<D>() + bf_ttile_bytes<D>());
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec_bf16<D, WO>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  const bf16_t* Et = (const bf16_t*)((const char*)E + et_offset_bytes(N, D));
  k_dec_bf16<D, WO><<<(unsigned)p.blocks, 256, lds, st>>>(U, ldu, (const bf16_t*)E, Et, enorm, nb, N, p.splits,
                                                         p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec_bf16");
  return HVAE_OK;
}

template <int D, bool WO>
static int launch_bf16_v3(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                          const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int lds = d3_lds_bytes(D);
  static_assert(lds <= 160 * 1024, "k_dec3_bf16 LDS");
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec3_bf16<D, WO>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  k_dec3_bf16<D, WO><<<(unsigned)p.blocks, 256, lds, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N, p.splits,
                                                          p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec3_bf16");
  return HVAE_OK;
}

template <int D, bool WO>
static int launch_bf16_v4(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                          const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int NW = D == 768 ? 4 : 8;
  constexpr int lds = d4_lds_bytes(D, NW);
  static_assert(lds <= 160 * 1024, "k_dec4_bf16 LDS");
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec4_bf16<D, NW, WO>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 lds));
    attr_set = true;
  }
  k_dec4_bf16<D, NW, WO><<<(unsigned)p.blocks, 64 * NW, lds, st>>>(U, ldu, (const bf16_t*)E, enorm, nb, N,
                                                                  p.splits, p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec4_bf16");
  return HVAE_OK;
}

template <bool WO>
static int launch_fp8_v4(const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                         const DecPlan& p, DecOut o, hipStream_t st) {
  constexpr int D = 768, lds = f8v4_lds_bytes();
  static bool attr_set = false;
  if (!attr_set) {
    HVAE_HIP(hipFuncSetAttribute((const void*)k_dec4_f8<WO>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  const unsigned char* T8 = (const unsigned char*)E + f8_offset_bytes(N, D);
  const int* ke = (const int*)((const char*)E + f8_tail_offset(N, D));
  k_dec4_f8<WO><<<(unsigned)p.blocks, 256, lds, st>>>(U, ldu, T8, ke, enorm, nb, N, p.splits, p.tiles_per_split, o);
  HVAE_LAUNCH_CHECK("k_dec4_f8");
  return HVAE_OK;
}

int ab_dec_v1(bool wo, int D, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st) {
  switch (D) {
    case 64: return wo ? launch_bf16<64, true>(U, ldu, E, enorm, nb, N, p, o, st)
                       : launch_bf16<64, false>(U, ldu, E, enorm, nb, N, p, o, st);
    case 128: return wo ? launch_bf16<128, true>(U, ldu, E, enorm, nb, N, p, o, st)
                        : launch_bf16<128, false>(U, ldu, E, enorm, nb, N, p, o, st);
    case 256: return wo ? launch_bf16<256, true>(U, ldu, E, enorm, nb, N, p, o, st)
                        : launch_bf16<256, false>(U, ldu, E, enorm, nb, N, p, o, st);
    case 384: return wo ? launch_bf16<384, true>(U, ldu, E, enorm, nb, N, p, o, st)
                        : launch_bf16<384, false>(U, ldu, E, enorm, nb, N, p, o, st);
    default: break;
  }
  HVAE_FAIL(HVAE_ERR_UNSUPPORTED, "ab_dec_v1: D=%d", D);
}

int ab_dec_v3(bool wo, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st) {
  return wo ? launch_bf16_v3<768, true>(U, ldu, E, enorm, nb, N, p, o, st)
            : launch_bf16_v3<768, false>(U, ldu, E, enorm, nb, N, p, o, st);
}

int ab_dec_v4(bool wo, int D, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
              const DecPlan& p, DecOut o, hipStream_t st) {
  if (D == 768)
    return wo ? launch_bf16_v4<768, true>(U, ldu, E, enorm, nb, N, p, o, st)
              : launch_bf16_v4<768, false>(U, ldu, E, enorm, nb, N, p, o, st);
  if (D == 384)
    return wo ? launch_bf16_v4<384, true>(U, ldu, E, enorm, nb, N, p, o, st)
              : launch_bf16_v4<384, false>(U, ldu, E, enorm, nb, N, p, o, st);
  HVAE_FAIL(HVAE_ERR_UNSUPPORTED, "ab_dec_v4: D=%d", D);
}

int ab_dec_f8v4(bool wo, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                const DecPlan& p, DecOut o, hipStream_t st) {
  return wo ? launch_fp8_v4<true>(U, ldu, E, enorm, nb, N, p, o, st)
            : launch_fp8_v4<false>(U, ldu, E, enorm, nb, N, p, o, st);
}

}  // namespace hvae

using namespace hvae;

#if DEC3_STAMPS
extern "C" int hvae_debug_dec3_stamps(void* out, size_t bytes) {  // diagnostic builds only (not in the ABI)
  HVAE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dec3_stamps), std::min(bytes, sizeof(g_dec3_stamps))));
  return HVAE_OK;
}
#endif
