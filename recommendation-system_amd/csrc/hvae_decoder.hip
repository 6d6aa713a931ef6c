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

#include "hvae_common.h"

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
  const float* kl_rows; float beta; float* loss3; double* accum3; unsigned* ticket;  // fused loss (optional)
};

__global__ void __launch_bounds__(256) k_dec_finalize(FinArgs a) {
  __shared__ float wsh[kMaxSplits];
  __shared__ float red[4];
  __shared__ float pbuf[256];
  __shared__ int any_flag;
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t D = a.D;
  if (tid == 0) any_flag = 0;
  __syncthreads();
  float lse_b;
  float o[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.splits > 1) {
    float M = -INFINITY;
    int fl = 0;
    for (int s = tid; s < a.splits; s += 256) {
      M = fmaxf(M, a.pm[(int64_t)s * a.nb + b]);
      if (a.flag) fl |= a.flag[(int64_t)s * a.nb + b];
    }
    if (fl) any_flag = 1;
    M = wave_max(M);
    if ((tid & 63) == 0) red[tid >> 6] = M;
    __syncthreads();
    M = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    float L = 0.f;
    for (int s = tid; s < a.splits; s += 256) {
      const float ms = a.pm[(int64_t)s * a.nb + b];
      const float wv = (ms == -INFINITY) ? 0.f : __expf(ms - M);
      wsh[s] = wv;
      L += wv * a.pl[(int64_t)s * a.nb + b];
    }
    L = block_sum<256>(L, red);  // its barriers also publish wsh and any_flag
    lse_b = M + logf(L);
    const float inv = 1.0f / L;
    if (a.pO) {
      // sum_s w_s O_s in split order; loads batched 8 splits x 4 columns deep so that
      // they are in flight together (a one-at-a-time chain is HBM-latency bound)
      const int nk = (int)min<int64_t>(4, (D - tid + 255) / 256);
      const int64_t sstride = a.nb * D;
      const float* base = a.pO + b * D + tid;
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      int s0 = 0;
      for (; s0 + 8 <= a.splits; s0 += 8) {
        float v[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) v[j][k] = k < nk ? base[(int64_t)(s0 + j) * sstride + 256 * k] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] += wsh[s0 + j] * v[j][k];
      }
      for (; s0 < a.splits; ++s0)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k < nk) acc[k] += wsh[s0] * base[(int64_t)s0 * sstride + 256 * k];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = acc[k] * inv;
    }
  } else {
    if (a.flag && a.flag[b]) any_flag = 1;
    lse_b = a.lse_in[b];
    if (a.O_in) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t d = tid + 256 * k;
        if (d < D) o[k] = a.O_in[b * D + d];
      }
    }
    __syncthreads();
  }
  if (any_flag) lse_b = exact_user(b, a.U, a.ldu, a.Ebf, a.N, D, o, red, pbuf);  // rare, block-uniform
  if (tid == 0) a.lse_out[b] = lse_b;
  if (a.O_out) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t d = tid + 256 * k;
      if (d < D) a.O_out[b * D + d] = o[k];
    }
  }
  if (!a.row_ptr) return;
  // ---- sparse terms against the fp32 E
  const int64_t r = batch_row(a.rows, a.rows_offset, b);
  const int64_t beg = a.row_ptr[r], end = a.row_ptr[r + 1];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float n = 0.f;
#pragma unroll 4
  for (int64_t e = beg; e < end; ++e) {
    const int64_t j = a.col_idx[e];
    const float x = a.vals[e];
    n += x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t d = tid + 256 * k;
      if (d < D) acc[k] += x * a.E32[j * D + d];
    }
  }
  float dot = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t d = tid + 256 * k;
    if (d < D) dot += a.U[b * a.ldu + d] * acc[k];
  }
  dot = block_sum<256>(dot, red);
  if (a.recon_rows && tid == 0) {
    if (a.loss3) st_shared_f(&a.recon_rows[b], n * lse_b - dot);
    else a.recon_rows[b] = n * lse_b - dot;
  }
  if (a.dU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t d = tid + 256 * k;
      if (d < D) a.dU[b * D + d] = a.scale * (n * o[k] - acc[k]);
    }
  }
  if (a.loss3 && last_block_arrives(a.ticket, gridDim.x))
    loss_block_reduce(a.recon_rows, true, a.kl_rows, a.nb, a.beta, a.loss3, a.accum3);
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

// ------------------------------------------------------------- planning ---
struct DecPlan {
  int splits;
  int64_t tiles_per_split;
  int64_t blocks;
  size_t lds;
};

static DecPlan dec_plan(int dtype, int64_t nb, int64_t N, int64_t D) {
  const int64_t upb = dtype == HVAE_BF16 ? kBfUsersPerBlock : kF32UsersPerBlock;
  const int64_t ti = dtype == HVAE_BF16 ? kBfTI : kF32TI;
  const int64_t target = dtype == HVAE_BF16 ? 256 : 512;
  const int64_t nub = cdiv(nb, upb), tiles = cdiv(N, ti);
  int64_t s = cdiv(target, nub);
  s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / 2));
  s = std::min<int64_t>(s, std::max<int64_t>(1, N / std::max<int64_t>(1, 2 * nb)));
  if (s >= 8) s = s / 8 * 8;
  s = std::max<int64_t>(1, std::min<int64_t>(s, kMaxSplits));
  DecPlan p;
  p.tiles_per_split = cdiv(tiles, s);
  p.splits = (int)cdiv(tiles, p.tiles_per_split);
  if (p.splits >= 8 && p.splits % 8) {  // keep "split shares an XCD" when possible
    const int64_t s8 = (int64_t)p.splits / 8 * 8;
    p.tiles_per_split = cdiv(tiles, s8);
    p.splits = (int)cdiv(tiles, p.tiles_per_split);
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
  if (dtype == HVAE_BF16) {
    switch (D) {
      case 64: return launch_bf16<64, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 128: return launch_bf16<128, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 256: return launch_bf16<256, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      case 384: return launch_bf16<384, WO>(U, ldu, E, enorm, nb, N, p, o, st);
      default: break;
    }
  } else {
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
            dtype == HVAE_BF16 ? "bf16" : "f32", (long long)D);
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_decoder_supported(int dtype, int64_t D) {
  if (dtype == HVAE_BF16) return D == 64 || D == 128 || D == 256 || D == 384;
  if (dtype == HVAE_F32) return D == 32 || D == 64 || D == 128 || D == 256 || D == 384;
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
  return (size_t)et_offset_bytes(N, D) + (size_t)cdiv(N, kBfTI) * D * kBfTI * sizeof(bf16_t);
}

extern "C" int hvae_decoder_image(int dtype, const float* E32, int64_t N, int64_t D, void* out, void* stream) {
  HVAE_REQUIRE(E32 && out && N > 0 && D > 0, "hvae_decoder_image: bad args");
  HVAE_REQUIRE(dtype == HVAE_BF16 || dtype == HVAE_F32, "hvae_decoder_image: bad dtype");
  hipStream_t st = as_stream(stream);
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

extern "C" size_t hvae_decoder_workspace(int dtype, int64_t nb, int64_t N, int64_t D) {
  const DecPlan p = dec_plan(dtype, nb, N, D);
  return dec_ws_bytes(p.splits, nb, D);
}

// flash sweep + finalize; csr / recon_rows / dU optional
static int decoder_run(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                       const float* E32, const hvae_csr_batch* x, int64_t nb, int64_t N, int64_t D, float scale,
                       float* lse, float* O, float* recon_rows, float* dU, const float* kl_rows, float beta,
                       float* loss3, double* accum3, void* ws, size_t ws_bytes, hipStream_t st) {
  HVAE_REQUIRE(dtype == HVAE_BF16 || dtype == HVAE_F32, "hvae decoder: bad dtype");
  HVAE_REQUIRE(U && E && lse && N > 0 && D > 0 && ldu >= D, "hvae decoder: bad args");
  HVAE_REQUIRE(dtype != HVAE_BF16 || e_maxnorm, "hvae decoder: bf16 needs e_maxnorm");
  HVAE_REQUIRE(D <= 1024, "hvae decoder: D > 1024 unsupported");
  HVAE_REQUIRE(ldu % 4 == 0 && ((uintptr_t)U % 16) == 0 && ((uintptr_t)E % 16) == 0 &&
                   (!O || ((uintptr_t)O % 16) == 0),
               "hvae decoder: U/E/O must be 16-B aligned with ldu %% 4 == 0");
  HVAE_REQUIRE(N < (1ll << 31), "hvae decoder: N too large");
  HVAE_REQUIRE(!x || (E32 && x->row_ptr && x->nb == nb && x->n_items == N), "hvae decoder: bad CSR batch");
  if (nb == 0) return HVAE_OK;
  DecPlan p = dec_plan(dtype, nb, N, D);
  if (!ws || ws_bytes < dec_ws_bytes(1, nb, D))
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae decoder: workspace %zu < %zu", ws_bytes, dec_ws_bytes(1, nb, D));
  if (p.splits > 1 && ws_bytes < dec_ws_bytes(p.splits, nb, D)) {  // fewer splits that fit
    int64_t fit = p.splits;
    while (fit > 1 && ws_bytes < dec_ws_bytes((int)fit, nb, D)) fit = fit * 3 / 4;
    const int64_t tiles = cdiv(N, dtype == HVAE_BF16 ? kBfTI : kF32TI);
    p.tiles_per_split = cdiv(tiles, fit);
    p.splits = (int)cdiv(tiles, p.tiles_per_split);
    p.blocks = cdiv(nb, dtype == HVAE_BF16 ? kBfUsersPerBlock : kF32UsersPerBlock) * p.splits;
  }
  const bool bf = dtype == HVAE_BF16;
  const bool want_o = O || dU;
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
  HVAE_REQUIRE(!loss3 || x, "hvae decoder: fused loss needs the batch");
  FinArgs a{};
  a.splits = p.splits;
  if (p.splits > 1) { a.pm = o.m; a.pl = o.l; a.pO = want_o ? o.O : nullptr; }
  else { a.lse_in = lse; a.O_in = o_scratch; }
  a.flag = bf ? o.flag : nullptr;
  a.U = U; a.ldu = ldu; a.Ebf = (const bf16_t*)E;
  a.E32 = E32; a.N = N; a.D = D; a.nb = nb;
  if (x) {
    a.row_ptr = x->row_ptr; a.col_idx = x->col_idx; a.vals = x->vals; a.rows = x->rows;
    a.rows_offset = x->rows_offset;
  }
  a.scale = scale;
  a.lse_out = lse;
  a.O_out = O ? O : (p.splits == 1 ? o_scratch : nullptr);
  a.recon_rows = recon_rows;
  a.dU = dU;
  if (loss3) {
    HVAE_REQUIRE(x && recon_rows && kl_rows, "hvae_decoder_train: fused loss needs recon_rows and kl_rows");
    a.kl_rows = kl_rows; a.beta = beta; a.loss3 = loss3; a.accum3 = accum3;
    if (!(a.ticket = ticket_slice())) return HVAE_ERR_HIP;
  }
  ProbeScope probe("decoder_finalize", st);
  k_dec_finalize<<<(unsigned)nb, 256, 0, st>>>(a);
  HVAE_LAUNCH_CHECK("k_dec_finalize");
  return HVAE_OK;
}

extern "C" int hvae_decoder_fwd(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                                int64_t nb, int64_t N, int64_t D, float* lse, float* O, void* ws,
                                size_t ws_bytes, void* stream) {
  return decoder_run(dtype, U, ldu, E, e_maxnorm, nullptr, nullptr, nb, N, D, 0.f, lse, O, nullptr, nullptr,
                     nullptr, 0.f, nullptr, nullptr, ws, ws_bytes, as_stream(stream));
}

extern "C" int hvae_decoder_train(int dtype, const float* U, int64_t ldu, const void* E, const float* e_maxnorm,
                                  const float* E32, const hvae_csr_batch* x, int64_t D, float grad_scale,
                                  float* lse, float* O, float* recon_rows, float* dU, const float* kl_rows,
                                  float beta, float* loss3, double* accum3, void* ws, size_t ws_bytes,
                                  void* stream) {
  HVAE_REQUIRE(x && recon_rows, "hvae_decoder_train: needs the CSR batch and recon_rows");
  return decoder_run(dtype, U, ldu, E, e_maxnorm, E32, x, x->nb, x->n_items, D, grad_scale, lse, O, recon_rows, dU,
                     kl_rows, beta, loss3, accum3, ws, ws_bytes, as_stream(stream));
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
  k_dec_finalize<<<(unsigned)x->nb, 256, 0, as_stream(stream)>>>(a);
  HVAE_LAUNCH_CHECK("k_dec_finalize");
  return HVAE_OK;
}
