// hvae_gemm.hip -- small dense fp32 GEMMs of the path on the exact-f32 MFMA.
//
// v_mfma_f32_16x16x4_f32: one f32 A and one f32 B per lane, 4 accumulators,
// numerically a k-ordered fmaf chain (no reduced-precision fast path exists
// on gfx950, and none is wanted: these GEMMs carry the fp32 parity of the
// reference's nn.Linear layers). Tile 64x64 or 32x32 per 4-wave block
// (2x2 or 1x1 MFMA tiles per wave); operands staged through LDS in memory
// order; K per block up to 384 loaded in one go; split-K through a caller
// workspace for the tall-skinny weight gradients (K = batch): every split
// block writes its partial tile, and the last block to arrive at a tile
// (device-scope ticket) sums the partials in split order 0..S-1 and applies
// the epilogue -- deterministic, and no second launch.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "hvae_common.h"

namespace hvae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GBK = 32;
// Block tiles BM x BN (64x64 or 32x32), 4 waves as 2x2, each wave (BM/2) x (BN/2) in
// 16x16 MFMA tiles. The 32x32 tile puts 4x more CUs on the batch-sized GEMMs of the
// step (M = 64 users): on the exact-f32 MFMA (256 flop/clk/CU) a 64x64x384 tile alone
// is ~5 us of one CU, so the output must be spread wide.
// LDS images keep each operand in its memory order (no transposing stores):
//   row-major A[m][k] / B^T[n][k]  -> [BM rows][GBK + 2] (float2 stores; fragment reads
//                                     hit banks 2*row + k: conflict-free for ds_read_b32)
//   k-major A^T[k][m] / B[k][n]    -> [GBK rows][BM + 16] (float4 stores)
constexpr int GSR = GBK + 2;  // stride of row-major images
template <int BM>
struct GTile {
  static constexpr int SK = BM + 16;                                  // stride of k-major images
  static constexpr int IMG = (BM * GSR > GBK * SK) ? BM * GSR : GBK * SK;
  static constexpr int LD4 = (BM * GBK / 4 + 255) / 256;             // float4 staged per thread
};
constexpr int kRegStages = 12;  // k-tiles a block keeps in flight at once (K per block <= 384)
// Register-staged k-tiles per instantiation (NST): 12 for k ranges of 5..12 tiles, which load every tile up
// front; 4 for the rest -- k ranges of at most 4 tiles load up front, longer ones stream through a ring of 4
// tiles in flight. The 12-tile staging alone holds 192 VGPRs, so a kernel compiled with it runs one wave per SIMD
// (248 VGPRs + 24 AGPRs at 64 x 64): long-K products (K = d = 768 at the Syn-10M shard) ran with one tile of
// lookahead at that occupancy (MFMA busy 27 %, profiles/r04_pmc_sq_gemm_syn10m_summary.txt).
constexpr int kRingStages = 4;
// The 4-tile ring pays for the x W^T products (row-major A, B^T: the forward layers, K = d = 768: 4096x768x768
// 77 -> 68 us); the [k][n] B of the x W data gradients ran slower on it (4096x768x768 79 -> 82 us), and run on a
// one-stage instance (NST = 1: one tile of lookahead, 83 VGPRs instead of the 12-stage instance's 221, and every
// fragment of a k-tile read before its MFMAs): 4096x768x768 79.98 -> 67.72 us (profiles/r04u_gemm_nn1_ab.jsonl).
static int nst_class(bool ta, bool tb, int64_t kps) {
  const int64_t n = (kps + GBK - 1) / GBK;
  if (n <= kRingStages) return kRingStages;
  if (n <= kRegStages) return kRegStages;
  // (x W^T long k on the one-stage instance measured equal to the ring, and fragment prefetch on the short-k
  // paths changed nothing: profiles/r04v_gemm_prefetch_ab.jsonl)
  if (!ta && tb) return kRingStages;
  const char* e = ab_getenv("HVAE_GEMM_NN1");
  return e && std::atoi(e) == 0 ? kRegStages : 1;
}

struct EpiArgs {
  int kind;
  const float* bias;
  float* pre_out;
  const float* pre_in;
  float p_drop, scale;
  const float* drop_mult;
  uint64_t seed;
  const int64_t* step_dev;
  uint32_t tag;
  int train;
  float* opa_rowsum;  // [M]: sum_k op(A)[m, k] (bias gradient alongside dY^T X)
  const float* aux;   // REPARAM_BWD: eps [M, N]
  float aux_scale;    // REPARAM_BWD: beta / B
  const float* aux_scale_dev;  // REPARAM_BWD: device beta / B (annealed schedule) or NULL
};

__device__ __forceinline__ float epi_apply(const EpiArgs& ep, int64_t step, int64_t row, int64_t col,
                                           int64_t N, int64_t ldc, float c, float* __restrict__ C) {
  switch (ep.kind) {
    case HVAE_EPI_REPARAM_BWD: {  // c = dz; same arithmetic as k_reparam_kl_bwd
      const float m = ep.pre_in[row * ldc + col], v = ep.pre_in[row * ldc + N + col];
      const float gz = ep.train ? c * ep.aux[row * N + col] * 0.5f * expf(0.5f * v) : 0.f;
      const float ks = ep.aux_scale_dev ? *ep.aux_scale_dev : ep.aux_scale;
      C[row * ldc + N + col] = gz + ks * 0.5f * (expf(v) - 1.f);
      return c + ks * m;
    }
    case HVAE_EPI_BIAS:
      return c + ep.bias[col];
    case HVAE_EPI_BIAS_GELU_DROP: {
      const float pre = c + (ep.bias ? ep.bias[col] : 0.f);
      ep.pre_out[row * ldc + col] = pre;
      const float g = gelu_f(pre);
      return ep.train ? g * dropout_mult(ep.p_drop, ep.scale, ep.drop_mult, (uint64_t)(row * N + col),
                                      ep.seed, step, ep.tag)
                      : g;
    }
    case HVAE_EPI_GELU_DROP_BWD: {
      const float dm = ep.train ? dropout_mult(ep.p_drop, ep.scale, ep.drop_mult,
                                            (uint64_t)(row * N + col), ep.seed, step, ep.tag)
                                : 1.f;
      return c * dm * gelu_grad_f(ep.pre_in[row * ldc + col]);
    }
    case HVAE_EPI_DROP_BWD: {
      const float dm = ep.train ? dropout_mult(ep.p_drop, ep.scale, ep.drop_mult,
                                            (uint64_t)(row * N + col), ep.seed, step, ep.tag)
                                : 1.f;
      return c * dm;
    }
    default:
      return c;
  }
}

// Load 4 consecutive elements along the contiguous dimension, zero-filled
// outside [0, lim); vectorised when the caller proved 16-B alignment.
__device__ __forceinline__ float4 load4(const float* __restrict__ p, int64_t idx, int64_t lim, bool vec) {
  if (vec && idx + 3 < lim) return *reinterpret_cast<const float4*>(p);
  float4 r;
  r.x = (idx + 0 < lim) ? p[0] : 0.f;
  r.y = (idx + 1 < lim) ? p[1] : 0.f;
  r.z = (idx + 2 < lim) ? p[2] : 0.f;
  r.w = (idx + 3 < lim) ? p[3] : 0.f;
  return r;
}

// One GEMM problem of a launch (hvae_gemm_f32, or one half of hvae_gemm_f32_pair).
struct GemmP {
  int64_t M, N, K, kps;
  float alpha;
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float beta;
  float* C; int64_t ldc;
  float* slab; unsigned* tickets;
  EpiArgs ep;
  bool vec_a, vec_b;
  unsigned gx, gy, gz;  // tiles along N, along M, k splits
};

template <int BM>
constexpr int gemm_smem_floats() { return 2 * GTile<BM>::IMG; }

// Epilogue of one block tile (acc in the 16x16 MFMA layout, wave (w >> 1, w & 1) of a 2x2 grid): alpha,
// beta, the fused epilogue; with split-K (g.slab) the partial tile goes to the slab and the last block to
// arrive at the tile sums the partials in split order and applies the epilogue.
template <int BM, int BN>
__device__ __forceinline__ void gemm_finish(const GemmP& g, const f32x4 (&acc)[BM / 32][BN / 32], unsigned bx,
                                            unsigned by, unsigned bz, bool do_rowsum, float rowsum) {
  constexpr int IM = BM / 32, JN = BN / 32;
  const int64_t M = g.M, N = g.N, ldc = g.ldc;
  const float alpha = g.alpha, beta = g.beta;
  float* __restrict__ C = g.C;
  float* __restrict__ slab = g.slab;
  unsigned* __restrict__ tickets = g.tickets;
  const EpiArgs& ep = g.ep;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t m0 = (int64_t)by * BM, n0 = (int64_t)bx * BN;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  if (do_rowsum && t < BM && m0 + t < M) {
    if (slab) st_shared_f(&slab[(int64_t)g.gz * M * N + (int64_t)bz * M + m0 + t], rowsum);
    else ep.opa_rowsum[m0 + t] = alpha * rowsum;
  }
  const int64_t step = (ep.kind >= HVAE_EPI_BIAS_GELU_DROP && ep.kind <= HVAE_EPI_DROP_BWD) ? load_step(ep.step_dev) : 0;
  if (!slab) {
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = m0 + wm + i * 16 + 4 * (lane >> 4) + r;
          const int64_t col = n0 + wn + j * 16 + (lane & 15);
          if (row >= M || col >= N) continue;
          float c = alpha * acc[i][j][r];
          if (beta != 0.f) c += beta * C[row * ldc + col];
          C[row * ldc + col] = epi_apply(ep, step, row, col, N, ldc, c, C);
        }
    return;
  }
  // ---- split-K: publish the partial tile, the last arrival reduces
  const unsigned tile = by * g.gx + bx;
  if (M % BM == 0 && N % BN == 0) {
    // whole tiles: the partials in fragment order, one 16-B coherent store per accumulator (a dword sc1 store
    // costs ~6x a dwordx4 per byte), read back by the same thread of the last block in split order -- the same
    // sums in the same order as the element-order slab below
    constexpr int FR = IM * JN * 4;
    const int64_t ntile = (int64_t)g.gx * g.gy;
    const __amdgpu_buffer_rsrc_t srs = coherent_rsrc(slab);
    const uint32_t mine = (uint32_t)((((int64_t)bz * ntile + tile) * (BM * BN) + (int64_t)t * FR) * 4);
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
        st_sc1_f4(srs, mine + 16u * (i * JN + j), make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]));
    if (!last_block_arrives(&tickets[tile], g.gz)) return;
    const int S = (int)g.gz;
    f32x4 sum[IM][JN];
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) sum[i][j][r] = 0.f;
    for (int z = 0; z < S; ++z) {
      const uint32_t src = (uint32_t)((((int64_t)z * ntile + tile) * (BM * BN) + (int64_t)t * FR) * 4);
      float4 v[IM][JN];  // every load of the split in flight together
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) v[i][j] = ld_sc1_f4(srs, src + 16u * (i * JN + j));
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          sum[i][j][0] += v[i][j].x; sum[i][j][1] += v[i][j].y; sum[i][j][2] += v[i][j].z; sum[i][j][3] += v[i][j].w;
        }
    }
#pragma unroll
    for (int i = 0; i < IM; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = m0 + wm + i * 16 + 4 * (lane >> 4) + r;
          const int64_t col = n0 + wn + j * 16 + (lane & 15);
          float c = alpha * sum[i][j][r];
          if (beta != 0.f) c += beta * C[row * ldc + col];
          C[row * ldc + col] = epi_apply(ep, step, row, col, N, ldc, c, C);
        }
    if (ep.opa_rowsum && bx == 0 && t < BM && m0 + t < M) {
      float r = 0.f;
      for (int z = 0; z < S; ++z) r += ld_shared_f(&slab[(int64_t)S * M * N + (int64_t)z * M + m0 + t]);
      ep.opa_rowsum[m0 + t] = alpha * r;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm + i * 16 + 4 * (lane >> 4) + r;
        const int64_t col = n0 + wn + j * 16 + (lane & 15);
        if (row < M && col < N) st_shared_f(&slab[((int64_t)bz * M + row) * N + col], acc[i][j][r]);
      }
  if (!last_block_arrives(&tickets[tile], g.gz)) return;
  // the tile's elements per thread: one coherent load each per split, all in flight together
  constexpr int Q = BM * BN / 256;
  const int S = (int)g.gz;
  float sum[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) sum[q] = 0.f;
  for (int z = 0; z < S; ++z) {
    float v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = t + 256 * q;
      const int64_t row = m0 + e / BN, col = n0 + e % BN;
      v[q] = (row < M && col < N) ? ld_shared_f(&slab[((int64_t)z * M + row) * N + col]) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) sum[q] += v[q];
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int e = t + 256 * q;
    const int64_t row = m0 + e / BN, col = n0 + e % BN;
    if (row >= M || col >= N) continue;
    float c = alpha * sum[q];
    if (beta != 0.f) c += beta * C[row * ldc + col];
    C[row * ldc + col] = epi_apply(ep, step, row, col, N, ldc, c, C);
  }
  if (ep.opa_rowsum && bx == 0 && t < BM && m0 + t < M) {
    float r = 0.f;
    for (int z = 0; z < S; ++z) r += ld_shared_f(&slab[(int64_t)S * M * N + (int64_t)z * M + m0 + t]);
    ep.opa_rowsum[m0 + t] = alpha * r;
  }
}

// The block (bx, by, bz) of problem g: tile rows by*BM.., columns bx*BN.., k split bz.
template <bool TA, bool TB, int BM, int BN, int NST>
__device__ __forceinline__ void gemm_block(const GemmP& g, unsigned bx, unsigned by, unsigned bz,
                                           float* __restrict__ sA_, float* __restrict__ sB_) {
  using TAo = GTile<BM>;
  using TBo = GTile<BN>;
  constexpr int IM = BM / 32, JN = BN / 32;  // 16x16 MFMA tiles per wave
  const int64_t M = g.M, N = g.N, K = g.K, k_per_split = g.kps, lda = g.lda, ldb = g.ldb, ldc = g.ldc;
  const float alpha = g.alpha, beta = g.beta;
  const float* __restrict__ A = g.A;
  const float* __restrict__ B = g.B;
  float* __restrict__ C = g.C;
  float* __restrict__ slab = g.slab;
  unsigned* __restrict__ tickets = g.tickets;
  const EpiArgs& ep = g.ep;
  const bool vec_a = g.vec_a, vec_b = g.vec_b;
  auto sA = [&](int buf) { return sA_ + buf * TAo::IMG; };
  auto sB = [&](int buf) { return sB_ + buf * TBo::IMG; };
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t m0 = (int64_t)by * BM, n0 = (int64_t)bx * BN;
  const int64_t kb = (int64_t)bz * k_per_split;
  const int64_t ke = min(K, kb + k_per_split);
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);

  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool do_rowsum = ep.opa_rowsum != nullptr && bx == 0;
  float rowsum = 0.f;  // thread t < BM: sum over this block's k range of op(A)[m0 + t][k]
  // Operand element (r = m or n, k): row-major sources stage f -> (r = f / (GBK/4), k = 4 (f % (GBK/4)));
  // k-major sources stage f -> (k = f / (R/4), r = 4 (f % (R/4))).
  constexpr int KQ = GBK / 4, MQ = BM / 4, NQ = BN / 4;
  constexpr int LA = TAo::LD4, LB = TBo::LD4;
  auto gload = [&](int64_t k0, float4 (&ra)[LA], float4 (&rb)[LB]) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int f = t + 256 * i;
      if (!TA) {
        const int64_t m = m0 + f / KQ, k = k0 + (f % KQ) * 4;
        ra[i] = (m < M) ? load4(A + m * lda + k, k, ke, vec_a) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        const int64_t k = k0 + f / MQ, m = m0 + (f % MQ) * 4;
        ra[i] = (k < ke) ? load4(A + k * lda + m, m, M, vec_a) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int f = t + 256 * i;
      if (!TB) {
        const int64_t k = k0 + f / NQ, n = n0 + (f % NQ) * 4;
        rb[i] = (k < ke) ? load4(B + k * ldb + n, n, N, vec_b) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        const int64_t n = n0 + f / KQ, k = k0 + (f % KQ) * 4;
        rb[i] = (n < N) ? load4(B + n * ldb + k, k, ke, vec_b) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  auto lstore = [&](int buf, const float4 (&ra)[LA], const float4 (&rb)[LB]) {
    float* a_ = sA(buf);
    float* b_ = sB(buf);
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int f = t + 256 * i;
      if (!TA) {
        float* d = &a_[(f / KQ) * GSR + (f % KQ) * 4];
        *reinterpret_cast<float2*>(d) = make_float2(ra[i].x, ra[i].y);
        *reinterpret_cast<float2*>(d + 2) = make_float2(ra[i].z, ra[i].w);
      } else {
        *reinterpret_cast<float4*>(&a_[(f / MQ) * TAo::SK + (f % MQ) * 4]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int f = t + 256 * i;
      if (!TB) {
        *reinterpret_cast<float4*>(&b_[(f / NQ) * TBo::SK + (f % NQ) * 4]) = rb[i];
      } else {
        float* d = &b_[(f / KQ) * GSR + (f % KQ) * 4];
        *reinterpret_cast<float2*>(d) = make_float2(rb[i].x, rb[i].y);
        *reinterpret_cast<float2*>(d + 2) = make_float2(rb[i].z, rb[i].w);
      }
    }
  };
  // one staged k-tile: MFMA chain in k order (+ the fused row sums)
  auto compute = [&](int buf) {
    const float* a_ = sA(buf);
    const float* b_ = sB(buf);
    auto a_at = [&](int m, int k) -> float { return TA ? a_[k * TAo::SK + m] : a_[m * GSR + k]; };
    auto b_at = [&](int k, int n) -> float { return TB ? b_[n * GSR + k] : b_[k * TBo::SK + n]; };
    if (do_rowsum && t < BM) {
#pragma unroll
      for (int k = 0; k < GBK; ++k) rowsum += a_at(t, k);
    }
#pragma unroll
    for (int kk = 0; kk < GBK / 4; ++kk) {
      const int kr = 4 * kk + (lane >> 4);
      float af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = a_at(wm + i * 16 + (lane & 15), kr);
#pragma unroll
      for (int j = 0; j < JN; ++j) bfr[j] = b_at(kr, wn + j * 16 + (lane & 15));
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // the long-k loop's stage: every fragment of the k-tile read before its MFMAs (the LDS latency once per tile
  // instead of once per 4 MFMAs behind an lgkmcnt(0)), used where the instantiation leaves the registers (NST = 1)
  auto compute_pf = [&](int buf) {
    const float* a_ = sA(buf);
    const float* b_ = sB(buf);
    auto a_at = [&](int m, int k) -> float { return TA ? a_[k * TAo::SK + m] : a_[m * GSR + k]; };
    auto b_at = [&](int k, int n) -> float { return TB ? b_[n * GSR + k] : b_[k * TBo::SK + n]; };
    if (do_rowsum && t < BM) {
#pragma unroll
      for (int k = 0; k < GBK; ++k) rowsum += a_at(t, k);
    }
    float af[GBK / 4][IM], bfr[GBK / 4][JN];
#pragma unroll
    for (int kk = 0; kk < GBK / 4; ++kk) {
      const int kr = 4 * kk + (lane >> 4);
#pragma unroll
      for (int i = 0; i < IM; ++i) af[kk][i] = a_at(wm + i * 16 + (lane & 15), kr);
#pragma unroll
      for (int j = 0; j < JN; ++j) bfr[kk][j] = b_at(kr, wn + j * 16 + (lane & 15));
    }
#pragma unroll
    for (int kk = 0; kk < GBK / 4; ++kk)
#pragma unroll
      for (int i = 0; i < IM; ++i)
#pragma unroll
        for (int j = 0; j < JN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
  };

  const int64_t nst = (ke > kb) ? (ke - kb + GBK - 1) / GBK : 0;
  if (nst > 0 && nst <= NST) {
    // short k range (the batch-sized GEMMs of the path): every global load of the block is issued
    // up front -- one memory latency instead of one per k-tile -- then the tiles stream through
    // double-buffered LDS with one barrier each
    float4 ra[NST][LA], rb[NST][LB];
#pragma unroll
    for (int st = 0; st < NST; ++st)
      if (st < nst) gload(kb + (int64_t)st * GBK, ra[st], rb[st]);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st < nst) {
        lstore(st & 1, ra[st], rb[st]);
        __syncthreads();
        compute(st & 1);
      }
    }
  } else if (nst > 0 && NST != kRingStages) {
    // long k range, one k-tile of lookahead (the kRegStages instantiation keeps its registers for the short path)
    float4 ra[LA], rb[LB];
    gload(kb, ra, rb);
    lstore(0, ra, rb);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += GBK) {
      const bool more = k0 + GBK < ke;
      if (more) gload(k0 + GBK, ra, rb);
      if (NST == 1) compute_pf(buf);
      else compute(buf);
      if (more) {
        lstore(buf ^ 1, ra, rb);
        __syncthreads();
        buf ^= 1;
      }
    }
  } else if (nst > 0) {
    // long k range: a ring of NST register-staged k-tiles, each slot refilled NST tiles ahead as soon as it
    // has been copied to LDS (LDS buffer st & 1 was last read by compute(st - 2), which every wave finished
    // before the barrier of st - 1)
    float4 ra[NST][LA], rb[NST][LB];
#pragma unroll
    for (int u = 0; u < NST; ++u) gload(kb + (int64_t)u * GBK, ra[u], rb[u]);
    for (int64_t st0 = 0; st0 < nst; st0 += NST) {
#pragma unroll
      for (int u = 0; u < NST; ++u) {
        const int64_t st = st0 + u;
        if (st < nst) {
          lstore((int)(st & 1), ra[u], rb[u]);
          __syncthreads();
          if (st + NST < nst) gload(kb + (st + NST) * GBK, ra[u], rb[u]);
          compute((int)(st & 1));
        }
      }
    }
  }

  gemm_finish<BM, BN>(g, acc, bx, by, bz, do_rowsum, rowsum);
}

// ------------------------------------------------------------ fast path ---
// Tiles that divide the problem (M % BM == N % BN == 0, every k range a multiple of 32, 16-B aligned
// operands with ld % 4 == 0 -- the batch GEMMs of the train step at B = 4096 or 64): no bounds checks,
// one barrier per 32-deep k stage, the next stage's global loads in flight under the current stage's
// MFMAs, and 128-bit fragment reads. Both operands are staged into the same LDS image whatever their
// memory order: [8 k-chunks][R rows][4 k], so a lane (row r, k-group q) reads four consecutive k of its
// row with one ds_read_b128. k-contiguous sources ([r][k]) are copied 16 B at a time; r-contiguous ones
// ([k][r], the fast path's operands) are transposed in the store (4 ds_write_b32 per float4).
// Banks (scripts/check_gemm_banks.py): a chunk stride of R rows (a multiple of 16 float4) keeps the q = 1
// lanes of each ds_read_b128 lane group ({0-3, 12-15, 20-27}, ...) off the q = 0 lanes' banks, and row r
// sits in slot r ^ ((r >> 3) & 3) of its chunk, so the four rows a store lane holds land on 16 distinct
// banks across a 16-row half-wave. FAST_LAYOUT 0 is the first image (R + 4 stride, no swizzle).
// MFMA order: the 16x16x4 MFMA (s) of 16-k group j sums k = 16 j + 4 q + s over the lane groups q,
// so the four k of a lane's float4 feed four consecutive MFMAs. Each k still enters the accumulator
// exactly once, in a fixed order (deterministic, exact fp32 products and fp32 accumulation).
constexpr int FBK = 32;
#ifndef FAST_PREFETCH
#define FAST_PREFETCH 4  // k stages of global loads in flight per thread
#endif
#ifndef FAST_LAYOUT
#define FAST_LAYOUT 1
#endif
template <int R>
struct FImg {
  static constexpr int CS = FAST_LAYOUT ? R : R + 4;  // float4 slots per k-chunk
  static __device__ __forceinline__ int slot(int r) { return FAST_LAYOUT ? r ^ ((r >> 3) & 3) : r; }
  static constexpr int F4 = (FBK / 4) * CS;    // float4 slots per image
  static constexpr int LD = R * FBK / 4 / 256; // float4 global loads per thread per stage
  static_assert(R * FBK / 4 % 256 == 0, "tile rows x 32 must be a multiple of 1024 floats");
};

// one operand of one stage: rows r0.., k0.. of a k-contiguous (KC) or row-contiguous source
template <bool KC, int R>
__device__ __forceinline__ void fast_gload(const float* __restrict__ X, int64_t ld, int64_t r0, int64_t k0,
                                           float4 (&v)[FImg<R>::LD]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < FImg<R>::LD; ++i) {
    const int f = t + 256 * i;
    if (KC) {  // [r][k]: 8 threads per row, 128 contiguous bytes
      const int r = f >> 3, c = f & 7;
      v[i] = *reinterpret_cast<const float4*>(X + (r0 + r) * ld + k0 + 4 * c);
    } else {   // [k][r]: R/4 threads per k row
      const int k = f / (R / 4), r4 = f % (R / 4);
      v[i] = *reinterpret_cast<const float4*>(X + (k0 + k) * ld + r0 + 4 * r4);
    }
  }
}

template <bool KC, int R>
__device__ __forceinline__ void fast_lstore(float4* __restrict__ img, const float4 (&v)[FImg<R>::LD]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < FImg<R>::LD; ++i) {
    const int f = t + 256 * i;
    if (KC) {
      const int r = f >> 3, c = f & 7;
      img[c * FImg<R>::CS + FImg<R>::slot(r)] = v[i];
    } else {
      const int k = f / (R / 4), r4 = f % (R / 4);
      float* d = reinterpret_cast<float*>(img + (k >> 2) * FImg<R>::CS) + (k & 3);
      d[4 * FImg<R>::slot(4 * r4)] = v[i].x;
      d[4 * FImg<R>::slot(4 * r4 + 1)] = v[i].y;
      d[4 * FImg<R>::slot(4 * r4 + 2)] = v[i].z;
      d[4 * FImg<R>::slot(4 * r4 + 3)] = v[i].w;
    }
  }
}

template <bool TA, bool TB, int BM, int BN>
__device__ __forceinline__ void gemm_fast_block(const GemmP& g, unsigned bx, unsigned by, unsigned bz,
                                                float4* __restrict__ smem) {
  constexpr int IM = BM / 32, JN = BN / 32;
  using IA = FImg<BM>;
  using IB = FImg<BN>;
  float4* sA[2] = {smem, smem + IA::F4};
  float4* sB[2] = {smem + 2 * IA::F4, smem + 2 * IA::F4 + IB::F4};
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t m0 = (int64_t)by * BM, n0 = (int64_t)bx * BN;
  const int64_t kb = (int64_t)bz * g.kps;
  const int nst = (int)((min(g.K, kb + g.kps) - kb) / FBK);
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const int q = lane >> 4, c16 = lane & 15;
  const bool do_rowsum = g.ep.opa_rowsum != nullptr && bx == 0;
  float rowsum = 0.f;

  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // a ring of FP stages of register-staged global loads (the k range's first FP stages issued at once,
  // each slot refilled FP stages ahead as soon as it has been copied to LDS)
  constexpr int FP = FAST_PREFETCH;
  float4 ra[FP][IA::LD], rb[FP][IB::LD];
  // A: op(A)[m][k] is A[m][k] (k-contiguous) unless TA; B: op(B)[k][n] is B[n][k] (k-contiguous) if TB
  auto gload = [&](int st, float4 (&xa)[IA::LD], float4 (&xb)[IB::LD]) {
    const int64_t k0 = kb + (int64_t)st * FBK;
    if (TA) fast_gload<false, BM>(g.A, g.lda, m0, k0, xa);
    else fast_gload<true, BM>(g.A, g.lda, m0, k0, xa);
    if (TB) fast_gload<true, BN>(g.B, g.ldb, n0, k0, xb);
    else fast_gload<false, BN>(g.B, g.ldb, n0, k0, xb);
  };
  auto lstore = [&](int buf, const float4 (&xa)[IA::LD], const float4 (&xb)[IB::LD]) {
    if (TA) fast_lstore<false, BM>(sA[buf], xa);
    else fast_lstore<true, BM>(sA[buf], xa);
    if (TB) fast_lstore<true, BN>(sB[buf], xb);
    else fast_lstore<false, BN>(sB[buf], xb);
  };
  auto compute = [&](int buf) {
    const float4* a_ = sA[buf];
    const float4* b_ = sB[buf];
    if (do_rowsum && t < BM) {
#pragma unroll
      for (int c = 0; c < FBK / 4; ++c) {
        const float4 x = sA[buf][c * IA::CS + IA::slot(t)];
        rowsum += x.x;
        rowsum += x.y;
        rowsum += x.z;
        rowsum += x.w;
      }
    }
#pragma unroll
    for (int j = 0; j < FBK / 16; ++j) {
      float4 af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) af[i] = a_[(4 * j + q) * IA::CS + IA::slot(wm + c16 + 16 * i)];
#pragma unroll
      for (int n = 0; n < JN; ++n) bfr[n] = b_[(4 * j + q) * IB::CS + IB::slot(wn + c16 + 16 * n)];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
          for (int n = 0; n < JN; ++n)
            acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bfr[n][s], acc[i][n], 0, 0, 0);
    }
  };

  // stage st: copy slot st % FP to LDS buffer st & 1, barrier, refill the slot with stage st + FP, MFMAs.
  // LDS buffer b was last read by compute(st - 2), which every wave finished before the barrier of st - 1.
#pragma unroll
  for (int u = 0; u < FP; ++u)
    if (u < nst) gload(u, ra[u], rb[u]);
  for (int st0 = 0; st0 < nst; st0 += FP) {
#pragma unroll
    for (int u = 0; u < FP; ++u) {
      const int st = st0 + u;
      if (st < nst) {
        lstore(st & 1, ra[u], rb[u]);
        __syncthreads();
        if (st + FP < nst) gload(st + FP, ra[u], rb[u]);
        compute(st & 1);
      }
    }
  }
  gemm_finish<BM, BN>(g, acc, bx, by, bz, do_rowsum, rowsum);
}

template <int BM, int BN>
constexpr int fast_smem_f4() { return 2 * (FImg<BM>::F4 + FImg<BN>::F4); }

// ------------------------------------------------------------- LDS-DMA path ---
// The whole-tile case of both kernels above (M % BM == N % BN == 0, k ranges multiples of 32, 16-B aligned
// operands, ld % 4 == 0 -- every GEMM of the train step at B = 4096), with the operands copied from global
// memory straight into LDS by buffer_load_dwordx4 ... lds (no register staging, no ds_write), a ring of DNS
// 32-deep k stages, one barrier per stage. Registers drop to the accumulators and fragments, so blocks of
// three or four per CU overlap each other's waits (the register-staged kernel ran one wave per SIMD at
// K = 768: MFMA busy 27 %, profiles/r04_pmc_sq_gemm_syn10m_summary.txt). Per operand and stage the tile is
// R x 32 floats = R / 8 one-KiB pieces, issued by the block's waves in turn. LDS images:
//   k-contiguous source ([r][k]: A, or B^T under TB) -- the fast path's image [8 k-chunks][R slots][4 k]:
//     piece lane i fills slot e = 64 p + i of chunk e / R from row slot^-1(e % R) (the XOR slot map is its own
//     inverse), so the swizzle costs nothing; fragments as the fast path, one ds_read_b128 per 4 MFMAs;
//   r-contiguous source ([k][r]: A^T under TA, or B): [32 k][R] floats with the 16-B chunk index XORed by
//     4 ((k >> 2) & 1), so the k = 16 j + 4 q + s rows a ds_read_b32 lane group reads (q = 0, 1 | 2, 3) land
//     on disjoint bank halves; one ds_read_b32 per MFMA.
// The k order (MFMA s of 16-k group j sums k = 16 j + 4 q + s over the lane groups q) and the accumulator
// layout are the fast path's, so gemm_finish (epilogues, split-K) is shared.
#ifndef GEMM_DNS
#define GEMM_DNS 2  // ring depth: 2 stages (32 KiB a 64 x 64 block, five blocks per CU) against 3 / 4 at the
                    // Syn-10M shapes: 269 / 276 / 292 us summed (profiles/r05_gemm_dma_tuning.txt) -- more blocks
                    // per CU hide the fill better than a deeper ring in fewer blocks
#endif
constexpr int DNS = GEMM_DNS;
template <int R>
struct DImg {
  static constexpr int BYTES = R * FBK * 4;  // one operand, one stage (either layout)
  static constexpr int PIECES = BYTES / 1024;
  static_assert(PIECES % 4 == 0, "pieces per operand and stage: a multiple of the block's 4 waves");
};

template <int i>
__device__ __forceinline__ void gemm_dma_piece(uint32_t m0, int voff, __amdgpu_buffer_rsrc_t rsrc, uint32_t soff) {
  // M0 and soffset come in computed (an s_add in the asm would write SCC behind the compiler's back; the
  // instruction's offset field would move the LDS destination too); the first piece of a group waits out the
  // readfirstlane of its SGPR operands. M0 is not in the clobber list on purpose: the AMDGPU backend reserves it
  // (never allocates it to an "s" operand, and re-initialises it before each of its own M0 uses), and it rejects
  // reserved registers there ("clobbering them may lead to undefined behaviour", -Winline-asm)
  if constexpr (i == 0)
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(m0), "v"(voff), "s"(rsrc), "s"(soff) : "memory");
  else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 :: "s"(m0), "v"(voff), "s"(rsrc), "s"(soff) : "memory");
}

template <int n>
__device__ __forceinline__ void gemm_wait_vmcnt() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14));
}

// lane offsets of this wave's pieces of one operand (bytes from the tile's first element at stage 0)
template <bool KC, int R>
__device__ __forceinline__ void dma_lane_offsets(int64_t ld, int (&voff)[DImg<R>::PIECES / 4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < DImg<R>::PIECES / 4; ++u) {
    const int p = w + 4 * u;
    const int e = 64 * p + lane;  // float4 slot of the image
    if (KC) {
      const int c = e / R, sl = e % R;
      const int r = FImg<R>::slot(sl);  // the slot map is an involution
      voff[u] = (int)((int64_t)r * ld * 4 + 16 * c);
    } else {
      const int k = e / (R / 4), d = e % (R / 4);
      const int c = d ^ (4 * ((k >> 2) & 1));
      voff[u] = (int)((int64_t)k * ld * 4 + 16 * c);
    }
  }
}

template <bool TA, bool TB, int BM, int BN>
__device__ __forceinline__ void gemm_dma_block(const GemmP& g, unsigned bx, unsigned by, unsigned bz,
                                               unsigned char* __restrict__ smem) {
  constexpr int IM = BM / 32, JN = BN / 32;
  constexpr bool AKC = !TA, BKC = TB;  // k-contiguous sources
  constexpr int SA = DImg<BM>::BYTES, SB = DImg<BN>::BYTES, STAGE = SA + SB;
  constexpr int PA = DImg<BM>::PIECES / 4, PB = DImg<BN>::PIECES / 4;  // pieces per wave and stage
  constexpr int P = PA + PB;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t m0 = (int64_t)by * BM, n0 = (int64_t)bx * BN;
  const int64_t kb = (int64_t)bz * g.kps;
  const int nst = (int)((min(g.K, kb + g.kps) - kb) / FBK);
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  const int q = lane >> 4, c16 = lane & 15;
  const bool do_rowsum = g.ep.opa_rowsum != nullptr && bx == 0;
  float rowsum = 0.f;

  // buffer resources over each operand's whole extent (byte offsets stay below 2^31: checked on the host)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.A), (short)0, 0x7fffffff,
                                                                      0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.B), (short)0, 0x7fffffff,
                                                                      0x00020000);
  int va[PA], vb[PB];
  dma_lane_offsets<AKC, BM>(g.lda, va);
  dma_lane_offsets<BKC, BN>(g.ldb, vb);
  // the tile's origin (stage 0) and the per-stage step, in bytes
  const int64_t a0 = AKC ? (m0 * g.lda + kb) * 4 : (kb * g.lda + m0) * 4;
  const int64_t b0 = BKC ? (n0 * g.ldb + kb) * 4 : (kb * g.ldb + n0) * 4;
  const int64_t ast = AKC ? FBK * 4 : (int64_t)FBK * g.lda * 4;
  const int64_t bst = BKC ? FBK * 4 : (int64_t)FBK * g.ldb * 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)smem;

  auto issue = [&](int st) {
    const int slot = st % DNS;
    const uint32_t la = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + slot * STAGE + w * 1024));
    const uint32_t lb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + slot * STAGE + SA + w * 1024));
    const uint32_t sa = (uint32_t)__builtin_amdgcn_readfirstlane((int)(a0 + st * ast));
    const uint32_t sb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(b0 + st * bst));
    gemm_dma_piece<0>(la, va[0], ra, sa);
#pragma unroll
    for (int u = 1; u < PA; ++u) gemm_dma_piece<1>(la + 4096u * u, va[u], ra, sa);
#pragma unroll
    for (int u = 0; u < PB; ++u) gemm_dma_piece<1>(lb + 4096u * u, vb[u], rb, sb);
  };

  f32x4 acc[IM][JN];
#pragma unroll
  for (int i = 0; i < IM; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int slot) {
    const unsigned char* ia = smem + slot * STAGE;
    const unsigned char* ib = ia + SA;
    const float4* a4 = reinterpret_cast<const float4*>(ia);
    const float4* b4 = reinterpret_cast<const float4*>(ib);
    const float* a1 = reinterpret_cast<const float*>(ia);
    const float* b1 = reinterpret_cast<const float*>(ib);
    if (do_rowsum && t < BM) {  // sum_k op(A)[m, k] of this stage, m = m0 + t
      if (AKC) {
#pragma unroll
        for (int c = 0; c < FBK / 4; ++c) {
          const float4 x = a4[c * BM + FImg<BM>::slot(t)];
          rowsum += x.x;
          rowsum += x.y;
          rowsum += x.z;
          rowsum += x.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < FBK; ++k) rowsum += a1[k * BM + 4 * ((t >> 2) ^ (4 * ((k >> 2) & 1))) + (t & 3)];
      }
    }
#pragma unroll
    for (int j = 0; j < FBK / 16; ++j) {
      float4 af[IM], bfr[JN];
#pragma unroll
      for (int i = 0; i < IM; ++i) {
        const int x = wm + c16 + 16 * i;
        if (AKC) {
          af[i] = a4[(4 * j + q) * BM + FImg<BM>::slot(x)];
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            const int k = 16 * j + 4 * q + s2;
            (&af[i].x)[s2] = a1[k * BM + 4 * ((x >> 2) ^ (4 * ((k >> 2) & 1))) + (x & 3)];
          }
        }
      }
#pragma unroll
      for (int n = 0; n < JN; ++n) {
        const int x = wn + c16 + 16 * n;
        if (BKC) {
          bfr[n] = b4[(4 * j + q) * BN + FImg<BN>::slot(x)];
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            const int k = 16 * j + 4 * q + s2;
            (&bfr[n].x)[s2] = b1[k * BN + 4 * ((x >> 2) ^ (4 * ((k >> 2) & 1))) + (x & 3)];
          }
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int i = 0; i < IM; ++i)
#pragma unroll
          for (int n = 0; n < JN; ++n)
            acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x4f32((&af[i].x)[s2], (&bfr[n].x)[s2], acc[i][n], 0, 0, 0);
    }
  };

  // ring: stages 0 .. DNS - 2 in flight before the loop; stage st + DNS - 1 is issued into the slot that
  // compute(st - 1) freed, right after the barrier that proves every wave is past it
#pragma unroll
  for (int u = 0; u < DNS - 1; ++u)
    if (u < nst) issue(u);
  for (int st = 0; st < nst; ++st) {
    if (st + DNS - 2 < nst) gemm_wait_vmcnt<P * (DNS - 2)>();  // this wave's pieces of stage st have landed
    else gemm_wait_vmcnt<0>();
    __syncthreads();
    if (st + DNS - 1 < nst) issue(st + DNS - 1);
    compute(st % DNS);
  }
  gemm_finish<BM, BN>(g, acc, bx, by, bz, do_rowsum, rowsum);
}

template <int BM, int BN>
constexpr int dma_smem_bytes() { return DNS * (DImg<BM>::BYTES + DImg<BN>::BYTES); }

template <bool TA, bool TB, int BM, int BN>
__global__ void __launch_bounds__(256) k_gemm_dma(GemmP g) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[dma_smem_bytes<BM, BN>()];
  gemm_dma_block<TA, TB, BM, BN>(g, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// a layer's backward pair (dW = dY^T X split-K, dX = dY W) both on the LDS-DMA path, in one launch
template <int BM0, int BM1>
__global__ void __launch_bounds__(256) k_gemm_dma_pair(GemmP g0, GemmP g1) {
  constexpr int S0 = dma_smem_bytes<BM0, BM0>(), S1 = dma_smem_bytes<BM1, BM1>();
  __shared__ __attribute__((aligned(1024))) unsigned char smem[S0 > S1 ? S0 : S1];
  const unsigned nb0 = g0.gx * g0.gy * g0.gz;
  unsigned b = blockIdx.x;
  if (b < nb0) {
    gemm_dma_block<true, false, BM0, BM0>(g0, b % g0.gx, (b / g0.gx) % g0.gy, b / (g0.gx * g0.gy), smem);
  } else {
    b -= nb0;
    gemm_dma_block<false, false, BM1, BM1>(g1, b % g1.gx, (b / g1.gx) % g1.gy, b / (g1.gx * g1.gy), smem);
  }
}

template <bool TA, bool TB, int BM, int BN>
__global__ void __launch_bounds__(256) k_gemm_fast(GemmP g) {
  __shared__ float4 smem[fast_smem_f4<BM, BN>()];
  gemm_fast_block<TA, TB, BM, BN>(g, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// the (dW = dY^T X, dX = dY W) pair of a layer's backward: the weight gradient (long K, split-K) on the
// fast path in F0 x F0 tiles, the data gradient (short K) on the register-staged kernel in BT1 x BT1 tiles
template <int F0, int BT1, int NST1>
__global__ void __launch_bounds__(256) k_gemm_mixed_pair(GemmP g0, GemmP g1) {
  constexpr int S0 = fast_smem_f4<F0, F0>() * 4, S1 = gemm_smem_floats<BT1>() * 2;
  __shared__ __attribute__((aligned(16))) float smem[S0 > S1 ? S0 : S1];
  const unsigned n0 = g0.gx * g0.gy * g0.gz;
  unsigned b = blockIdx.x;
  if (b < n0) {
    gemm_fast_block<true, false, F0, F0>(g0, b % g0.gx, (b / g0.gx) % g0.gy, b / (g0.gx * g0.gy),
                                         reinterpret_cast<float4*>(smem));
  } else {
    b -= n0;
    gemm_block<false, false, BT1, BT1, NST1>(g1, b % g1.gx, (b / g1.gx) % g1.gy, b / (g1.gx * g1.gy), smem,
                                       smem + gemm_smem_floats<BT1>());
  }
}

template <bool TA, bool TB, int BM, int BN, int NST>
__global__ void __launch_bounds__(256) k_gemm_f32(GemmP g) {
  __shared__ __attribute__((aligned(16))) float sA[gemm_smem_floats<BM>()];
  __shared__ __attribute__((aligned(16))) float sB[gemm_smem_floats<BN>()];
  gemm_block<TA, TB, BM, BN, NST>(g, blockIdx.x, blockIdx.y, blockIdx.z, sA, sB);
}

// Two independent GEMMs in one launch (a weight gradient dW = dY^T X and the data gradient
// dX = dY W of one layer): the first g0.gx*g0.gy*g0.gz blocks run g0, the rest g1. Both depend
// only on inputs already complete, so the launch costs max(t0, t1) instead of t0 + t1 plus a
// kernel boundary.
template <int BM0, int BM1, int NST0, int NST1>
__global__ void __launch_bounds__(256) k_gemm_f32_pair(GemmP g0, GemmP g1) {
  constexpr int SA = gemm_smem_floats<BM0>() > gemm_smem_floats<BM1>() ? gemm_smem_floats<BM0>()
                                                                       : gemm_smem_floats<BM1>();
  __shared__ __attribute__((aligned(16))) float sA[SA];
  __shared__ __attribute__((aligned(16))) float sB[SA];
  const unsigned n0 = g0.gx * g0.gy * g0.gz;
  unsigned b = blockIdx.x;
  if (b < n0) {
    gemm_block<true, false, BM0, BM0, NST0>(g0, b % g0.gx, (b / g0.gx) % g0.gy, b / (g0.gx * g0.gy), sA, sB);
  } else {
    b -= n0;
    gemm_block<false, false, BM1, BM1, NST1>(g1, b % g1.gx, (b / g1.gx) % g1.gy, b / (g1.gx * g1.gy), sA, sB);
  }
}

// Up to kMultiMax independent weight gradients dW = A^T B in one launch (the latent / projection MLP's three
// after hvae_mlp_bwd_rows): block b runs the problem whose block range holds it, on the register-staged kernel
// in 32 x 32 tiles, without split-K.
constexpr int kMultiMax = 8;
struct GemmMulti {
  GemmP g[kMultiMax];
  unsigned start[kMultiMax + 1];
  int n;
};

__global__ void __launch_bounds__(256) k_gemm_f32_multi(GemmMulti m) {
  __shared__ __attribute__((aligned(16))) float sA[gemm_smem_floats<32>()];
  __shared__ __attribute__((aligned(16))) float sB[gemm_smem_floats<32>()];
  unsigned b = blockIdx.x;
  int i = 0;
  while (i + 1 < m.n && b >= m.start[i + 1]) ++i;
  b -= m.start[i];
  const GemmP& g = m.g[i];
  gemm_block<true, false, 32, 32, kRingStages>(g, b % g.gx, (b / g.gx) % g.gy, b / (g.gx * g.gy), sA, sB);
}

// ---------------------------------------------------------------- colsum ---
__global__ void k_colsum_part(const float* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                              int64_t rows_per_part, float beta, float* __restrict__ out,
                              bool direct) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_part, r1 = min(M, r0 + rows_per_part);
  float s = 0.f;
  for (int64_t r = r0; r < r1; ++r) s += X[r * ldx + n];
  if (direct) {
    out[n] = (beta != 0.f ? beta * out[n] : 0.f) + s;
  } else {
    out[(int64_t)blockIdx.y * N + n] = s;
  }
}

__global__ void k_colsum_final(const float* __restrict__ part, int64_t P, int64_t N, float beta,
                               float* __restrict__ out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int64_t p = 0; p < P; ++p) s += part[p * N + n];
  out[n] = (beta != 0.f ? beta * out[n] : 0.f) + s;
}

// Tile choice: 32x32 for the batch-sized GEMMs (short K, few 64x64 tiles: spread the
// output over more CUs); 64x64 when that already gives >= 512 tiles (two blocks per CU)
// or K is long (then split-K into register-staged ranges fills the machine instead).
// At B = 4096 (scripts/bench_gemm.py, MI355X) the 512 threshold moved 4096x128x384 from
// 21.2 to 14.2 us and 4096x256x512 from 26.2 to 24.3 us against the old 64, while
// 4096x512x256 keeps its 64x64 tiles (23.9 us; 27.6 with 32x32).
// HVAE_GEMM_TILE64_MIN (A/B knob, read once): the 64x64-tile count from which 64x64 tiles are used.
static int64_t tile64_min() {
  static const int64_t v = [] {
    const char* e = ab_getenv("HVAE_GEMM_TILE64_MIN");
    return e ? std::max<int64_t>(1, std::atoll(e)) : (int64_t)512;
  }();
  return v;
}

static int gemm_tile(int64_t M, int64_t N, int64_t K) {
  // long K (split-K weight gradients): 64x64 unless that leaves under 24 tiles -- 384x128x4096 ran in
  // 27.4 us with 32x32 against 38.4 us with 64x64, while 384x384 and 256x512 (32-36 tiles) were faster
  // with 64x64 (45.8 / 39.3 us against 60.1 / 52.7)
  if (K > 4 * (int64_t)GBK * kRegStages) return cdiv(M, 64) * cdiv(N, 64) >= 24 ? 64 : 32;
  return cdiv(M, 64) * cdiv(N, 64) >= tile64_min() ? 64 : 32;
}

static int gemm_splits(int64_t M, int64_t N, int64_t K) {
  const int bt = gemm_tile(M, N, K);
  const int64_t tiles = cdiv(M, bt) * cdiv(N, bt);
  const int64_t kreg = (int64_t)GBK * kRegStages;
  if (K <= kreg || tiles == 0 || tiles >= 256) return 1;  // (tiles == 0: an empty product)  // short K: all loads in flight at once, no split needed
  // about 256 blocks, with no floor at K / kreg: a block may stream more k-tiles than it stages in
  // registers. Fewer partial tiles measured faster on MI355X: 256x512x4096 47.1 -> 39.9 us, 384x384x4096
  // 46.9 -> 45.6 us (profiles/r01_gemm_dw_splitk_ab_v19.jsonl)
  int64_t s = std::min<int64_t>(cdiv(256, tiles), K / 128);
  if (tiles * s > (int64_t)kTicketSlice * 4) s = std::max<int64_t>(1, (int64_t)kTicketSlice * 4 / tiles);
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

// ---- fast-path plan: a tile (BM x BN from the instantiated set) and a split count, or none
struct FastPlan {
  int bm = 0, bn = 0, splits = 1;
  int64_t kps = 0;
};
// The fast path serves the weight gradients dW = dY^T X (trans_a, K = the batch): split-K over 32-deep
// stages with four stages of loads in flight beat the register-staged kernel there (B = 4096, MI355X:
// 384x384x4096 44.8 -> 32.8 us, 768x768x4096 124.6 -> 89.0, 256x512x4096 38.4 -> 27.6;
// profiles/r02_gemm_fast_sweep.txt), while the short-K batch GEMMs (K = d, H or 2L) stay faster on the
// register-staged kernel, which issues every k stage's loads at once (4096x384x384 27.3 us against
// 38.8 at best); so do batches under 1024 (K = B). Tile: 32 x 32 while that gives <= 256 tiles, else 64 x 64.
// A/B knobs, read at every call: HVAE_GEMM_FAST=0 (register-staged kernel only), HVAE_GEMM_FAST_TILE=32|64,
// HVAE_GEMM_FAST_SPLITS=s
static FastPlan fast_plan(bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                          const float* B, int64_t ldb, bool /*pair_w*/) {
  FastPlan f;
  const char* e = ab_getenv("HVAE_GEMM_FAST");
  if (e && std::atoi(e) == 0) return f;
  if (!ta) {
    // HVAE_GEMM_FAST_SHORT=1 (A/B): the batch GEMMs (x W^T, x W; K = d, H or 2L) on the fast path too, one k range
    const char* fs = ab_getenv("HVAE_GEMM_FAST_SHORT");
    if (!fs || std::atoi(fs) == 0) return f;
    if (K % FBK || ((uintptr_t)A) % 16 || ((uintptr_t)B) % 16 || lda % 4 || ldb % 4) return f;
    int bt = cdiv(M, 64) * cdiv(N, 64) >= 256 ? 64 : 32;
    if (const char* t = ab_getenv("HVAE_GEMM_FAST_TILE")) bt = std::atoi(t) == 64 ? 64 : 32;
    if (M % bt || N % bt) return f;
    f.bm = f.bn = bt;
    f.splits = 1;
    f.kps = K;
    return f;
  }
  if (tb) return f;
  if (K < 1024 || K % FBK || ((uintptr_t)A) % 16 || ((uintptr_t)B) % 16 || lda % 4 || ldb % 4) return f;
  int bt = cdiv(M, 32) * cdiv(N, 32) <= 256 ? 32 : 64;
  if (const char* t = ab_getenv("HVAE_GEMM_FAST_TILE")) bt = std::atoi(t) == 64 ? 64 : 32;
  if (M % bt || N % bt) return f;
  const int64_t tiles = (M / bt) * (N / bt);
  int64_t s = 1;
  // ~512 blocks in 32-square tiles; in 64-square ones (768 x 768 at the Syn-10M shard) ~1024, which the
  // LDS-DMA path's five blocks per CU can hold: 768x768x4096 65.9 us with 8 splits against 69.4 with 4
  if (K > 1024) s = std::max<int64_t>(1, std::min<int64_t>(((bt == 64 ? 1024 : 512) + tiles - 1) / tiles, K / 256));
  if (const char* t = ab_getenv("HVAE_GEMM_FAST_SPLITS")) s = std::max(1, std::atoi(t));
  s = std::min<int64_t>(s, 64);
  if (s > 1 && tiles > (int64_t)kTicketSlice) s = 1;
  const int64_t kps = cdiv(cdiv(K, s), FBK) * FBK;
  f.bm = f.bn = bt;
  f.splits = (int)cdiv(K, kps);
  f.kps = kps;
  return f;
}

// ---- LDS-DMA path plan: the tile when the problem is whole tiles of it, 0 otherwise: 64 (64 x 64), 32 (32 x 32)
// or kTile6432 (64 x 32, single launches only). A/B knobs (read at every call): HVAE_GEMM_DMA=0 keeps the
// register-staged / fast kernels, HVAE_GEMM_DMA_TILE=32|64|6432 forces a tile.
constexpr int kTile6432 = 6432;
static int dma_tile(bool ta, bool tb, const GemmP& g, bool pair = false) {
  if (const char* e = ab_getenv("HVAE_GEMM_DMA"))
    if (std::atoi(e) == 0) return 0;
  const int64_t M = g.M, N = g.N, K = g.K;
  if (K == 0 || K % FBK || g.kps % FBK || ((uintptr_t)g.A) % 16 || ((uintptr_t)g.B) % 16 || g.lda % 4 || g.ldb % 4)
    return 0;
  const int64_t ea = (ta ? K * g.lda : M * g.lda) * 4, eb = (tb ? N * g.ldb : K * g.ldb) * 4;
  if (ea >= ((int64_t)1 << 31) || eb >= ((int64_t)1 << 31)) return 0;  // 32-bit buffer offsets
  // 64 x 64 from two blocks per CU; 64 x 32 where that doubles one block per CU to two; else 64 x 64 at one
  // block per CU; else 32 x 32
  const int64_t t64 = (M % 64 == 0 && N % 64 == 0) ? (M / 64) * (N / 64) * (int64_t)g.gz : 0;
  const int64_t t6432 = (M % 64 == 0 && N % 32 == 0) ? (M / 64) * (N / 32) * (int64_t)g.gz : 0;
  int bt = t64 >= 512 ? 64 : (!pair && !ta && t6432 >= 512) ? kTile6432 : t64 >= 256 ? 64 : 32;
  if (const char* e = ab_getenv("HVAE_GEMM_DMA_TILE")) {
    const int v = std::atoi(e);
    bt = v == 64 ? 64 : (v == kTile6432 && !pair) ? kTile6432 : 32;
  }
  const int bm = bt == kTile6432 ? 64 : bt, bn = bt == kTile6432 ? 32 : bt;
  if (M % bm || N % bn) return 0;
  if (g.slab && (M / bm) * (N / bn) > (int64_t)kTicketSlice) return 0;
  // the weight gradients in 32-square tiles (768 x 128, 256 x 512 over K = 4096) stay on the fast path: 20.5 /
  // 21.3 us there against 23.0 / 26.9 here (profiles/r05_gemm_dma_trace_ab.jsonl)
  if (ta && !tb && bt == 32 && !ab_getenv("HVAE_GEMM_DMA_TILE")) return 0;
  return bt;
}

static int colsum_parts(int64_t M) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(M, 64), 64)); }

}  // namespace hvae

using namespace hvae;

extern "C" size_t hvae_gemm_f32_workspace(int64_t M, int64_t N, int64_t K) {
  int s = gemm_splits(M, N, K);
  // the fast path's split count (operands assumed aligned; as a pair's weight-gradient half or alone)
  static const float dummy[4] = {0.f, 0.f, 0.f, 0.f};
  for (int pw = 0; pw < 2; ++pw)
    for (int ta = 0; ta < 2; ++ta) {
      const FastPlan f = fast_plan(ta, false, M, N, K, dummy, 4, dummy, 4, pw);
      if (f.bm) s = std::max(s, f.splits);
    }
  return s > 1 ? (size_t)s * (M * N + M) * sizeof(float) : 0;
}

// Validate one problem and fill its launch record (tile size in *bt).
static int gemm_setup(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                      int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                      const hvae_epilogue* epi, void* ws, size_t ws_bytes, GemmP& g, int& bt,
                      FastPlan* fp = nullptr, bool pair_w = false) {
  HVAE_REQUIRE(M >= 0 && N >= 0 && K >= 0 && C, "hvae_gemm_f32: bad shape / null C");
  HVAE_REQUIRE(ldc >= N, "hvae_gemm_f32: ldc < N");
  HVAE_REQUIRE(M < (1ll << 31) / 64 * 64 && N < (1ll << 31), "hvae_gemm_f32: too large");
  HVAE_REQUIRE(K == 0 || (A && B) || M == 0 || N == 0, "hvae_gemm_f32: null A/B");
  HVAE_REQUIRE(trans_a ? lda >= M : lda >= K, "hvae_gemm_f32: bad lda");
  HVAE_REQUIRE(trans_b ? ldb >= K : ldb >= N, "hvae_gemm_f32: bad ldb");
  EpiArgs ep{};
  ep.kind = HVAE_EPI_NONE;
  if (epi) {
    ep.kind = epi->kind;
    ep.bias = epi->bias;
    ep.pre_out = epi->pre_out;
    ep.pre_in = epi->pre_in;
    ep.p_drop = epi->p_drop;
    ep.scale = (epi->p_drop < 1.f) ? 1.0f / (1.0f - epi->p_drop) : 0.f;
    ep.drop_mult = epi->drop_mult;
    ep.seed = epi->seed;
    ep.step_dev = epi->step_dev;
    ep.tag = epi->tag;
    ep.train = epi->train;
    ep.opa_rowsum = epi->opa_rowsum;
    ep.aux = epi->aux;
    ep.aux_scale = epi->aux_scale;
    ep.aux_scale_dev = epi->aux_scale_dev;
    HVAE_REQUIRE(ep.kind >= 0 && ep.kind <= HVAE_EPI_REPARAM_BWD, "hvae_gemm_f32: bad epilogue");
    HVAE_REQUIRE(ep.kind != HVAE_EPI_REPARAM_BWD || (ep.pre_in && (ep.aux || !ep.train) && ldc >= 2 * N),
                 "hvae_gemm_f32: REPARAM_BWD needs heads (pre_in), eps (aux) and ldc >= 2N");
    HVAE_REQUIRE(ep.kind != HVAE_EPI_BIAS || ep.bias, "hvae_gemm_f32: BIAS without bias");
    HVAE_REQUIRE(ep.kind != HVAE_EPI_BIAS_GELU_DROP || ep.pre_out, "hvae_gemm_f32: no pre_out");
    HVAE_REQUIRE(ep.kind != HVAE_EPI_GELU_DROP_BWD || ep.pre_in, "hvae_gemm_f32: no pre_in");
  }
  FastPlan f;
  if (fp) f = fast_plan(trans_a, trans_b, M, N, K, A, lda, B, ldb, pair_w);
  int splits = f.bm ? f.splits : gemm_splits(M, N, K);
  if (splits > 1) {
    const int64_t fit = ws ? (int64_t)(ws_bytes / ((size_t)(M * N + M) * sizeof(float))) : 0;
    splits = (int)std::min<int64_t>(splits, fit);
    if (splits < 2) splits = 1;
  }
  int64_t kps = K;
  if (splits > 1) {
    kps = cdiv(cdiv(K, splits), GBK) * GBK;
    splits = (int)cdiv(K, kps);
  }
  bt = gemm_tile(M, N, K);
  if (fp) {
    f.splits = splits;
    f.kps = kps;
    *fp = f;
  }
  g.M = M; g.N = N; g.K = K; g.kps = (K == 0) ? 0 : kps;
  g.alpha = alpha; g.A = A; g.lda = lda; g.B = B; g.ldb = ldb; g.beta = beta; g.C = C; g.ldc = ldc;
  g.ep = ep;
  g.vec_a = (((uintptr_t)A) % 16 == 0) && (lda % 4 == 0);
  g.vec_b = (((uintptr_t)B) % 16 == 0) && (ldb % 4 == 0);
  g.gx = (unsigned)cdiv(N, f.bm ? f.bn : bt); g.gy = (unsigned)cdiv(M, f.bm ? f.bm : bt);
  g.gz = (unsigned)std::max(splits, 1);
  g.slab = splits > 1 ? (float*)ws : nullptr;
  g.tickets = nullptr;
  if (g.slab) {
    HVAE_REQUIRE((uint64_t)g.gx * g.gy <= (uint64_t)kTicketSlice, "hvae_gemm_f32: too many split tiles");
    g.tickets = ticket_slice();
    if (!g.tickets) return HVAE_ERR_HIP;
  }
  return HVAE_OK;
}

extern "C" int hvae_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                             const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                             float* C, int64_t ldc, const hvae_epilogue* epi, void* ws,
                             size_t ws_bytes, void* stream) {
  if (M == 0 || N == 0) {
    HVAE_REQUIRE(M >= 0 && N >= 0 && C, "hvae_gemm_f32: bad shape / null C");
    return HVAE_OK;
  }
  GemmP g{};
  int bt = 32;
  FastPlan f;
  if (int rc = gemm_setup(trans_a, trans_b, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, epi, ws, ws_bytes, g,
                          bt, &f))
    return rc;
  hipStream_t st = as_stream(stream);
  if (const int dt = dma_tile(trans_a, trans_b, g)) {
    const int bm = dt == kTile6432 ? 64 : dt, bn = dt == kTile6432 ? 32 : dt;
    g.gx = (unsigned)(N / bn);
    g.gy = (unsigned)(M / bm);
    dim3 grid(g.gx, g.gy, g.gz);
    ProbeScope probe("gemm", st);
#define HVAE_DMA_CALL(TA_, TB_)                                                       \
  (dt == 64 ? (k_gemm_dma<TA_, TB_, 64, 64><<<grid, 256, 0, st>>>(g))                \
   : dt == kTile6432 ? (k_gemm_dma<TA_, TB_, 64, 32><<<grid, 256, 0, st>>>(g))       \
                     : (k_gemm_dma<TA_, TB_, 32, 32><<<grid, 256, 0, st>>>(g)))
    if (!trans_a && !trans_b) HVAE_DMA_CALL(false, false);
    else if (!trans_a && trans_b) HVAE_DMA_CALL(false, true);
    else if (trans_a && !trans_b) HVAE_DMA_CALL(true, false);
    else HVAE_DMA_CALL(true, true);
#undef HVAE_DMA_CALL
    HVAE_LAUNCH_CHECK("k_gemm_dma");
    return HVAE_OK;
  }
  dim3 grid(g.gx, g.gy, g.gz);
  ProbeScope probe("gemm", st);
  if (f.bm) {  // trans_a && !trans_b (or, under HVAE_GEMM_FAST_SHORT, !trans_a)
#define HVAE_FAST_CALL(TA_, TB_)                                                  \
  (f.bm == 64 ? (k_gemm_fast<TA_, TB_, 64, 64><<<grid, 256, 0, st>>>(g))        \
              : (k_gemm_fast<TA_, TB_, 32, 32><<<grid, 256, 0, st>>>(g)))
    if (trans_a) HVAE_FAST_CALL(true, false);
#ifdef HVAE_AB
    else if (trans_b) HVAE_FAST_CALL(false, true);
    else HVAE_FAST_CALL(false, false);
#endif
#undef HVAE_FAST_CALL
    HVAE_LAUNCH_CHECK("k_gemm_fast");
    return HVAE_OK;
  }
  const int nstc = nst_class(trans_a, trans_b, g.kps);
#define HVAE_GEMM_CALL(TA_, TB_)                                                                  \
  (bt == 64 ? (nstc == kRegStages ? (k_gemm_f32<TA_, TB_, 64, 64, kRegStages><<<grid, 256, 0, st>>>(g))  \
               : nstc == 1 ? (k_gemm_f32<TA_, TB_, 64, 64, 1><<<grid, 256, 0, st>>>(g))                   \
                           : (k_gemm_f32<TA_, TB_, 64, 64, kRingStages><<<grid, 256, 0, st>>>(g)))        \
            : (nstc == kRegStages ? (k_gemm_f32<TA_, TB_, 32, 32, kRegStages><<<grid, 256, 0, st>>>(g))  \
               : nstc == 1 ? (k_gemm_f32<TA_, TB_, 32, 32, 1><<<grid, 256, 0, st>>>(g))                   \
                           : (k_gemm_f32<TA_, TB_, 32, 32, kRingStages><<<grid, 256, 0, st>>>(g))))
  if (!trans_a && !trans_b) HVAE_GEMM_CALL(false, false);
  else if (!trans_a && trans_b) HVAE_GEMM_CALL(false, true);
  else if (trans_a && !trans_b) HVAE_GEMM_CALL(true, false);
  else HVAE_GEMM_CALL(true, true);
#undef HVAE_GEMM_CALL
  HVAE_LAUNCH_CHECK("k_gemm_f32");
  return HVAE_OK;
}

static int gemm_desc(const hvae_gemm_desc* d, void* stream) {
  return hvae_gemm_f32(d->trans_a, d->trans_b, d->M, d->N, d->K, d->alpha, d->A, d->lda, d->B, d->ldb, d->beta,
                       d->C, d->ldc, d->epi, d->ws, d->ws_bytes, stream);
}

extern "C" int hvae_gemm_f32_pair(const hvae_gemm_desc* w, const hvae_gemm_desc* x, void* stream) {
  HVAE_REQUIRE(w && x, "hvae_gemm_f32_pair: null descriptor");
  // one launch for the (A^T B, A B) pair of a layer's backward; any other pairing runs as two launches
  const bool shared_ws = w->ws && w->ws == x->ws && gemm_splits(w->M, w->N, w->K) > 1 &&
                         gemm_splits(x->M, x->N, x->K) > 1;  // both split-K into one slab: two launches
  const bool fused = w->trans_a && !w->trans_b && !x->trans_a && !x->trans_b && w->M > 0 && w->N > 0 &&
                     x->M > 0 && x->N > 0 && !shared_ws;
  if (!fused) {
    if (int rc = gemm_desc(w, stream)) return rc;
    return gemm_desc(x, stream);
  }
  GemmP g0{}, g1{};
  int bt0 = 32, bt1 = 32;
  FastPlan f0, f1;
  if (int rc = gemm_setup(1, 0, w->M, w->N, w->K, w->alpha, w->A, w->lda, w->B, w->ldb, w->beta, w->C, w->ldc,
                          w->epi, w->ws, w->ws_bytes, g0, bt0, &f0, true))
    return rc;
  if (int rc = gemm_setup(0, 0, x->M, x->N, x->K, x->alpha, x->A, x->lda, x->B, x->ldb, x->beta, x->C, x->ldc,
                          x->epi, x->ws, x->ws_bytes, g1, bt1, &f1))
    return rc;
  hipStream_t st = as_stream(stream);
  {
    const int d0 = dma_tile(true, false, g0, true), d1 = dma_tile(false, false, g1, true);
    if ((d0 != 0) != (d1 != 0) || (d0 && d1 && g0.slab && g1.slab)) {
      // one half on the LDS-DMA path, the other not: two launches, so that each half runs the kernel its own
      // hvae_gemm_f32 call would (the pair stays bitwise the two launches)
      if (int rc = gemm_desc(w, stream)) return rc;
      return gemm_desc(x, stream);
    }
    if (d0 && d1) {  // both on the LDS-DMA path, one launch
      g0.gx = (unsigned)(g0.N / d0); g0.gy = (unsigned)(g0.M / d0);
      g1.gx = (unsigned)(g1.N / d1); g1.gy = (unsigned)(g1.M / d1);
      const unsigned nblk = g0.gx * g0.gy * g0.gz + g1.gx * g1.gy * g1.gz;
      ProbeScope probe("gemm", st);
      if (d0 == 64 && d1 == 64) k_gemm_dma_pair<64, 64><<<nblk, 256, 0, st>>>(g0, g1);
      else if (d0 == 64) k_gemm_dma_pair<64, 32><<<nblk, 256, 0, st>>>(g0, g1);
      else if (d1 == 64) k_gemm_dma_pair<32, 64><<<nblk, 256, 0, st>>>(g0, g1);
      else k_gemm_dma_pair<32, 32><<<nblk, 256, 0, st>>>(g0, g1);
      HVAE_LAUNCH_CHECK("k_gemm_dma_pair");
      return HVAE_OK;
    }
  }
  if (f0.bm || f1.bm) {
    if (!f0.bm || f1.bm || (g0.slab && g1.slab)) {  // not (fast dW, register-staged dX): two launches
      if (int rc = gemm_desc(w, stream)) return rc;
      return gemm_desc(x, stream);
    }
    const unsigned nblk = g0.gx * g0.gy * g0.gz + g1.gx * g1.gy * g1.gz;
    ProbeScope probe("gemm", st);
    const int c1 = nst_class(false, false, g1.kps);
#define HVAE_MIXED(F0_, BT1_)                                                                            \
  (c1 == kRegStages ? (k_gemm_mixed_pair<F0_, BT1_, kRegStages><<<nblk, 256, 0, st>>>(g0, g1))           \
   : c1 == 1 ? (k_gemm_mixed_pair<F0_, BT1_, 1><<<nblk, 256, 0, st>>>(g0, g1))                           \
             : (k_gemm_mixed_pair<F0_, BT1_, kRingStages><<<nblk, 256, 0, st>>>(g0, g1)))
    if (f0.bm == 64 && bt1 == 64) HVAE_MIXED(64, 64);
    else if (f0.bm == 64) HVAE_MIXED(64, 32);
    else if (bt1 == 64) HVAE_MIXED(32, 64);
    else HVAE_MIXED(32, 32);
#undef HVAE_MIXED
    HVAE_LAUNCH_CHECK("k_gemm_mixed_pair");
    return HVAE_OK;
  }
  const unsigned nblk = g0.gx * g0.gy * g0.gz + g1.gx * g1.gy * g1.gz;
  ProbeScope probe("gemm", st);
  // (the register-staged pair keeps two classes: long k ranges on the kRegStages instance's one-tile lookahead)
  const bool q0 = nst_class(true, false, g0.kps) != kRingStages, q1 = nst_class(false, false, g1.kps) != kRingStages;
#define HVAE_PAIR(B0_, B1_)                                                                              \
  (q0 ? (q1 ? (k_gemm_f32_pair<B0_, B1_, kRegStages, kRegStages><<<nblk, 256, 0, st>>>(g0, g1))          \
            : (k_gemm_f32_pair<B0_, B1_, kRegStages, kRingStages><<<nblk, 256, 0, st>>>(g0, g1)))        \
      : (q1 ? (k_gemm_f32_pair<B0_, B1_, kRingStages, kRegStages><<<nblk, 256, 0, st>>>(g0, g1))         \
            : (k_gemm_f32_pair<B0_, B1_, kRingStages, kRingStages><<<nblk, 256, 0, st>>>(g0, g1))))
  if (bt0 == 64 && bt1 == 64) HVAE_PAIR(64, 64);
  else if (bt0 == 64) HVAE_PAIR(64, 32);
  else if (bt1 == 64) HVAE_PAIR(32, 64);
  else HVAE_PAIR(32, 32);
#undef HVAE_PAIR
  HVAE_LAUNCH_CHECK("k_gemm_f32_pair");
  return HVAE_OK;
}

extern "C" int hvae_gemm_f32_multi(const hvae_gemm_desc* d, int n, void* stream) {
  HVAE_REQUIRE(d && n >= 1 && n <= kMultiMax, "hvae_gemm_f32_multi: 1..8 descriptors");
  GemmMulti m{};
  m.n = 0;
  unsigned nblk = 0;
  for (int i = 0; i < n; ++i) {
    HVAE_REQUIRE(d[i].trans_a == 1 && d[i].trans_b == 0, "hvae_gemm_f32_multi: weight gradients only (A^T B)");
    if (d[i].M == 0 || d[i].N == 0) continue;
    GemmP g{};
    int bt = 32;
    // no workspace: one k range per tile
    if (int rc = gemm_setup(1, 0, d[i].M, d[i].N, d[i].K, d[i].alpha, d[i].A, d[i].lda, d[i].B, d[i].ldb, d[i].beta,
                            d[i].C, d[i].ldc, d[i].epi, nullptr, 0, g, bt))
      return rc;
    g.gx = (unsigned)cdiv(d[i].N, 32);
    g.gy = (unsigned)cdiv(d[i].M, 32);
    g.gz = 1;
    m.start[m.n] = nblk;
    m.g[m.n++] = g;
    nblk += g.gx * g.gy;
  }
  if (m.n == 0) return HVAE_OK;
  m.start[m.n] = nblk;
  hipStream_t st = as_stream(stream);
  ProbeScope probe("gemm", st);
  k_gemm_f32_multi<<<nblk, 256, 0, st>>>(m);
  HVAE_LAUNCH_CHECK("k_gemm_f32_multi");
  return HVAE_OK;
}

extern "C" size_t hvae_colsum_workspace(int64_t M, int64_t N) {
  const int P = colsum_parts(M);
  return P > 1 ? (size_t)P * N * sizeof(float) : 0;
}

extern "C" int hvae_colsum(const float* X, int64_t M, int64_t N, int64_t ldx, float beta, float* out,
                           void* ws, size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(out && N >= 0 && M >= 0 && ldx >= N, "hvae_colsum: bad args");
  if (N == 0) return HVAE_OK;
  hipStream_t st = as_stream(stream);
  if (M == 0) {
    if (beta == 0.f) HVAE_HIP(hipMemsetAsync(out, 0, N * sizeof(float), st));
    return HVAE_OK;
  }
  HVAE_REQUIRE(X, "hvae_colsum: null X");
  int P = colsum_parts(M);
  if (P > 1 && (!ws || ws_bytes < (size_t)P * N * sizeof(float))) P = 1;
  const int64_t rpp = cdiv(M, P);
  dim3 grid((unsigned)cdiv(N, 256), (unsigned)P);
  k_colsum_part<<<grid, 256, 0, st>>>(X, M, N, ldx, rpp, beta, P > 1 ? (float*)ws : out, P == 1);
  HVAE_LAUNCH_CHECK("k_colsum_part");
  if (P > 1) {
    k_colsum_final<<<(unsigned)cdiv(N, 256), 256, 0, st>>>((const float*)ws, P, N, beta, out);
    HVAE_LAUNCH_CHECK("k_colsum_final");
  }
  return HVAE_OK;
}
