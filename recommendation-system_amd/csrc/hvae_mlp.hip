// hvae_mlp.hip -- the latent / projection MLP of small batches, row-parallel, one launch per direction.
//
// Between the encoder and the decoder the step runs three Linear layers and the reparameterisation
// (src/ml/model.py:126-127,152-153 fc_mu / fc_logvar, :157-179 reparameterize, :90-95,195 the projection
// Linear -> GELU -> Dropout -> Linear). At the batches of `make train-best` (B = 64) each of them is a
// launch of a few microseconds of work behind a few microseconds of dispatch, and the chain of them is
// what the step waits on. Every row of the chain depends only on its own batch row, so here a block owns
// R batch rows and runs the whole chain for them, the activations never leaving LDS: the cost is one
// pass over the three weight matrices per block (1.3 MB at d = 384, from L2) instead of four (forward)
// or three (backward data gradients) dependent launches.
//
// Forward layers are x W^T with W = [out][in] (k-contiguous): lane (j = l >> 3, c = l & 7) of a wave
// takes output 8 g + j and k-chunk 4 c of every 32 k, so each 16-B load of a wave reads eight whole
// 128-B lines, and the eight partial dots of an output meet in a 3-step butterfly. Backward layers are
// x W (n-contiguous): thread t takes the four outputs 4 (t % N/4).. over the k-slice t / (N/4), and
// the slices' partial sums meet in LDS in slice order. Sums run in fp32 in a fixed order (deterministic;
// not the GEMM's order, so agreement with the GEMM path is to fp32 rounding, tests/test_gpu_kernels.py).
#include <algorithm>
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "hvae_common.h"
#include "hvae_rgplan.h"
#include "hvae_encoder_row.h"
#include "hvae_adam.h"

namespace hvae {

constexpr int kMlpThreads = 1024;
constexpr int kMlpWaves = kMlpThreads / 64;

struct MlpP {
  int64_t nb;
  int H, L, D;
  const float* Wh; const float* bh;
  const float* Wa; const float* ba;
  const float* Wb; const float* bb;
  int train;
  float p_drop, scale;
  const float* drop_mult;
  const float* eps_in;
  uint64_t seed;
  const int64_t* step_dev;
  const float* h;
  float* heads; float* z; float* eps; float* kl_rows; float* p1; float* q; float* u;
  const float* dU;
  float ks; const float* ks_dev;
  float* dp1; float* dheads; float* dh;
  int rot;  // rotate each block's walk over the weights (A/B: HVAE_MLP_ROT=0 walks them in one order)
  // the row-gradient plan of the batch, run by block gridDim.x - 1 when plan_slot_of != NULL
  const int64_t* pl_row_ptr; const int32_t* pl_col_idx; const float* pl_vals; const int32_t* pl_rows;
  const int64_t* pl_rows_offset; int64_t pl_nb;
  int32_t* plan_slot_of; int32_t* pl_item_of; int32_t* pl_seg_off; int32_t* pl_contrib_row; float* pl_contrib_val;
  int32_t* pl_contrib_slot; int32_t* pl_n_unique;
  // backward: the last hidden layer's LayerNorm -> GELU -> Dropout backward, when ln_w != NULL
  const float* ln_w; const float* ln_b; const float* xhat; const float* rstd; const float* enc_drop_mult;
  uint32_t enc_tag;
  float* da; float* d_ln_w; float* d_ln_b; float* d_bias;
  float* ln_part; unsigned* ln_ticket;
  // forward: the first encoder layer of the rows, when enc_w1t != NULL (writes h_out, xhat, rstd)
  const int64_t* e_row_ptr; const int32_t* e_col_idx; const float* e_vals; const int32_t* e_rows;
  const int64_t* e_rows_offset;
  const float* enc_w1t; const float* enc_b1;
  float* h_out; float* xhat_out; float* rstd_out;
  // forward: w1t through exact lazy Adam (enc_lazy): rows replayed to *aa.step_dev steps in registers
  int enc_lazy;
  AdamArgs aa;
  const float* am; const float* av; const int32_t* ls; const float2* atab;
};

// The fused encoder layer's share of wave `sub` of row b with W1t read through lazy Adam: each entry's (p, m, v)
// row and stamp are loaded (two entries in flight) and p is brought to `to` steps by col_math_lazy -- the float
// operations of the CSR catch-up -- before x p is added; nothing is stored
template <int NV>
__device__ __forceinline__ void encoder_row_partial_lazy(const MlpP& p, int64_t b, int H, int sub, int nsub, int to,
                                                         float4 (&acc)[NV]) {
  const int lane = threadIdx.x & 63;
  const int64_t r = batch_row(p.e_rows, p.e_rows_offset, b);
  const int64_t beg = p.e_row_ptr[r], end = p.e_row_ptr[r + 1];
  const int64_t H4 = H / 4;
  const AdamK none{};
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int EU = 2;
  for (int64_t e0 = beg + sub; e0 < end; e0 += EU * (int64_t)nsub) {
    int64_t j[EU];
    float x[EU];
    int32_t st[EU];
    bool ok[EU];
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      const int64_t e = e0 + (int64_t)u * nsub;
      ok[u] = e < end;
      j[u] = ok[u] ? p.e_col_idx[e] : 0;
      x[u] = ok[u] ? p.e_vals[e] : 0.f;
      st[u] = ok[u] ? p.ls[j[u]] : to;
    }
    ColState cs[EU][NV];
#pragma unroll
    for (int u = 0; u < EU; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int64_t c4 = lane + 64 * k;
        if (ok[u] && c4 < H4) cs[u][k] = col_load(p.enc_w1t, p.am, p.av, j[u] * H4 + c4);
      }
#pragma unroll
    for (int u = 0; u < EU; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (lane + 64 * k >= H4) continue;
        col_math_lazy(p.aa, p.atab, cs[u][k], ls_mv(st[u]), ls_p(st[u]), to, false, none, make_float4(0.f, 0.f, 0.f, 0.f));
        acc[k].x += x[u] * cs[u][k].p.x; acc[k].y += x[u] * cs[u][k].p.y;
        acc[k].z += x[u] * cs[u][k].p.z; acc[k].w += x[u] * cs[u][k].p.w;
      }
    }
  }
}

__device__ __forceinline__ float dot4(float4 w, float4 x, float acc) {
  acc = fmaf(w.x, x.x, acc);
  acc = fmaf(w.y, x.y, acc);
  acc = fmaf(w.z, x.z, acc);
  return fmaf(w.w, x.w, acc);
}

// A block barrier that orders LDS only: this wave's LDS writes have landed (lgkmcnt 0), its global loads stay in
// flight (__syncthreads' workgroup fence would wait for them too). The layers issue their first weight loads
// before it, so that their latency overlaps the previous phase (the encoder gather, an epilogue) of other waves.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt, expcnt left at their maxima
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The layers are bound by how many bytes of weights a CU has in flight (one block streams all three matrices
// from L2: 1.3 MB at d = 384), so every lane keeps kMlpLoads 16-B loads outstanding.
constexpr int kMlpLoads = 16;

// ys[r][n] = sum_k xs[r][k] W[n][k] for n < N (N % 8 == 0, K % 32 == 0).
// G output groups of 8 per wave at once, so that kMlpLoads loads are in flight per lane; chunks past K re-read
// the last one and add it with a zero activation (every load unconditional)
// PRE: the block barrier that makes xs visible is taken here, after every wave has issued the weight loads of its
// first pass (by every wave once, outside any branch)
template <int R, int G, int LOADS, bool PRE>
__device__ __forceinline__ void rows_nt_g(const float* __restrict__ W, int N, int K, const float* xs, float* ys,
                                          int rotate) {
  constexpr int KCH = LOADS / G;  // 32-k chunks per pass
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane >> 3, c = lane & 7;
  const int NG = N / 8;
  // blocks start at different output groups, so that the blocks of an XCD stream different lines at a time
  // (all of them walking the matrix in the same order camp on the same L2 channels)
  const int rot = rotate ? (int)((blockIdx.x * 8u) % (unsigned)NG) : 0;
  auto row_ptr = [&](int g0, int gi) {
    return W + (int64_t)(8 * ((min(g0 + gi, NG - 1) + rot) % NG) + j) * K + 4 * c;
  };
  // the first pass of this wave's first output groups (k0 = 0; the clamp covers a K shorter than the pass), into
  // the registers that pass then uses
  float4 wv[G][KCH];
  if (PRE && w * G < NG) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int s = 0; s < KCH; ++s) wv[gi][s] = *reinterpret_cast<const float4*>(row_ptr(w * G, gi) + min(32 * s, K - 32));
  }
  if (PRE) lds_barrier();
  for (int g0 = w * G; g0 < NG; g0 += kMlpWaves * G) {
    float acc[G][R];
#pragma unroll
    for (int gi = 0; gi < G; ++gi)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[gi][r] = 0.f;
    const float* wrow[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) wrow[gi] = row_ptr(g0, gi);
    auto pass = [&](int k0, auto full) {
      constexpr bool FULL = decltype(full)::value;
      if (!(PRE && g0 == w * G && k0 == 0)) {
#pragma unroll
        for (int gi = 0; gi < G; ++gi)
#pragma unroll
          for (int s = 0; s < KCH; ++s)
            wv[gi][s] = *reinterpret_cast<const float4*>(wrow[gi] + (FULL ? k0 + 32 * s : min(k0 + 32 * s, K - 32)));
      }
#pragma unroll
      for (int s = 0; s < KCH; ++s) {
        const int k = FULL ? k0 + 32 * s : min(k0 + 32 * s, K - 32);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          float4 xv = *reinterpret_cast<const float4*>(xs + r * K + k + 4 * c);
          if (!FULL && k0 + 32 * s >= K) xv = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int gi = 0; gi < G; ++gi) acc[gi][r] = dot4(wv[gi][s], xv, acc[gi][r]);
        }
      }
    };
    int k0 = 0;
    for (; k0 + 32 * KCH <= K; k0 += 32 * KCH) pass(k0, std::true_type{});
    if (k0 < K) pass(k0, std::false_type{});
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      // the eight k-chunks of an output: every lane of the group ends with the same total (fp add commutes)
#pragma unroll
      for (int r = 0; r < R; ++r) {
        acc[gi][r] += __shfl_xor(acc[gi][r], 1, 64);
        acc[gi][r] += __shfl_xor(acc[gi][r], 2, 64);
        acc[gi][r] += __shfl_xor(acc[gi][r], 4, 64);
      }
      // lane c of the group stores row c
      float v = acc[gi][0];
#pragma unroll
      for (int r = 1; r < R; ++r) v = (c == r) ? acc[gi][r] : v;
      if (c < R && g0 + gi < NG) ys[c * N + 8 * ((g0 + gi + rot) % NG) + j] = v;
    }
  }
}

// PRE (R > 1): the first weight loads before the barrier that publishes xs; R = 1 takes the barrier first (its 16
// loads per lane leave no room for them to wait across it)
template <int R, bool PRE = (R > 1)>
__device__ __forceinline__ void rows_nt(const float* __restrict__ W, int N, int K, const float* xs, float* ys,
                                        int rotate) {
  if (!PRE) __syncthreads();
  constexpr int LOADS = R == 1 ? kMlpLoads : kMlpLoads / 2;  // more rows: more arithmetic per byte, fewer registers
  if (K >= 32 * LOADS * 3 / 4) rows_nt_g<R, 1, LOADS, PRE>(W, N, K, xs, ys, rotate);
  else if (K >= 32 * LOADS * 3 / 8) rows_nt_g<R, 2, LOADS, PRE>(W, N, K, xs, ys, rotate);
  else rows_nt_g<R, 4, LOADS, PRE>(W, N, K, xs, ys, rotate);
}

// out[r][n] = sum_k xs[r][k] W[k][n] for n < N (N % 4 == 0, N / 4 <= threads); part: LDS of
// (threads / (N / 4)) * R * N <= 4 * threads * R floats. epi(r, n, v) for every (r < R, n).
// Rows past the slice re-read its last row and add it with a zero activation (every load unconditional)
template <int R, class Epi>
__device__ __forceinline__ void rows_nn(const float* __restrict__ W, int N, int K, const float* xs, float* part,
                                        int rotate, Epi epi) {
  const int t = threadIdx.x, NQ = N / 4, S = kMlpThreads / NQ;
  const int qd = t % NQ, s = t / NQ;
  constexpr int LOADS = kMlpLoads / R;  // more rows: more arithmetic per byte, fewer registers
  // blocks take the k slices in rotated order (L2 channels, as in rows_nt_g); partials keep slice order
  const bool act = s < S;
  const int sk = !act ? 0 : rotate ? (int)((s + blockIdx.x) % (unsigned)S) : s;
  const int k_lo = act ? (int)((int64_t)K * sk / S) : 0, k_hi = act ? (int)((int64_t)K * (sk + 1) / S) : 0;
  const float* wp = W + 4 * qd;
  float4 wv[LOADS];
  auto load = [&](int k) {
    const float* pk = wp + (int64_t)k * N;
#pragma unroll
    for (int e = 0; e < LOADS; ++e) {
      wv[e] = *reinterpret_cast<const float4*>(pk);
      pk += (k + e + 1 < k_hi) ? N : 0;
    }
  };
  // the first chunk's weight loads go out before the barrier that makes xs visible (taken by every thread once,
  // outside any branch); R = 1 (16 loads per lane) takes the barrier first
  constexpr bool PRE = R > 1;
  if (PRE && k_lo < k_hi) load(k_lo);
  lds_barrier();
  if (act) {
    float4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = k_lo; k < k_hi; k += LOADS) {
      if (!PRE || k != k_lo) load(k);
#pragma unroll
      for (int e = 0; e < LOADS; ++e) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const float x = (k + e < k_hi) ? xs[r * K + min(k + e, k_hi - 1)] : 0.f;
          acc[r].x = fmaf(wv[e].x, x, acc[r].x);
          acc[r].y = fmaf(wv[e].y, x, acc[r].y);
          acc[r].z = fmaf(wv[e].z, x, acc[r].z);
          acc[r].w = fmaf(wv[e].w, x, acc[r].w);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) *reinterpret_cast<float4*>(part + (sk * R + r) * N + 4 * qd) = acc[r];
  }
  __syncthreads();
  for (int i = t; i < R * N; i += kMlpThreads) {
    const int r = i / N, n = i % N;
    float v = 0.f;
    for (int s2 = 0; s2 < S; ++s2) v += part[(s2 * R + r) * N + n];
    epi(r, n, v);
  }
  __syncthreads();
}

template <int R>
__global__ void __launch_bounds__(kMlpThreads) k_mlp_fwd_rows(MlpP p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int H = p.H, L = p.L, D = p.D, L2 = 2 * p.L;
  float* xs = smem;          // [R][H]  encoder output rows
  float* hs = xs + R * H;    // [R][2L] mu | logvar
  float* zs = hs + R * L2;   // [R][L]
  float* ys = zs + R * L;    // [R][D]  a layer's sums before its epilogue
  float* qs = ys + R * D;    // [R][D]
  if (p.plan_slot_of && blockIdx.x == gridDim.x - 1) {  // the batch's row-gradient plan, beside the rows
    unsigned long long* key = reinterpret_cast<unsigned long long*>(smem);
    float* kv = reinterpret_cast<float*>(key + kPlanSmallCap);
    int64_t* rbeg = reinterpret_cast<int64_t*>(kv + kPlanSmallCap);
    int* roff = reinterpret_cast<int*>(rbeg + kPlanSmallRows);
    int* wsum = roff + kPlanSmallRows + 1;
    rg_plan_small_block(p.pl_row_ptr, p.pl_col_idx, p.pl_vals, p.pl_rows, p.pl_rows_offset, p.pl_nb, p.plan_slot_of,
                        p.pl_item_of, p.pl_seg_off, p.pl_contrib_row, p.pl_contrib_val, p.pl_contrib_slot,
                        p.pl_n_unique, key, kv, roff, rbeg, wsum);
    return;
  }
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * R;
  const int64_t step = load_step(p.step_dev);
  float* bsh = qs + R * D;  // [2L] b_heads | [D] b_a | [D] b_b: the epilogues' biases, fetched ahead (below)
  auto fetch_biases = [&](int t0, int nt) {
    for (int i = t0; i < L2 + 2 * D; i += nt) bsh[i] = i < L2 ? p.bh[i] : i < L2 + D ? p.ba[i - L2] : p.bb[i - L2 - D];
  };
  if (p.enc_w1t) {
    // the first encoder layer, each row's entries dealt over kMlpWaves / R waves (one memory round trip each at
    // ~10 entries a row, where one wave per row walked them four at a time): partials into LDS, then the row's
    // first wave adds them in wave order to the bias and runs the LayerNorm / GELU / dropout
    constexpr int WPR = kMlpWaves / R;
    float* encp = bsh + L2 + 2 * D;  // [R][WPR][H]
    const int r = w / WPR, sub = w % WPR;
    const int64_t b = b0 + r;
    auto part = [&](auto nv) {
      constexpr int NV = decltype(nv)::value;
      float4 acc[NV];
      if (p.enc_lazy)
        encoder_row_partial_lazy<NV>(p, b, H, sub, WPR, (int)load_step(p.aa.step_dev), acc);
      else
        encoder_row_partial<NV>(p.e_row_ptr, p.e_col_idx, p.e_vals, p.e_rows, p.e_rows_offset, b, p.enc_w1t, H, sub,
                                WPR, acc);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = 4 * (lane + 64 * k);
        if (c < H) *reinterpret_cast<float4*>(encp + (r * WPR + sub) * H + c) = acc[k];
      }
    };
    auto fin = [&](auto nv) {
      constexpr int NV = decltype(nv)::value;
      float4 acc[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = 4 * (lane + 64 * k);
        acc[k] = c < H ? *reinterpret_cast<const float4*>(p.enc_b1 + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      for (int s2 = 0; s2 < WPR; ++s2)
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const int c = 4 * (lane + 64 * k);
          if (c >= H) continue;
          const float4 v = *reinterpret_cast<const float4*>(encp + (r * WPR + s2) * H + c);
          acc[k].x += v.x; acc[k].y += v.y; acc[k].z += v.z; acc[k].w += v.w;
        }
      ln_gelu_drop_row<NV>(acc, lane, H, b, p.ln_w, p.ln_b, p.p_drop, p.scale, p.enc_drop_mult, p.seed, step,
                           kTagEncDrop + 0u, p.train, p.h_out, p.xhat_out, p.rstd_out, xs + r * H);
    };
    if (b < p.nb) {
      if (H <= 256) part(std::integral_constant<int, 1>{});
      else part(std::integral_constant<int, 2>{});  // H <= 512 (host check)
    }
    __syncthreads();
    if (sub == 0) {
      if (b < p.nb) {
        if (H <= 256) fin(std::integral_constant<int, 1>{});
        else fin(std::integral_constant<int, 2>{});
      } else {
        for (int e = lane; e < H; e += 64) xs[r * H + e] = 0.f;
      }
    } else {  // the waves the LayerNorm leaves idle fetch the biases meanwhile
      fetch_biases((r * (WPR - 1) + sub - 1) * 64 + lane, R * (WPR - 1) * 64);
    }
  } else {
    fetch_biases(t, kMlpThreads);
    for (int i = t; i < R * H / 4; i += kMlpThreads) {
      const int r = i / (H / 4), k4 = i % (H / 4);
      reinterpret_cast<float4*>(xs)[i] = (b0 + r < p.nb)
          ? reinterpret_cast<const float4*>(p.h + (b0 + r) * H)[k4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  rows_nt<R>(p.Wh, L2, H, xs, hs, p.rot);  // (its barrier publishes xs)
  __syncthreads();
  for (int i = t; i < R * L2; i += kMlpThreads) {
    const int r = i / L2, n = i % L2;
    const float v = hs[i] + bsh[n];
    hs[i] = v;
    if (b0 + r < p.nb) p.heads[(b0 + r) * L2 + n] = v;
  }
  __syncthreads();
  // reparameterisation + KL of row w (k_reparam_kl_fwd's arithmetic and lane order)
  if (w < R) {
    const int64_t b = b0 + w;
    const bool valid = b < p.nb;
    float kl = 0.f;
    for (int l = lane; l < L; l += 64) {
      const float m = hs[w * L2 + l], v = hs[w * L2 + L + l];
      const float ev = expf(v);
      kl += ((1.f + v) - m * m) - ev;
      float zv = m;
      if (p.train) {
        const float e = !valid ? 0.f : p.eps_in ? p.eps_in[b * L + l] : normal_f(p.seed, step, kTagEps, (uint64_t)(b * L + l));
        if (valid && p.eps) p.eps[b * L + l] = e;
        zv = m + e * expf(0.5f * v);
      }
      zs[w * L + l] = zv;
      if (valid) p.z[b * L + l] = zv;
    }
    kl = wave_sum(kl);
    if (lane == 0 && valid) p.kl_rows[b] = -0.5f * kl;
  }
  rows_nt<R>(p.Wa, D, L, zs, ys, p.rot);  // (its barrier publishes zs)
  __syncthreads();
  for (int i = t; i < R * D; i += kMlpThreads) {
    const int r = i / D, n = i % D;
    const int64_t b = b0 + r;
    const float pre = ys[i] + bsh[L2 + n];
    const float g = gelu_f(pre);
    float qv = g;
    if (p.train && b < p.nb)
      qv = g * dropout_mult(p.p_drop, p.scale, p.drop_mult, (uint64_t)(b * D + n), p.seed, step, kTagProjDrop);
    qs[i] = qv;
    if (b < p.nb) {
      p.p1[b * D + n] = pre;
      p.q[b * D + n] = qv;
    }
  }
  rows_nt<R>(p.Wb, D, D, qs, ys, p.rot);  // (its barrier publishes qs)
  __syncthreads();
  for (int i = t; i < R * D; i += kMlpThreads) {
    const int r = i / D, n = i % D;
    if (b0 + r < p.nb) p.u[(b0 + r) * D + n] = ys[i] + bsh[L2 + D + n];
  }
}

template <int R>
__global__ void __launch_bounds__(kMlpThreads) k_mlp_bwd_rows(MlpP p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int H = p.H, L = p.L, D = p.D, L2 = 2 * p.L;
  float* gs = smem;            // [R][D]  dU rows
  float* ps = gs + R * D;      // [R][D]  dp1
  float* ds = ps + R * D;      // [R][2L] dheads
  float* dhs = ds + R * L2;    // [R][H]  dh (LayerNorm backward)
  float* dxs = dhs + R * H;    // [R][H]  dxhat (LayerNorm backward)
  float* part = dxs + R * H;   // slice partials of rows_nn; then the LayerNorm column terms [3][R][H]
  // the epilogues' row inputs, fetched with dU so that no epilogue waits on its own loads
  float* pf_p1 = part + 4 * kMlpThreads * R;  // [R][D]
  float* pf_heads = pf_p1 + R * D;             // [R][2L]
  float* pf_eps = pf_heads + R * L2;           // [R][L]
  float* pf_xhat = pf_eps + R * L;             // [R][H]
  float* pf_lnw = pf_xhat + R * H;             // [H]
  float* pf_lnb = pf_lnw + H;                  // [H]
  float* pf_rstd = pf_lnb + H;                 // [R]
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * R;
  const int64_t step = load_step(p.step_dev);
  const float ks = p.ks_dev ? *p.ks_dev : p.ks;
  auto rows4 = [&](float* dst, const float* src, int w4) {  // R rows of w4 float4 (zero past the batch)
    for (int i = t; i < R * w4; i += kMlpThreads) {
      const int r = i / w4, k4 = i % w4;
      reinterpret_cast<float4*>(dst)[i] = (b0 + r < p.nb)
          ? reinterpret_cast<const float4*>(src + (b0 + r) * (int64_t)w4 * 4)[k4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  rows4(gs, p.dU, D / 4);
  rows4(pf_p1, p.p1, D / 4);
  rows4(pf_heads, p.heads, L2 / 4);
  if (p.train) rows4(pf_eps, p.eps, L / 4);
  if (p.ln_w) {
    rows4(pf_xhat, p.xhat, H / 4);
    for (int i = t; i < 2 * H; i += kMlpThreads) pf_lnw[i] = i < H ? p.ln_w[i] : p.ln_b[i - H];  // (pf_lnb follows)
    if (t < R) pf_rstd[t] = b0 + t < p.nb ? p.rstd[b0 + t] : 0.f;
  }
  // dp1 = (dU W_b) * dropmult * GELU'(p1)   (HVAE_EPI_GELU_DROP_BWD)
  rows_nn<R>(p.Wb, D, D, gs, part, p.rot, [&](int r, int n, float v) {
    const int64_t b = b0 + r;
    float g = 0.f;
    if (b < p.nb) {
      const float dm = p.train ? dropout_mult(p.p_drop, p.scale, p.drop_mult, (uint64_t)(b * D + n), p.seed, step,
                                              kTagProjDrop)
                               : 1.f;
      g = v * dm * gelu_grad_f(pf_p1[r * D + n]);
      p.dp1[b * D + n] = g;
    }
    ps[r * D + n] = g;
  });
  // dz = dp1 W_a -> dheads (HVAE_EPI_REPARAM_BWD)
  rows_nn<R>(p.Wa, L, D, ps, part, p.rot, [&](int r, int l, float v) {
    const int64_t b = b0 + r;
    float dmu = 0.f, dlv = 0.f;
    if (b < p.nb) {
      const float m = pf_heads[r * L2 + l], lv = pf_heads[r * L2 + L + l];
      const float gz = p.train ? v * pf_eps[r * L + l] * 0.5f * expf(0.5f * lv) : 0.f;
      dlv = gz + ks * 0.5f * (expf(lv) - 1.f);
      dmu = v + ks * m;
      p.dheads[b * L2 + l] = dmu;
      p.dheads[b * L2 + L + l] = dlv;
    }
    ds[r * L2 + l] = dmu;
    ds[r * L2 + L + l] = dlv;
  });
  // dh = dheads W_heads
  rows_nn<R>(p.Wh, H, L2, ds, part, p.rot, [&](int r, int n, float v) {
    if (b0 + r < p.nb) p.dh[(b0 + r) * H + n] = v;
    dhs[r * H + n] = v;
  });
  if (!p.ln_w) return;
  // ---- the last hidden layer's Dropout(GELU(LayerNorm(a))) backward (k_ln_gelu_drop_bwd's per-row arithmetic
  // and lane order, so da is the same): wave w takes row w; its column terms go to LDS, the block sums its rows
  // in order, and the last block to finish sums the blocks' partials in block order
  float* cg = part;          // dy * xhat
  float* cb = part + R * H;  // dy
  float* ca = part + 2 * R * H;  // da
  const int lane = t & 63, w = t >> 6;
  if (w < R) {
    const int64_t b = b0 + w;
    if (b < p.nb) {
      const float invH = 1.0f / (float)H, rs = pf_rstd[w];
      float s1 = 0.f, s2 = 0.f;
      for (int e = 4 * lane; e < H; e += 256) {
        const float4 xh = *reinterpret_cast<const float4*>(pf_xhat + w * H + e);
        const float4 lw = *reinterpret_cast<const float4*>(pf_lnw + e);
        const float4 lb = *reinterpret_cast<const float4*>(pf_lnb + e);
        const float xv[4] = {xh.x, xh.y, xh.z, xh.w}, wv[4] = {lw.x, lw.y, lw.z, lw.w};
        const float bv[4] = {lb.x, lb.y, lb.z, lb.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint64_t idx = (uint64_t)(b * H + e + i);
          const float dm = p.train ? dropout_mult(p.p_drop, p.scale, p.enc_drop_mult, idx, p.seed, step, p.enc_tag)
                                   : 1.f;
          const float dy = dhs[w * H + e + i] * dm * gelu_grad_f(xv[i] * wv[i] + bv[i]);
          const float dx = dy * wv[i];
          s1 += dx;
          s2 += dx * xv[i];
          cg[w * H + e + i] = dy * xv[i];
          cb[w * H + e + i] = dy;
          dxs[w * H + e + i] = dx;
        }
      }
      const float m1 = wave_sum(s1) * invH, m2 = wave_sum(s2) * invH;
      for (int e = 4 * lane; e < H; e += 256) {
        const float4 xh = *reinterpret_cast<const float4*>(pf_xhat + w * H + e);
        float4 o;
        o.x = rs * (dxs[w * H + e + 0] - m1 - xh.x * m2);
        o.y = rs * (dxs[w * H + e + 1] - m1 - xh.y * m2);
        o.z = rs * (dxs[w * H + e + 2] - m1 - xh.z * m2);
        o.w = rs * (dxs[w * H + e + 3] - m1 - xh.w * m2);
        *reinterpret_cast<float4*>(p.da + b * H + e) = o;
        ca[w * H + e + 0] = o.x; ca[w * H + e + 1] = o.y; ca[w * H + e + 2] = o.z; ca[w * H + e + 3] = o.w;
      }
    } else {
      for (int e = lane; e < H; e += 64) cg[w * H + e] = cb[w * H + e] = ca[w * H + e] = 0.f;
    }
  }
  __syncthreads();
  float* gpart = p.ln_part;  // [blocks][3][H]
  if (!p.d_ln_w) {  // deferred: the block's partials only, added in block order by the caller's next launch
    for (int i = t; i < 3 * H; i += kMlpThreads) {
      const int kind = i / H, col = i % H;
      const float* src = part + kind * R * H + col;
      float v = src[0];
#pragma unroll
      for (int r = 1; r < R; ++r) v += src[r * H];
      gpart[(int64_t)blockIdx.x * 3 * H + i] = v;
    }
    return;
  }
  for (int i = t; i < 3 * H; i += kMlpThreads) {
    const int kind = i / H, col = i % H;
    const float* src = part + kind * R * H + col;
    float v = src[0];
#pragma unroll
    for (int r = 1; r < R; ++r) v += src[r * H];
    st_shared_f(&gpart[(int64_t)blockIdx.x * 3 * H + i], v);
  }
  if (!last_block_arrives(p.ln_ticket, gridDim.x)) return;
  const int np = gridDim.x;
  for (int i = t; i < 3 * H; i += kMlpThreads) {
    // the blocks' partials in block order, 32 loads in flight (one round trip at B = 64)
    float sum = 0.f;
    for (int q = 0; q < np; q += 32) {
      float v[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) v[j] = q + j < np ? ld_shared_f(&gpart[(int64_t)(q + j) * 3 * H + i]) : 0.f;
#pragma unroll
      for (int j = 0; j < 32; ++j)
        if (q + j < np) sum += v[j];
    }
    if (i < H) p.d_ln_w[i] = sum;
    else if (i < 2 * H) p.d_ln_b[i - H] = sum;
    else if (p.d_bias) p.d_bias[i - 2 * H] = sum;
  }
}

// rows per block: enough blocks to spread the weight streaming over the CUs, few enough that the
// weights are not re-read from L2 more often than needed
// HVAE_MLP_R (A/B build): force 1, 2 or 4 rows per block
static int mlp_rows_per_block(int64_t nb) {
  if (const char* e = ab_getenv("HVAE_MLP_R")) {
    const int r = std::atoi(e);
    if (r == 1 || r == 2 || r == 4) return r;
  }
  return nb <= 32 ? 1 : nb <= 512 ? 2 : 4;
}

static size_t mlp_fwd_smem(int R, const hvae_mlp_rows* a) {
  // + the biases, + the encoder layer's per-wave partials (kMlpWaves rows of H)
  return ((size_t)R * (a->H + 3 * a->L + 2 * a->D) + 2 * a->L + 2 * a->D + (a->enc_x ? (size_t)kMlpWaves * a->H : 0)) * 4;
}
static size_t mlp_bwd_smem(int R, const hvae_mlp_rows* a) {
  return (size_t)R * (2 * a->D + 2 * a->L + 2 * a->H) * 4 + (size_t)4 * kMlpThreads * R * 4 +
         ((size_t)R * (a->D + 3 * a->L + a->H) + 2 * a->H + 4) * 4;  // + the prefetched epilogue inputs
}

constexpr size_t kMlpLdsMax = 159 * 1024;  // gfx950 LDS per CU (160 KiB) less the kernels' static LDS

// launch with `smem` bytes of dynamic LDS, the kernel's limit raised to kMlpLdsMax once
#define HVAE_MLP_LAUNCH(KERNEL)                                                                        \
  do {                                                                                                 \
    static const bool attr_ok =                                                                        \
        hipFuncSetAttribute((const void*)KERNEL, hipFuncAttributeMaxDynamicSharedMemorySize,           \
                            (int)kMlpLdsMax) == hipSuccess;                                            \
    HVAE_REQUIRE(attr_ok, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");                   \
    KERNEL<<<grid, kMlpThreads, smem, st>>>(p);                                                        \
  } while (0)

static int mlp_setup(const hvae_mlp_rows* a, bool fwd, MlpP& p) {
  HVAE_REQUIRE(a, "hvae_mlp_rows: null args");
  HVAE_REQUIRE(a->nb >= 0 && a->nb <= HVAE_MLP_ROWS_MAX_NB, "hvae_mlp_rows: nb outside [0, HVAE_MLP_ROWS_MAX_NB]");
  for (int64_t v : {a->H, a->L, a->D})
    HVAE_REQUIRE(v >= 32 && v <= 1024 && v % 32 == 0, "hvae_mlp_rows: H, L, D must be multiples of 32 in [32, 1024]");
  HVAE_REQUIRE(a->W_heads && a->W_a && a->W_b, "hvae_mlp_rows: null weights");
  if (fwd) {
    HVAE_REQUIRE(a->b_heads && a->b_a && a->b_b, "hvae_mlp_fwd_rows: null biases");
    HVAE_REQUIRE(a->h && a->heads && a->z && a->kl_rows && a->p1 && a->q && a->u, "hvae_mlp_fwd_rows: null buffer");
    if (a->enc_x) {
      const hvae_csr_batch* x = a->enc_x;
      HVAE_REQUIRE(x->row_ptr && x->col_idx && x->vals && x->nb == a->nb && a->w1t && a->b1 && a->ln_w && a->ln_b,
                   "hvae_mlp_fwd_rows: the encoder layer needs enc_x (nb rows), w1t, b1, ln_w, ln_b");
      HVAE_REQUIRE(a->H <= 512, "hvae_mlp_fwd_rows: the fused encoder layer takes H <= 512 (hvae_encoder_fwd beyond)");
      p.e_row_ptr = x->row_ptr; p.e_col_idx = x->col_idx; p.e_vals = x->vals; p.e_rows = x->rows;
      p.e_rows_offset = x->rows_offset;
      p.enc_w1t = a->w1t; p.enc_b1 = a->b1; p.ln_w = a->ln_w; p.ln_b = a->ln_b; p.enc_drop_mult = a->enc_drop_mult;
      p.h_out = const_cast<float*>(a->h); p.xhat_out = const_cast<float*>(a->xhat);
      p.rstd_out = const_cast<float*>(a->rstd);
      if (a->adam) {
        HVAE_REQUIRE(a->adam->step_dev && a->adam_m && a->adam_v && a->last_step && a->adam_tab && a->H % 4 == 0,
                     "hvae_mlp_fwd_rows: lazy-Adam reads need adam (step_dev), adam_m, adam_v, last_step, adam_tab");
        p.enc_lazy = 1;
        p.aa = to_args(a->adam);
        p.am = a->adam_m; p.av = a->adam_v; p.ls = a->last_step; p.atab = (const float2*)a->adam_tab;
      }
    }
  } else {
    HVAE_REQUIRE(a->dU && a->p1 && a->heads && a->dp1 && a->dheads && a->dh, "hvae_mlp_bwd_rows: null buffer");
    HVAE_REQUIRE(!a->train || a->eps, "hvae_mlp_bwd_rows: train backward needs eps");
  }
  p.nb = a->nb;
  p.H = (int)a->H; p.L = (int)a->L; p.D = (int)a->D;
  p.Wh = a->W_heads; p.bh = a->b_heads; p.Wa = a->W_a; p.ba = a->b_a; p.Wb = a->W_b; p.bb = a->b_b;
  p.train = a->train;
  p.p_drop = a->p_drop;
  p.scale = (a->p_drop < 1.f) ? 1.0f / (1.0f - a->p_drop) : 0.f;
  p.drop_mult = a->drop_mult; p.eps_in = a->eps_in; p.seed = a->seed; p.step_dev = a->step_dev;
  p.h = a->h; p.heads = a->heads; p.z = a->z; p.eps = a->eps; p.kl_rows = a->kl_rows;
  p.p1 = a->p1; p.q = a->q; p.u = a->u;
  p.dU = a->dU; p.ks = a->ks; p.ks_dev = a->ks_dev; p.dp1 = a->dp1; p.dheads = a->dheads; p.dh = a->dh;
  const char* rot = ab_getenv("HVAE_MLP_ROT");
  p.rot = rot ? std::atoi(rot) : 1;
  return HVAE_OK;
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_mlp_fwd_rows(const hvae_mlp_rows* a, void* stream) {
  MlpP p{};
  if (int rc = mlp_setup(a, true, p)) return rc;
  if (a->nb == 0) return HVAE_OK;
  const int R = mlp_rows_per_block(a->nb);
  size_t smem = mlp_fwd_smem(R, a);
  HVAE_REQUIRE(smem <= kMlpLdsMax, "hvae_mlp_fwd_rows: activations exceed the LDS");
  unsigned nblk = (unsigned)cdiv(a->nb, R);
  HVAE_REQUIRE(!a->plan_x == !a->plan_rg, "hvae_mlp_fwd_rows: plan_x and plan_rg go together");
  if (a->plan_x) {
    const hvae_csr_batch* x = a->plan_x;
    const hvae_rowgrad* rg = a->plan_rg;
    HVAE_REQUIRE(x->row_ptr && x->col_idx && x->vals && x->nb == a->nb, "hvae_mlp_fwd_rows: bad plan batch");
    HVAE_REQUIRE(rg->slot_of && rg->item_of && rg->seg_off && rg->contrib_row && rg->contrib_val &&
                 rg->contrib_slot && rg->n_unique && rg->n_items == x->n_items,
                 "hvae_mlp_fwd_rows: bad plan row gradient");
    HVAE_REQUIRE(rg->cap <= kPlanSmallCap && x->nb <= kPlanSmallRows,
                 "hvae_mlp_fwd_rows: the batch's plan does not fit one block (use hvae_w1_rowgrad_plan)");
    p.pl_row_ptr = x->row_ptr; p.pl_col_idx = x->col_idx; p.pl_vals = x->vals; p.pl_rows = x->rows;
    p.pl_rows_offset = x->rows_offset; p.pl_nb = x->nb;
    p.plan_slot_of = rg->slot_of; p.pl_item_of = rg->item_of; p.pl_seg_off = rg->seg_off;
    p.pl_contrib_row = rg->contrib_row; p.pl_contrib_val = rg->contrib_val; p.pl_contrib_slot = rg->contrib_slot;
    p.pl_n_unique = rg->n_unique;
    smem = std::max(smem, kPlanSmallLds);
    ++nblk;
  }
  const dim3 grid(nblk);
  hipStream_t st = as_stream(stream);
  ProbeScope probe("mlp_fwd", st);
  if (R == 1) HVAE_MLP_LAUNCH(k_mlp_fwd_rows<1>);
  else if (R == 2) HVAE_MLP_LAUNCH(k_mlp_fwd_rows<2>);
  else HVAE_MLP_LAUNCH(k_mlp_fwd_rows<4>);
  HVAE_LAUNCH_CHECK("k_mlp_fwd_rows");
  return HVAE_OK;
}

// the shapes hvae_mlp_fwd_rows / _bwd_rows accept (mlp_setup's width rules, both directions' LDS at this batch's
// rows per block), so that the host picks the GEMM chain instead of a launch that would fail its HVAE_REQUIRE
extern "C" int hvae_mlp_rows_supported(int64_t nb, int64_t H, int64_t L, int64_t D, int fused_enc) {
  if (nb <= 0 || nb > HVAE_MLP_ROWS_MAX_NB) return 0;
  for (int64_t v : {H, L, D})
    if (v < 32 || v > 1024 || v % 32) return 0;
  if (fused_enc && H > 512) return 0;
  hvae_mlp_rows a{};
  hvae_csr_batch x{};  // (only its presence counts: the fused encoder layer's LDS)
  a.nb = nb; a.H = H; a.L = L; a.D = D;
  if (fused_enc) a.enc_x = &x;
  const int R = mlp_rows_per_block(nb);
  return mlp_fwd_smem(R, &a) <= kMlpLdsMax && mlp_bwd_smem(R, &a) <= kMlpLdsMax;
}

extern "C" int64_t hvae_mlp_rows_blocks(int64_t nb) { return nb > 0 ? cdiv(nb, mlp_rows_per_block(nb)) : 0; }

extern "C" size_t hvae_mlp_bwd_rows_workspace(int64_t nb, int64_t H) {
  return nb > 0 ? (size_t)cdiv(nb, mlp_rows_per_block(nb)) * 3 * H * sizeof(float) : 0;
}

extern "C" int hvae_mlp_bwd_rows(const hvae_mlp_rows* a, void* stream) {
  MlpP p{};
  if (int rc = mlp_setup(a, false, p)) return rc;
  if (a->ln_w) {
    const bool deferred = !a->d_ln_w && !a->d_ln_b && !a->d_bias;
    HVAE_REQUIRE(a->ln_b && a->xhat && a->rstd && a->da && ((a->d_ln_w && a->d_ln_b) || deferred),
                 "hvae_mlp_bwd_rows: LayerNorm backward needs ln_b, xhat, rstd, da and d_ln_w, d_ln_b (or none of "
                 "d_ln_w, d_ln_b, d_bias: deferred column sums)");
    if (a->nb == 0) {
      hipStream_t st = as_stream(stream);
      if (deferred) return HVAE_OK;  // no blocks, no partials
      HVAE_HIP(hipMemsetAsync(a->d_ln_w, 0, a->H * sizeof(float), st));
      HVAE_HIP(hipMemsetAsync(a->d_ln_b, 0, a->H * sizeof(float), st));
      if (a->d_bias) HVAE_HIP(hipMemsetAsync(a->d_bias, 0, a->H * sizeof(float), st));
      return HVAE_OK;
    }
    const size_t need = hvae_mlp_bwd_rows_workspace(a->nb, a->H);
    if (!a->ws || a->ws_bytes < need)
      HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae_mlp_bwd_rows: workspace %zu < %zu", a->ws_bytes, need);
    p.ln_w = a->ln_w; p.ln_b = a->ln_b; p.xhat = a->xhat; p.rstd = a->rstd; p.enc_drop_mult = a->enc_drop_mult;
    p.enc_tag = kTagEncDrop + a->enc_layer;
    p.da = a->da; p.d_ln_w = a->d_ln_w; p.d_ln_b = a->d_ln_b; p.d_bias = a->d_bias;
    p.ln_part = (float*)a->ws;
    if (!deferred && !(p.ln_ticket = ticket_slice())) return HVAE_ERR_HIP;
  }
  if (a->nb == 0) return HVAE_OK;
  const int R = mlp_rows_per_block(a->nb);
  const size_t smem = mlp_bwd_smem(R, a);
  HVAE_REQUIRE(smem <= kMlpLdsMax, "hvae_mlp_bwd_rows: activations exceed the LDS");
  const dim3 grid((unsigned)cdiv(a->nb, R));
  hipStream_t st = as_stream(stream);
  ProbeScope probe("mlp_bwd", st);
  if (R == 1) HVAE_MLP_LAUNCH(k_mlp_bwd_rows<1>);
  else if (R == 2) HVAE_MLP_LAUNCH(k_mlp_bwd_rows<2>);
  else HVAE_MLP_LAUNCH(k_mlp_bwd_rows<4>);
  HVAE_LAUNCH_CHECK("k_mlp_bwd_rows");
  return HVAE_OK;
}
