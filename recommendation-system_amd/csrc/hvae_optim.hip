// hvae_optim.hip -- gradient clipping and Adam (K13, K14 of SURVEY §2.1).
//
// Reference: VAETrainer.train_epoch (src/ml/train.py:88-92):
//   torch.nn.utils.clip_grad_norm_(params, max_norm=5.0); optimizer.step()
// with optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8, weight_decay) built at
// src/ml/train.py:63. Both passes are HBM-bound; the clip multiplier never
// takes its own pass over the gradients -- it is read by the Adam launches.
#include <algorithm>
#include <cstdlib>

#include "hvae_common.h"
#include "hvae_adam.h"

namespace hvae {

constexpr int kNormBlocks = 512;

// Sum of squares over a dense flat gradient + the valid rows of a row-sparse
// one, fixed grid, per-block partials in fp64 (deterministic).
// Global squared norm in fp64 over [dense grads | row-sparse W1 rows]; the last
// block to finish reduces the per-block partials in block order, forms torch's
// clip coefficient and (optionally) advances the step counters:
//   step_snap = step; step += 1; boff += advance
// so that the Adam launches that follow read the pre-increment step from
// step_snap and no separate counter launch is needed.

struct ClipArgs {
  const float* g; int64_t n;
  const float* rows; const int32_t* n_unique; int64_t H;
  const double* rowsq;  // per-row sums of squares from the apply (then rows is not read), or NULL
  double* part; unsigned* ticket;
  float max_norm; float* norm_out; float* coef_out;
  int64_t* step; int64_t* step_snap; int64_t* boff; int64_t advance;
  float2* tab; double lr, b1, b2;  // optional: record the coming Adam step's scalars in tab[step + 1]
};

__global__ void __launch_bounds__(256) k_clip_norm(ClipArgs a) {
  __shared__ double red[4];
  const int64_t nr = a.rows ? (int64_t)(*a.n_unique) * a.H : 0;
  double s = 0.0;
  const int64_t gtid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // sum of squares of one segment: float4 loads, 4 of them in flight per thread per round (a
  // one-load-per-iteration loop is a chain of memory latencies), scalar tail; fixed order
  auto seg = [&](const float* __restrict__ x, int64_t n) {
    const bool vec = ((uintptr_t)x % 16) == 0;
    const int64_t n4 = vec ? n / 4 : 0;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (int64_t i = gtid; i < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t j = i + u * stride;
        v[u] = j < n4 ? x4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        s += ((double)v[u].x * v[u].x + (double)v[u].y * v[u].y) + ((double)v[u].z * v[u].z + (double)v[u].w * v[u].w);
    }
    for (int64_t i = 4 * n4 + gtid; i < n; i += stride) s += (double)x[i] * (double)x[i];
  };
  if (a.n) seg(a.g, a.n);
  if (a.rowsq) {
    const int64_t np = a.rows ? (int64_t)(*a.n_unique) * kRowSqParts : 0;
    for (int64_t i = gtid; i < np; i += stride) s += a.rowsq[i];
  } else if (nr) {
    seg(a.rows, nr);
  }
  s = wave_sum_d(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) st_shared_d(&a.part[blockIdx.x], ((red[0] + red[1]) + red[2]) + red[3]);
  if (!last_block_arrives(a.ticket, gridDim.x)) return;
  double t = 0.0;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) t += ld_shared_d(&a.part[i]);
  t = wave_sum_d(t);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(((red[0] + red[1]) + red[2]) + red[3]);
    // torch: clip_coef = max_norm / (total_norm + 1e-6); clamp(max=1.0)
    const float coef = fminf(a.max_norm / (norm + 1e-6f), 1.0f);
    if (a.norm_out) *a.norm_out = norm;
    *a.coef_out = coef;
    if (a.step) {
      const int64_t st = *a.step;
      if (a.step_snap) *a.step_snap = st;
      *a.step = st + 1;
      // computed once here, so the Adam launch that follows reads them instead of every
      // thread of it evaluating two double pow()s
      if (a.tab) a.tab[st + 1] = adam_step_consts(a.lr, a.b1, a.b2, st + 1);
    }
    if (a.boff) *a.boff += a.advance;
  }
}

__global__ void __launch_bounds__(256) k_adam_dense(AdamArgs a, float* __restrict__ p, float* __restrict__ m,
                                                    float* __restrict__ v, const float* __restrict__ g,
                                                    int64_t n) {
  const AdamKExact k = adam_consts_exact(a);  // the eager drop-in step: torch's CPU arithmetic (hvae_adam.h)
  const float coef = a.coef_dev ? *a.coef_dev : 1.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem_exact(pp, mm, vv, g[i] * coef, k);
    p[i] = pp; m[i] = mm; v[i] = vv;
  }
}

// Item-major W1t [N, H] with a row-sparse gradient: float4 per thread.
__global__ void __launch_bounds__(256) k_adam_rows(AdamArgs a, float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, const float* __restrict__ rows,
                                                   const int32_t* __restrict__ slot_of,
                                                   const int32_t* __restrict__ item_of,
                                                   const int32_t* __restrict__ n_unique, int64_t N,
                                                   int64_t H) {
  const AdamK k = adam_consts(a);
  const float coef = a.coef_dev ? *a.coef_dev : 1.f;
  const int nu = *n_unique;
  const int64_t H4 = H / 4, n4 = N * H4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const int64_t row = i / H4, c = i - row * H4;
    const int s = slot_of[row];
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (s >= 0 && s < nu && item_of[s] == (int32_t)row) {
      gv = *reinterpret_cast<const float4*>(rows + (int64_t)s * H + 4 * c);
      gv.x *= coef; gv.y *= coef; gv.z *= coef; gv.w *= coef;
    }
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adam_elem(pp.x, mm.x, vv.x, gv.x, k);
    adam_elem(pp.y, mm.y, vv.y, gv.y, k);
    adam_elem(pp.z, mm.z, vv.z, gv.z, k);
    adam_elem(pp.w, mm.w, vv.w, gv.w, k);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
}

// Both updates of the step in one launch: blocks [0, nb_rows) stream W1t (as
// k_adam_rows), the rest the dense segment (as k_adam_dense).
__global__ void __launch_bounds__(256) k_adam_flat(AdamArgs a, float* __restrict__ p, float* __restrict__ m,
                                                   float* __restrict__ v, const float* __restrict__ rows,
                                                   const int32_t* __restrict__ slot_of,
                                                   const int32_t* __restrict__ item_of,
                                                   const int32_t* __restrict__ n_unique, int64_t N, int64_t H,
                                                   const float* __restrict__ g_dense, int64_t dense_off,
                                                   int64_t n_dense, int nb_rows) {
  const AdamK k = adam_consts(a);
  const float coef = a.coef_dev ? *a.coef_dev : 1.f;
  if ((int)blockIdx.x < nb_rows) {
    const int nu = *n_unique;
    const int64_t H4 = H / 4, n4 = N * H4;
    const int64_t stride = (int64_t)nb_rows * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
      const int64_t row = i / H4, c = i - row * H4;
      const int s = slot_of[row];
      float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s >= 0 && s < nu && item_of[s] == (int32_t)row) {
        gv = *reinterpret_cast<const float4*>(rows + (int64_t)s * H + 4 * c);
        gv.x *= coef; gv.y *= coef; gv.z *= coef; gv.w *= coef;
      }
      float4 pp = reinterpret_cast<float4*>(p)[i];
      float4 mm = reinterpret_cast<float4*>(m)[i];
      float4 vv = reinterpret_cast<float4*>(v)[i];
      adam_elem(pp.x, mm.x, vv.x, gv.x, k);
      adam_elem(pp.y, mm.y, vv.y, gv.y, k);
      adam_elem(pp.z, mm.z, vv.z, gv.z, k);
      adam_elem(pp.w, mm.w, vv.w, gv.w, k);
      reinterpret_cast<float4*>(p)[i] = pp;
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
  } else {
    float* pd = p + dense_off;
    float* md = m + dense_off;
    float* vd = v + dense_off;
    const int64_t stride = (int64_t)(gridDim.x - nb_rows) * blockDim.x;
    for (int64_t i = (int64_t)(blockIdx.x - nb_rows) * blockDim.x + threadIdx.x; i < n_dense; i += stride) {
      float pp = pd[i], mm = md[i], vv = vd[i];
      adam_elem(pp, mm, vv, g_dense[i] * coef, k);
      pd[i] = pp; md[i] = mm; vd[i] = vv;
    }
  }
}

constexpr int kCatchupBlocks = 1024;  // k_adam_catchup_csr: blocks to aim for over a small batch
// Row groups (rows x float4 columns) per barrier in the row kernels. Four groups' loads in flight per barrier
// (HVAE_ADAM_UNROLL=4, A/B build) ran slower than one everywhere -- Syn-10M 11.55-11.62 vs 11.52 ms per step,
// Syn-1M 1.208 vs 1.194, All_Beauty 0.143 vs 0.134 (adam_rows 20 vs 13 us; profiles/r04_adam_unroll_ab.jsonl):
// the unrolled kernels hold 164 VGPRs (3 waves per SIMD) and a quarter of the blocks.
constexpr int kAdamUnroll = 1;
// A/B (HVAE_AB builds): HVAE_ADAM_UNROLL=4 keeps four row groups in flight, HVAE_CATCHUP_PONLY=0 stores m, v in
// the CSR catch-up too
static int adam_unroll() {
  const char* e = ab_getenv("HVAE_ADAM_UNROLL");
  return e && std::atoi(e) == 4 ? 4 : kAdamUnroll;
}
static int catchup_p_only() {
  const char* e = ab_getenv("HVAE_CATCHUP_PONLY");
  return e && std::atoi(e) == 0 ? 0 : 1;
}
#ifdef HVAE_AB
#define HVAE_ADAM_U_CALL(U_, CALL) \
  do { if ((U_) == 4) { constexpr int U = 4; CALL; } else { constexpr int U = kAdamUnroll; CALL; } } while (0)
#else
#define HVAE_ADAM_U_CALL(U_, CALL) do { constexpr int U = kAdamUnroll; CALL; } while (0)
#endif

// Bring rows up to the completed step count *step: the batch's rows (item_of /
// n_unique) or, with item_of == NULL, all N rows.
template <int U>
__global__ void __launch_bounds__(256) k_adam_catchup(AdamArgs a, const float2* __restrict__ tab, float* p, float* m,
                                                      float* v, int32_t* __restrict__ last_step,
                                                      const int32_t* __restrict__ item_of,
                                                      const int32_t* __restrict__ n_unique, int64_t N, int64_t H,
                                                      RowMap rm) {
  const int to = (int)load_step(a.step_dev);
  const int64_t nrows = item_of ? (int64_t)*n_unique : N;
  const int64_t H4 = H / 4;
  const int rr = threadIdx.x / rm.h4s, c0 = threadIdx.x % rm.h4s;
  const AdamK none{};
  const int64_t span = (int64_t)rm.rpb * U;
  for (int64_t g0 = (int64_t)blockIdx.x * span; g0 < nrows; g0 += (int64_t)gridDim.x * span) {
    int64_t j[U];
    int from[U], pst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = g0 + (int64_t)u * rm.rpb + rr;
      const bool act = rr < rm.rpb && r < nrows;
      j[u] = act ? (item_of ? (int64_t)item_of[r] : r) : 0;
      const int32_t ls = act ? last_step[j[u]] : to;
      from[u] = ls_mv(ls);
      pst[u] = ls_p(ls);
    }
    for (int64_t c = c0; c < H4; c += rm.h4s) {
      ColState cs[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (from[u] < to) cs[u] = col_load(p, m, v, j[u] * H4 + c);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (from[u] < to)
          col_math_lazy(a, tab, cs[u], from[u], pst[u], to, false, none, make_float4(0.f, 0.f, 0.f, 0.f));
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (from[u] < to) col_store(p, m, v, j[u] * H4 + c, cs[u]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c0 == 0 && from[u] < to) last_step[j[u]] = to;
  }
}

// The same catch-up from the batch's CSR entries instead of the W1-gradient plan's unique-row list, so
// that it does not wait for the plan (which then runs beside the forward on another stream). A row listed
// by several entries is claimed once: the entry's thread moves last_step[j] from its value to `to` with an
// atomicCAS, and only the winner's row is replayed; the replayed arithmetic is the same, so the result is
// bitwise that of k_adam_catchup. Blocks take (batch row, slice) pairs: slice s of a row is its entries
// s, s + S, s + 2 S, .. (S slices per row, so that a small batch still spreads its rows' replays over the
// machine: at B = 64 one block per row left 64 blocks walking ~20 rows each, one memory round trip after
// another); all of a group's entries claim at once, then every thread walks the claimed rows' float4 columns.
// With a deferred step recorded (hdr != NULL, ABI 5), a listed row that carries it (last_step bit 30) is claimed
// like any other and takes that step here -- its missed steps replayed, then step hdr->t with its gradient row
// times hdr->coef, k_adam_lazy's float operations -- and stores p, m and v (the caller passes to == hdr->t).
template <int U>
__global__ void __launch_bounds__(256) k_adam_catchup_csr(AdamArgs a, const float2* __restrict__ tab, float* p,
                                                          float* m, float* v, int32_t* __restrict__ last_step,
                                                          hvae_csr_batch x, int64_t H, int S, int p_only_arg,
                                                          const int32_t* __restrict__ pend_slot,
                                                          const PendHdr* __restrict__ hdr) {
  __shared__ int s_j[256], s_from[256], s_pst[256], s_slot[256];
  __shared__ int s_n;
  const int to = (int)load_step(a.step_dev);
  const int64_t H4 = H / 4;
  const AdamK none{};
  // the recorded step's constants and gradient rows (when one is pending at step `to`)
  const bool pend_on = hdr != nullptr && hdr->t == (int64_t)to && to > 0;
  const float* prow = pend_on ? hdr->rows : nullptr;
  const int64_t pld = pend_on ? hdr->ld : 0;
  const float pcoef = pend_on ? hdr->coef : 1.f;
  const AdamK kp = pend_on ? adam_consts_tab(a, tab[to]) : none;
  // p alone moves ahead unless weight decay couples m, v to p, or m, v are too far behind to say so in the stamp
  const bool p_only_ok = a.wd == 0.0 && p_only_arg;
  const int sl = (int)(blockIdx.x % (unsigned)S);
  for (int64_t b = blockIdx.x / S; b < x.nb; b += gridDim.x / S) {
    const int64_t r = batch_row(x.rows, x.rows_offset, b);
    const int64_t e0 = x.row_ptr[r], e1 = x.row_ptr[r + 1];
    const int64_t cnt = e1 - e0 > sl ? (e1 - e0 - sl + S - 1) / S : 0;  // this slice's entries
    for (int64_t g0 = 0; g0 < cnt; g0 += 256) {
      if (threadIdx.x == 0) s_n = 0;
      __syncthreads();
      const int64_t i = g0 + threadIdx.x;
      if (i < cnt) {
        const int j = x.col_idx[e0 + sl + i * S];
        // one compare-and-swap claims the row: the entry that moves last_step[j] from its value to the caught-up
        // stamp replays it; entries that find p already at `to` (another entry claimed it) do nothing
        int32_t old = __hip_atomic_load(last_step + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (ls_p(old) < to) {
          const bool pend = pend_on && (old & kPendBit);
          const int mv = ls_mv(old);
          const bool p_only = !pend && p_only_ok && to - mv <= kPAheadMax;
          const int32_t want = p_only ? (int32_t)(mv | ((to - mv) << kStepBits)) : (int32_t)to;
          if (__hip_atomic_compare_exchange_strong(last_step + j, &old, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)) {
            const int k = atomicAdd(&s_n, 1);
            s_j[k] = j;
            s_from[k] = p_only ? -1 - mv : mv;  // negative: store p only
            s_pst[k] = ls_p(old);
            s_slot[k] = pend ? pend_slot[j] : -1;  // >= 0: take the recorded step with this gradient row
            break;
          }
        }
      }
      __syncthreads();
      const int64_t work = (int64_t)s_n * H4;
      for (int64_t i0 = threadIdx.x; i0 < work; i0 += (int64_t)blockDim.x * U) {
        ColState cs[U];
        int64_t col[U];
        int fr[U], ps[U], sl[U];
        float4 gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t idx = i0 + (int64_t)u * blockDim.x;
          const int k = idx < work ? (int)(idx / H4) : 0;
          col[u] = idx < work ? (int64_t)s_j[k] * H4 + idx % H4 : -1;
          fr[u] = s_from[k];
          ps[u] = s_pst[k];
          sl[u] = pend_on ? s_slot[k] : -1;
          if (col[u] >= 0) cs[u] = col_load(p, m, v, col[u]);
          if (col[u] >= 0 && sl[u] >= 0) gv[u] = *reinterpret_cast<const float4*>(prow + sl[u] * pld + 4 * (idx % H4));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (col[u] < 0) continue;
          if (sl[u] >= 0) {  // k_adam_lazy's row update: replay to to - 1, then step `to` with coef * g
            float4 g = gv[u];
            g.x *= pcoef; g.y *= pcoef; g.z *= pcoef; g.w *= pcoef;
            col_math_lazy(a, tab, cs[u], fr[u], ps[u], to - 1, true, kp, g);
          } else {
            col_math_lazy(a, tab, cs[u], fr[u] < 0 ? -1 - fr[u] : fr[u], ps[u], to, false, none,
                          make_float4(0.f, 0.f, 0.f, 0.f));
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (col[u] < 0) continue;
          if (fr[u] < 0) reinterpret_cast<float4*>(p)[col[u]] = cs[u].p;
          else col_store(p, m, v, col[u], cs[u]);
        }
      }
      __syncthreads();
    }
  }
}

// The step's update with lazy W1t. Blocks [0, nb_rows) take the gradient rows
// (replay missed steps, then step t = *step + 1 with the clipped gradient);
// blocks [nb_rows, nb_rows + nb_sweep) bring one of `period` row ranges (rotating
// with t) through step t with g = 0 -- skipping rows with a gradient, which the first
// group owns -- so that no row ever lags more than `period` steps; the rest run the
// dense segment. Row work is column-parallel (RowMap).
// The period trades the sweep's bytes (24 H B per swept row) against longer replays in the catch-up: with the
// hardware square root and reciprocal (adam_elem) the replays are cheap, and at the Syn-10M shard a period of
// 8 / 16 / 32 ran 11.74 / 11.59 / 11.53 ms per step (adam_rows 457 / 318 / 251 us, catch-up 168 / 172 / 186 us;
// profiles/r04_lazy_sweep_period_ab.jsonl), at Syn-1M (N = 100 K) 32 saved 11 us; but where a batch touches a
// large share of the items (All_Beauty, N = 12,101: ~500 rows a step) the catch-up's longer replays cost more
// than the sweep saves (0.136 -> 0.146 ms per step at 32), so small item counts keep 8. Replays stay at most
// `period` steps long. HVAE_LAZY_SWEEP forces one period for every N.
#ifndef HVAE_LAZY_SWEEP
#define HVAE_LAZY_SWEEP 0
#endif
constexpr int64_t kLazySweepLargeN = 65536;
static int lazy_sweep_period(int64_t N) {
  if (HVAE_LAZY_SWEEP > 0) return HVAE_LAZY_SWEEP;
  return N >= kLazySweepLargeN ? 32 : 8;
}
template <int U>
__global__ void __launch_bounds__(256) k_adam_lazy(AdamArgs a, float2* __restrict__ tab, float* __restrict__ p,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int32_t* __restrict__ last_step, const float* __restrict__ rows,
                                                   const int32_t* __restrict__ slot_of,
                                                   const int32_t* __restrict__ item_of,
                                                   const int32_t* __restrict__ n_unique, int64_t N, int64_t H,
                                                   const float* __restrict__ g_dense, int64_t dense_off,
                                                   int64_t n_dense, int nb_rows, int nb_sweep, int period,
                                                   RowMap rm, int32_t* __restrict__ pend_slot,
                                                   int32_t* __restrict__ pend_item, PendHdr* __restrict__ hdr) {
  const int t = (int)load_step(a.step_dev) + 1;
  // tab[t] is written by hvae_clip_grad_norm_step_adam just before; a zero entry means no one did
  const float2 c0t = tab[t];
  const bool have = c0t.x != 0.f || c0t.y != 0.f;
  const AdamK k = have ? adam_consts_tab(a, c0t) : adam_consts(a);
  const float coef = a.coef_dev ? *a.coef_dev : 1.f;
  if (!have && blockIdx.x == 0 && threadIdx.x == 0) tab[t] = make_float2(k.lr_over_bc1, k.inv_bc2_sqrt);
  const int nu = *n_unique;
  const int64_t H4 = H / 4;
  const int rr = threadIdx.x / rm.h4s, cc = threadIdx.x % rm.h4s;
  const int64_t span = (int64_t)rm.rpb * U;
  if (hdr != nullptr && (int)blockIdx.x < nb_rows) {
    // deferred (hvae_adam_lazy_defer): the gradient rows are recorded as pending, nothing moves; the next
    // catch-up or k_adam_pending applies step t to each of them
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      hdr->t = t; hdr->rows = rows; hdr->ld = H; hdr->coef = coef; hdr->n = nu;
    }
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nu; s += (int64_t)nb_rows * blockDim.x) {
      const int32_t j = item_of[s];
      pend_item[s] = j;
      pend_slot[j] = (int32_t)s;
      last_step[j] = last_step[j] | kPendBit;
    }
  } else if ((int)blockIdx.x < nb_rows) {
    for (int64_t g0 = (int64_t)blockIdx.x * span; g0 < nu; g0 += (int64_t)nb_rows * span) {
      int64_t sidx[U], j[U];
      int from[U], pst[U];
      bool act[U];
      // the row's stamp, its first column's (p, m, v) and gradient are loaded together (one round trip after
      // item_of instead of two)
      ColState cs0[U];
      float4 gv0[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        sidx[u] = g0 + (int64_t)u * rm.rpb + rr;
        act[u] = rr < rm.rpb && sidx[u] < nu;
        j[u] = act[u] ? (int64_t)item_of[sidx[u]] : 0;
        const int32_t ls = act[u] ? last_step[j[u]] : t;
        if (act[u] && cc < H4) {
          cs0[u] = col_load(p, m, v, j[u] * H4 + cc);
          gv0[u] = *reinterpret_cast<const float4*>(rows + sidx[u] * H + 4 * cc);
        }
        from[u] = ls_mv(ls);
        pst[u] = ls_p(ls);
      }
      for (int64_t c = cc; c < H4; c += rm.h4s) {
        ColState cs[U];
        float4 gv[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) {
            if (c == cc) {
              cs[u] = cs0[u];
              gv[u] = gv0[u];
            } else {
              cs[u] = col_load(p, m, v, j[u] * H4 + c);
              gv[u] = *reinterpret_cast<const float4*>(rows + sidx[u] * H + 4 * c);
            }
          }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) {
            float4 g = gv[u];
            g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
            col_math_lazy(a, tab, cs[u], from[u], pst[u], t - 1, true, k, g);
          }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) col_store(p, m, v, j[u] * H4 + c, cs[u]);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (act[u] && cc == 0) last_step[j[u]] = t;
    }
  } else if ((int)blockIdx.x < nb_rows + nb_sweep) {
    const int64_t chunk = (N + period - 1) / period;
    const int64_t r0 = (int64_t)((t - 1) % period) * chunk, r1 = min(N, r0 + chunk);
    for (int64_t g0 = r0 + (int64_t)(blockIdx.x - nb_rows) * span; g0 < r1; g0 += (int64_t)nb_sweep * span) {
      int64_t j[U];
      int from[U], pst[U];
      bool act[U];
      // the row's slot, stamp and first column's (p, m, v) are loaded together, before it is known whether the row
      // is this group's (no gradient) and stale: the speculative loads of the skipped rows cost bytes, not a round
      // trip
      ColState cs0[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        j[u] = g0 + (int64_t)u * rm.rpb + rr;
        act[u] = rr < rm.rpb && j[u] < r1;
        from[u] = pst[u] = t;
        if (act[u]) {
          const int sl = slot_of[j[u]];
          const int32_t ls = last_step[j[u]];
          if (cc < H4) cs0[u] = col_load(p, m, v, j[u] * H4 + cc);
          if (sl >= 0 && sl < nu && item_of[sl] == (int32_t)j[u]) {
            act[u] = false;  // has a gradient: first group's row
          } else {
            from[u] = ls_mv(ls);
            pst[u] = ls_p(ls);
          }
        }
        act[u] = act[u] && from[u] < t;
      }
      for (int64_t c = cc; c < H4; c += rm.h4s) {
        ColState cs[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) cs[u] = c == cc ? cs0[u] : col_load(p, m, v, j[u] * H4 + c);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) col_math_lazy(a, tab, cs[u], from[u], pst[u], t - 1, true, k, make_float4(0.f, 0.f, 0.f, 0.f));
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (act[u]) col_store(p, m, v, j[u] * H4 + c, cs[u]);
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (act[u] && cc == 0) last_step[j[u]] = t;
    }
  } else {
    // the small dense parameters: float4 where the segment is 16-B aligned, scalar tail
    float* pd = p + dense_off;
    float* md = m + dense_off;
    float* vd = v + dense_off;
    const int nb_rest = nb_rows + nb_sweep;
    const int64_t gtid = (int64_t)(blockIdx.x - nb_rest) * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)(gridDim.x - nb_rest) * blockDim.x;
    const bool vec = ((((uintptr_t)pd) | ((uintptr_t)md) | ((uintptr_t)vd) | ((uintptr_t)g_dense)) % 16) == 0;
    const int64_t n4 = vec ? n_dense / 4 : 0;
    for (int64_t i = gtid; i < n4; i += stride) {
      float4 pp = reinterpret_cast<float4*>(pd)[i], mm = reinterpret_cast<float4*>(md)[i];
      float4 vv = reinterpret_cast<float4*>(vd)[i];
      const float4 gg = reinterpret_cast<const float4*>(g_dense)[i];
      adam_elem(pp.x, mm.x, vv.x, gg.x * coef, k);
      adam_elem(pp.y, mm.y, vv.y, gg.y * coef, k);
      adam_elem(pp.z, mm.z, vv.z, gg.z * coef, k);
      adam_elem(pp.w, mm.w, vv.w, gg.w * coef, k);
      reinterpret_cast<float4*>(pd)[i] = pp;
      reinterpret_cast<float4*>(md)[i] = mm;
      reinterpret_cast<float4*>(vd)[i] = vv;
    }
    for (int64_t i = 4 * n4 + gtid; i < n_dense; i += stride) {
      float pp = pd[i], mm = md[i], vv = vd[i];
      adam_elem(pp, mm, vv, g_dense[i] * coef, k);
      pd[i] = pp; md[i] = mm; vd[i] = vv;
    }
  }
}

// The recorded step's W1t rows (hvae_adam_lazy_pending): blocks [0, nb_rows) take the pending gradient rows that
// no catch-up has claimed since (k_adam_lazy's row update: missed steps replayed, then step t with coef * g);
// blocks [nb_rows, nb_rows + nb_sweep) take step t's sweep range (k_adam_lazy's sweep: rows without a pending
// update brought through step t; a row the catch-up moved p of to t replays m and v alone). Same float operations
// as the undeferred update, so the rows are bitwise k_adam_lazy's. A second run finds nothing left to do.
__global__ void __launch_bounds__(256) k_adam_pending(AdamArgs a, const float2* __restrict__ tab,
                                                     float* __restrict__ p, float* __restrict__ m,
                                                     float* __restrict__ v, int32_t* __restrict__ last_step,
                                                     const int32_t* __restrict__ pend_slot,
                                                     const int32_t* __restrict__ pend_item,
                                                     const PendHdr* __restrict__ hdr, int64_t N, int64_t H,
                                                     int nb_rows, int nb_sweep, int period, RowMap rm) {
  const int64_t t64 = hdr->t;
  if (t64 <= 0) return;
  const int t = (int)t64;
  const float* __restrict__ rows = hdr->rows;
  const int64_t ld = hdr->ld;
  const float coef = hdr->coef;
  const int nu = hdr->n;
  const AdamK k = adam_consts_tab(a, tab[t]);
  const int64_t H4 = H / 4;
  const int rr = threadIdx.x / rm.h4s, cc = threadIdx.x % rm.h4s;
  if ((int)blockIdx.x < nb_rows) {
    for (int64_t g0 = (int64_t)blockIdx.x * rm.rpb; g0 < nu; g0 += (int64_t)nb_rows * rm.rpb) {
      const int64_t s = g0 + rr;
      bool act = rr < rm.rpb && s < nu;
      const int64_t j = act ? (int64_t)pend_item[s] : 0;
      const int32_t ls = act ? last_step[j] : 0;
      act = act && (ls & kPendBit) && pend_slot[j] == (int32_t)s;
      const int from = ls_mv(ls), pst = ls_p(ls);
      for (int64_t c = cc; c < H4; c += rm.h4s) {
        if (!act) continue;
        ColState cs = col_load(p, m, v, j * H4 + c);
        float4 g = *reinterpret_cast<const float4*>(rows + s * ld + 4 * c);
        g.x *= coef; g.y *= coef; g.z *= coef; g.w *= coef;
        col_math_lazy(a, tab, cs, from, pst, t - 1, true, k, g);
        col_store(p, m, v, j * H4 + c, cs);
      }
      __syncthreads();
      if (act && cc == 0) last_step[j] = t;
    }
  } else if ((int)blockIdx.x < nb_rows + nb_sweep) {
    const int64_t chunk = (N + period - 1) / period;
    const int64_t r0 = (int64_t)((t - 1) % period) * chunk, r1 = min(N, r0 + chunk);
    for (int64_t g0 = r0 + (int64_t)(blockIdx.x - nb_rows) * rm.rpb; g0 < r1; g0 += (int64_t)nb_sweep * rm.rpb) {
      const int64_t j = g0 + rr;
      bool act = rr < rm.rpb && j < r1;
      const int32_t ls = act ? last_step[j] : 0;
      act = act && !(ls & kPendBit) && ls_mv(ls) < t;
      const int from = ls_mv(ls), pst = ls_p(ls);
      for (int64_t c = cc; c < H4; c += rm.h4s) {
        if (!act) continue;
        ColState cs = col_load(p, m, v, j * H4 + c);
        // through step t with g = 0: adam_elem0 (or adam_elem at g = 0 with weight decay) is bitwise k_adam_lazy's
        // adam_elem(g = 0) step; steps p already has move m and v alone
        col_math_lazy(a, tab, cs, from, pst, t, false, k, make_float4(0.f, 0.f, 0.f, 0.f));
        col_store(p, m, v, j * H4 + c, cs);
      }
      __syncthreads();
      if (act && cc == 0) last_step[j] = t;
    }
  }
}


}  // namespace hvae

using namespace hvae;

extern "C" size_t hvae_clip_grad_norm_workspace(int64_t, int64_t, int64_t) {
  return kNormBlocks * sizeof(double);
}

// Blocks of the clip: enough for four 16-B loads in flight per thread over the largest possible input (the dense
// gradient plus the cap's row partials or rows), at most kNormBlocks -- a small batch's clip is one memory round
// trip and a last-block reduction, which fewer partials shorten
static unsigned clip_blocks(const ClipArgs& a, const hvae_rowgrad* rg) {
  int64_t units = a.n / 4;  // float4 of the dense gradient
  if (rg) units += a.rowsq ? rg->cap * kRowSqParts / 2 : rg->cap * a.H / 4;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(units, 256 * 4), kNormBlocks));
}

static int clip_launch(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg, int64_t H, float max_norm,
                       float* norm_out, float* coef_out, int64_t* step, int64_t* step_snap, int64_t* boff,
                       int64_t advance, void* ws, size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(coef_out && n_dense >= 0 && (n_dense == 0 || g_dense), "hvae_clip_grad_norm: bad args");
  HVAE_REQUIRE(!rg || (rg->rows && rg->n_unique && H > 0), "hvae_clip_grad_norm: bad rowgrad");
  if (!ws || ws_bytes < kNormBlocks * sizeof(double))
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae_clip_grad_norm: workspace too small");
  ClipArgs a{};
  a.g = g_dense; a.n = n_dense;
  a.rows = rg ? rg->rows : nullptr; a.n_unique = rg ? rg->n_unique : nullptr; a.H = H;
  a.rowsq = rg ? rg->rowsq : nullptr;
  if (const char* e = ab_getenv("HVAE_ROWSQ")) if (std::atoi(e) == 0) a.rowsq = nullptr;
  a.part = (double*)ws;
  if (!(a.ticket = ticket_slice())) return HVAE_ERR_HIP;
  a.max_norm = max_norm; a.norm_out = norm_out; a.coef_out = coef_out;
  a.step = step; a.step_snap = step_snap; a.boff = boff; a.advance = advance;
  ProbeScope probe("clip", as_stream(stream));
  k_clip_norm<<<clip_blocks(a, rg), 256, 0, as_stream(stream)>>>(a);
  HVAE_LAUNCH_CHECK("k_clip_norm");
  return HVAE_OK;
}

extern "C" int hvae_clip_grad_norm(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg,
                                   int64_t H, float max_norm, float* norm_out, float* coef_out,
                                   void* ws, size_t ws_bytes, void* stream) {
  return clip_launch(g_dense, n_dense, rg, H, max_norm, norm_out, coef_out, nullptr, nullptr, nullptr, 0, ws,
                     ws_bytes, stream);
}

extern "C" int hvae_clip_grad_norm_step(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg,
                                        int64_t H, float max_norm, float* norm_out, float* coef_out,
                                        int64_t* step_dev, int64_t* step_snap, int64_t* boff, int64_t advance,
                                        void* ws, size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(step_dev && step_snap, "hvae_clip_grad_norm_step: null step counters");
  HVAE_REQUIRE(advance == 0 || boff, "hvae_clip_grad_norm_step: advance without boff");
  return clip_launch(g_dense, n_dense, rg, H, max_norm, norm_out, coef_out, step_dev, step_snap, boff, advance,
                     ws, ws_bytes, stream);
}

extern "C" int hvae_clip_grad_norm_step_adam(const float* g_dense, int64_t n_dense, const hvae_rowgrad* rg,
                                             int64_t H, float max_norm, float* norm_out, float* coef_out,
                                             int64_t* step_dev, int64_t* step_snap, int64_t* boff, int64_t advance,
                                             const hvae_adam* cfg, float* tab, void* ws, size_t ws_bytes,
                                             void* stream) {
  HVAE_REQUIRE(step_dev && step_snap && cfg && tab, "hvae_clip_grad_norm_step_adam: null step counters / cfg / tab");
  HVAE_REQUIRE(advance == 0 || boff, "hvae_clip_grad_norm_step_adam: advance without boff");
  HVAE_REQUIRE(coef_out && n_dense >= 0 && (n_dense == 0 || g_dense), "hvae_clip_grad_norm: bad args");
  HVAE_REQUIRE(!rg || (rg->rows && rg->n_unique && H > 0), "hvae_clip_grad_norm: bad rowgrad");
  if (!ws || ws_bytes < kNormBlocks * sizeof(double))
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae_clip_grad_norm: workspace too small");
  ClipArgs a{};
  a.g = g_dense; a.n = n_dense;
  a.rows = rg ? rg->rows : nullptr; a.n_unique = rg ? rg->n_unique : nullptr; a.H = H;
  a.rowsq = rg ? rg->rowsq : nullptr;
  if (const char* e = ab_getenv("HVAE_ROWSQ")) if (std::atoi(e) == 0) a.rowsq = nullptr;
  a.part = (double*)ws;
  if (!(a.ticket = ticket_slice())) return HVAE_ERR_HIP;
  a.max_norm = max_norm; a.norm_out = norm_out; a.coef_out = coef_out;
  a.step = step_dev; a.step_snap = step_snap; a.boff = boff; a.advance = advance;
  a.tab = (float2*)tab; a.lr = cfg->lr; a.b1 = cfg->beta1; a.b2 = cfg->beta2;
  ProbeScope probe("clip", as_stream(stream));
  k_clip_norm<<<clip_blocks(a, rg), 256, 0, as_stream(stream)>>>(a);
  HVAE_LAUNCH_CHECK("k_clip_norm");
  return HVAE_OK;
}

extern "C" int hvae_adam_dense(const hvae_adam* cfg, float* p, float* m, float* v, const float* g,
                               int64_t n, void* stream) {
  HVAE_REQUIRE(cfg && (n == 0 || (p && m && v && g)), "hvae_adam_dense: bad args");
  if (n == 0) return HVAE_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(n, 256), 4096);
  ProbeScope probe("adam_dense", as_stream(stream));
  k_adam_dense<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(to_args(cfg), p, m, v, g, n);
  HVAE_LAUNCH_CHECK("k_adam_dense");
  return HVAE_OK;
}

extern "C" int hvae_adam_rows(const hvae_adam* cfg, float* p, float* m, float* v, const hvae_rowgrad* rg,
                              int64_t N, int64_t H, void* stream) {
  HVAE_REQUIRE(cfg && p && m && v && rg && rg->rows && rg->slot_of && rg->item_of && rg->n_unique,
               "hvae_adam_rows: bad args");
  HVAE_REQUIRE(H % 4 == 0 && ((uintptr_t)p % 16) == 0 && ((uintptr_t)m % 16) == 0 &&
                   ((uintptr_t)v % 16) == 0,
               "hvae_adam_rows: H %% 4 and 16-B alignment required");
  if (N == 0) return HVAE_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(N * H / 4, 256), 8192);
  ProbeScope probe("adam_rows", as_stream(stream));
  k_adam_rows<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(to_args(cfg), p, m, v, rg->rows, rg->slot_of,
                                                             rg->item_of, rg->n_unique, N, H);
  HVAE_LAUNCH_CHECK("k_adam_rows");
  return HVAE_OK;
}

extern "C" int hvae_adam_flat(const hvae_adam* cfg, float* p, float* m, float* v, const hvae_rowgrad* rg,
                              int64_t N, int64_t H, const float* g_dense, int64_t dense_off, int64_t n_dense,
                              void* stream) {
  HVAE_REQUIRE(cfg && p && m && v && rg && rg->rows && rg->slot_of && rg->item_of && rg->n_unique,
               "hvae_adam_flat: bad args");
  HVAE_REQUIRE(H % 4 == 0 && ((uintptr_t)p % 16) == 0 && ((uintptr_t)m % 16) == 0 && ((uintptr_t)v % 16) == 0,
               "hvae_adam_flat: H %% 4 and 16-B alignment required");
  HVAE_REQUIRE(n_dense == 0 || (g_dense && dense_off >= N * H), "hvae_adam_flat: dense segment overlaps W1t");
  const int64_t b_rows = std::max<int64_t>(1, std::min<int64_t>(cdiv(N * H / 4, 256), 8192));
  const int64_t b_dense = std::min<int64_t>(cdiv(n_dense, 256), 2048);
  ProbeScope probe("adam_rows", as_stream(stream));
  k_adam_flat<<<(unsigned)(b_rows + b_dense), 256, 0, as_stream(stream)>>>(
      to_args(cfg), p, m, v, rg->rows, rg->slot_of, rg->item_of, rg->n_unique, N, H, g_dense, dense_off, n_dense,
      (int)b_rows);
  HVAE_LAUNCH_CHECK("k_adam_flat");
  return HVAE_OK;
}

extern "C" int hvae_adam_lazy_catchup(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                                      int32_t* last_step, const hvae_rowgrad* rows, int64_t N, int64_t H,
                                      void* stream) {
  HVAE_REQUIRE(cfg && cfg->step_dev && tab && p && m && v && last_step && H % 4 == 0,
               "hvae_adam_lazy_catchup: bad args");
  HVAE_REQUIRE(!rows || (rows->item_of && rows->n_unique), "hvae_adam_lazy_catchup: bad row list");
  if (N == 0) return HVAE_OK;
  const int64_t nrows = rows ? rows->cap : N;
  const RowMap rm = row_map(H);
  const int uu = adam_unroll();
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(nrows, (int64_t)rm.rpb * uu), 16384));
  ProbeScope probe("adam_catchup", as_stream(stream));
  HVAE_ADAM_U_CALL(uu, (k_adam_catchup<U><<<grid, 256, 0, as_stream(stream)>>>(to_args(cfg), (const float2*)tab, p, m, v,
                                                      last_step, rows ? rows->item_of : nullptr,
                                                      rows ? rows->n_unique : nullptr, N, H, rm)));
  HVAE_LAUNCH_CHECK("k_adam_catchup");
  return HVAE_OK;
}

extern "C" int hvae_adam_lazy_catchup_csr(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                                          int32_t* last_step, const hvae_csr_batch* x, int64_t H, void* stream) {
  HVAE_REQUIRE(cfg && cfg->step_dev && tab && p && m && v && last_step && H % 4 == 0 && x && x->row_ptr &&
                   x->col_idx,
               "hvae_adam_lazy_catchup_csr: bad args");
  if (x->nb == 0) return HVAE_OK;
  // slices per batch row: about kCatchupBlocks blocks in all (1 from that many batch rows up)
  const int S = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(kCatchupBlocks, x->nb), 64));
  const unsigned grid = (unsigned)(std::min<int64_t>(x->nb, 16384) * S);
  ProbeScope probe("adam_catchup", as_stream(stream));
  const int pon = catchup_p_only();
  HVAE_ADAM_U_CALL(adam_unroll(), (k_adam_catchup_csr<U><<<grid, 256, 0, as_stream(stream)>>>(
                                      to_args(cfg), (const float2*)tab, p, m, v, last_step, *x, H, S, pon, nullptr,
                                      nullptr)));
  HVAE_LAUNCH_CHECK("k_adam_catchup_csr");
  return HVAE_OK;
}

extern "C" int hvae_adam_lazy_catchup_csr_pending(const hvae_adam* cfg, const float* tab, float* p, float* m,
                                                  float* v, int32_t* last_step, const hvae_csr_batch* x, int64_t H,
                                                  const hvae_adam_pend* pend, void* stream) {
  HVAE_REQUIRE(cfg && cfg->step_dev && tab && p && m && v && last_step && H % 4 == 0 && x && x->row_ptr &&
                   x->col_idx && pend && pend->slot_of && pend->hdr,
               "hvae_adam_lazy_catchup_csr_pending: bad args");
  if (x->nb == 0) return HVAE_OK;
  const int S = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(kCatchupBlocks, x->nb), 64));
  const unsigned grid = (unsigned)(std::min<int64_t>(x->nb, 16384) * S);
  ProbeScope probe("adam_catchup", as_stream(stream));
  const int pon = catchup_p_only();
  k_adam_catchup_csr<kAdamUnroll><<<grid, 256, 0, as_stream(stream)>>>(
      to_args(cfg), (const float2*)tab, p, m, v, last_step, *x, H, S, pon, pend->slot_of,
      (const PendHdr*)pend->hdr);
  HVAE_LAUNCH_CHECK("k_adam_catchup_csr");
  return HVAE_OK;
}

extern "C" int hvae_adam_lazy_pending(const hvae_adam* cfg, const float* tab, float* p, float* m, float* v,
                                      int32_t* last_step, int64_t N, int64_t H, int64_t max_rows,
                                      const hvae_adam_pend* pend, void* stream) {
  HVAE_REQUIRE(cfg && tab && p && m && v && last_step && pend && pend->slot_of && pend->item_of && pend->hdr &&
                   H % 4 == 0 && N >= 0 && max_rows >= 0,
               "hvae_adam_lazy_pending: bad args");
  HVAE_REQUIRE(((uintptr_t)p % 16) == 0 && ((uintptr_t)m % 16) == 0 && ((uintptr_t)v % 16) == 0,
               "hvae_adam_lazy_pending: 16-B alignment required");
  if (N == 0) return HVAE_OK;
  const RowMap rm = row_map(H);
  const int64_t b_rows = std::max<int64_t>(1, std::min<int64_t>(cdiv(std::min(max_rows, N), (int64_t)rm.rpb), 4096));
  const int period = lazy_sweep_period(N);
  const int64_t b_sweep = std::max<int64_t>(1, std::min<int64_t>(cdiv(cdiv(N, period), (int64_t)rm.rpb), 4096));
  ProbeScope probe("adam_pending", as_stream(stream));
  k_adam_pending<<<(unsigned)(b_rows + b_sweep), 256, 0, as_stream(stream)>>>(
      to_args(cfg), (const float2*)tab, p, m, v, last_step, pend->slot_of, pend->item_of,
      (const PendHdr*)pend->hdr, N, H, (int)b_rows, (int)b_sweep, period, rm);
  HVAE_LAUNCH_CHECK("k_adam_pending");
  return HVAE_OK;
}

static int adam_lazy_launch(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                            int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense,
                            int64_t dense_off, int64_t n_dense, const hvae_adam_pend* pend, void* stream);

extern "C" int hvae_adam_lazy(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                              int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense,
                              int64_t dense_off, int64_t n_dense, void* stream) {
  return adam_lazy_launch(cfg, tab, tab_len, p, m, v, last_step, rg, H, g_dense, dense_off, n_dense, nullptr,
                          stream);
}

extern "C" int hvae_adam_lazy_defer(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                                    int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense,
                                    int64_t dense_off, int64_t n_dense, const hvae_adam_pend* pend, void* stream) {
  HVAE_REQUIRE(pend && pend->slot_of && pend->item_of && pend->hdr, "hvae_adam_lazy_defer: bad pend");
  return adam_lazy_launch(cfg, tab, tab_len, p, m, v, last_step, rg, H, g_dense, dense_off, n_dense, pend, stream);
}

static int adam_lazy_launch(const hvae_adam* cfg, float* tab, int64_t tab_len, float* p, float* m, float* v,
                            int32_t* last_step, const hvae_rowgrad* rg, int64_t H, const float* g_dense,
                            int64_t dense_off, int64_t n_dense, const hvae_adam_pend* pend, void* stream) {
  HVAE_REQUIRE(cfg && cfg->step_dev && tab && p && m && v && last_step && rg && rg->rows && rg->item_of &&
                   rg->n_unique,
               "hvae_adam_lazy: bad args");
  HVAE_REQUIRE(H % 4 == 0 && ((uintptr_t)p % 16) == 0 && ((uintptr_t)m % 16) == 0 && ((uintptr_t)v % 16) == 0,
               "hvae_adam_lazy: H %% 4 and 16-B alignment required");
  HVAE_REQUIRE(n_dense == 0 || (g_dense && dense_off >= rg->n_items * H), "hvae_adam_lazy: dense overlaps W1t");
  HVAE_REQUIRE(tab_len >= 2, "hvae_adam_lazy: step table too short");
  HVAE_REQUIRE(tab_len <= ((int64_t)1 << kStepBits), "hvae_adam_lazy: step table longer than last_step's 2^24 steps");
  const int64_t N = rg->n_items;
  HVAE_REQUIRE(rg->slot_of, "hvae_adam_lazy: rowgrad without slot_of");
  const RowMap rm = row_map(H);
  const int uu = adam_unroll();
  // deferred: the row blocks only record the rows (one thread a row) and the sweep waits for k_adam_pending
  const int64_t b_rows = pend ? std::max<int64_t>(1, std::min<int64_t>(cdiv(rg->cap, 256), 1024))
                              : std::max<int64_t>(1, std::min<int64_t>(cdiv(rg->cap, (int64_t)rm.rpb * uu), 4096));
  const int period = lazy_sweep_period(N);
  const int64_t b_sweep =
      pend ? 0 : std::max<int64_t>(1, std::min<int64_t>(cdiv(cdiv(N, period), (int64_t)rm.rpb * uu), 4096));
  const int64_t b_dense = std::min<int64_t>(cdiv(cdiv(n_dense, 4), 256), 512);
  ProbeScope probe("adam_rows", as_stream(stream));
  HVAE_ADAM_U_CALL(uu, (k_adam_lazy<U><<<(unsigned)(b_rows + b_sweep + b_dense), 256, 0, as_stream(stream)>>>(
      to_args(cfg), (float2*)tab, p, m, v, last_step, rg->rows, rg->slot_of, rg->item_of, rg->n_unique, N, H,
      g_dense, dense_off, n_dense, (int)b_rows, (int)b_sweep, period, rm, pend ? pend->slot_of : nullptr,
      pend ? pend->item_of : nullptr, pend ? (PendHdr*)pend->hdr : nullptr)));
  HVAE_LAUNCH_CHECK("k_adam_lazy");
  return HVAE_OK;
}

extern "C" int hvae_adam_lazy_sweep_period(int64_t N) { return hvae::lazy_sweep_period(N); }
