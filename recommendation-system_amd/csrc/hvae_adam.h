// hvae_adam.h -- torch.optim.Adam's element update and the exact lazy replay of W1t rows, shared by the optimizer
// launches (hvae_optim.hip) and the row-parallel MLP forward's fused encoder layer (hvae_mlp.hip), so that every
// place that moves a W1t row does it with the same float operations.
#pragma once

#include "hvae_common.h"

namespace hvae {

// torch's per-step Adam scalars for step t, in double as torch computes them (Python floats):
// (step_size = lr / (1 - b1^t), 1 / sqrt(1 - b2^t)), rounded to fp32 where the kernels use them (the element
// update multiplies by the reciprocal of bias_correction2_sqrt instead of dividing by it: adam_elem).
__device__ __forceinline__ float2 adam_step_consts(double lr, double b1, double b2, int64_t t) {
  const double bc1 = 1.0 - pow(b1, (double)t);
  const double bc2 = 1.0 - pow(b2, (double)t);
  return make_float2((float)(lr / bc1), (float)(1.0 / sqrt(bc2)));
}

struct AdamK {
  float lr_over_bc1;  // step_size
  float inv_bc2_sqrt;  // 1 / bias_correction2_sqrt
  float omb1, b2, omb2, eps, wd;
};

// torch.optim.Adam single-tensor arithmetic, element-wise, with the hardware square root and reciprocal
// (v_sqrt_f32, v_rcp_f32: 1 ulp) where torch divides and takes a correctly rounded root: the parameter update
// differs from torch's by a few ulp of the step (compared at STEP_TOL, tests/test_gpu_train.py), and the lazy
// replays run VALU-light enough to stay near the HBM bound (the IEEE division / square-root sequences made
// the exact replays VALU-bound).
// No FMA contraction: every kernel that applies a step (dense, flat, lazy rows, replays) must round
// identically whatever code shape the compiler sees around it, or the lazy update would drift off
// the dense one by an ulp (hipcc contracts a*b+c freely by default).
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamK& k) {
#pragma clang fp contract(off)
  if (k.wd != 0.f) g = g + k.wd * p;
  m = m + k.omb1 * (g - m);                 // exp_avg.lerp_(grad, 1 - beta1)
  v = v * k.b2 + k.omb2 * g * g;            // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = __builtin_amdgcn_sqrtf(v) * k.inv_bc2_sqrt + k.eps;  // (sqrt(v) / bc2_sqrt).add_(eps)
  p = p - k.lr_over_bc1 * (m * __builtin_amdgcn_rcpf(denom));             // param.addcdiv_(m, denom, -step_size)
}

// adam_elem with g = 0 and no weight decay (the lazy replays), bitwise equal to it: m + omb1 (0 - m) is
// m - omb1 m for every m (signed zeros and NaN included: 0 - m is -m but for m = +0, where both forms give +0),
// and v b2 + omb2 0 0 is v b2 because v is never -0 (it starts at +0 and only ever adds g g >= +0)
__device__ __forceinline__ void adam_elem0(float& p, float& m, float& v, const AdamK& k) {
#pragma clang fp contract(off)
  m = m - k.omb1 * m;
  v = v * k.b2;
  const float denom = __builtin_amdgcn_sqrtf(v) * k.inv_bc2_sqrt + k.eps;
  p = p - k.lr_over_bc1 * (m * __builtin_amdgcn_rcpf(denom));
}

// torch.optim.Adam as the reference's optimizer evaluates it on the CPU (src/ml/train.py:63 -> torch/optim/adam.py
// _single_tensor_adam), operation for operation, for the eager drop-in step (hvae_adam_dense: the fused trainer's
// optimizer.step() and ModuleAdam): grad.add(param, alpha = wd) = fma(wd, p, g), exp_avg.lerp_ = fma(1 - b1,
// g - m, m) and addcmul_ = fma((1 - b2) g, g, v b2) -- the contractions torch's vectorised CPU kernels make,
// probed against torch 2.10's CPU Adam -- then denom = sqrt(v) / bias_correction2_sqrt + eps and
// param.addcdiv_(m, denom, -step_size) = p + ((-step_size) m) / denom, with the correctly rounded square root
// and divisions. The only difference left is torch's own CPU sqrt, which is not correctly rounded (AVX-512
// build: 1 ulp off in ~0.7 % of elements), so on the same inputs p, m, v agree bitwise except where it rounds
// differently (tests/test_gpu_api.py::test_adam_dense_matches_torch_cpu).
struct AdamKExact {
  float neg_step_size;  // -(lr / (1 - b1^t)), rounded to fp32 as addcdiv_'s value is
  float bc2_sqrt;       // sqrt(1 - b2^t)
  float omb1, b2, omb2, eps, wd;
};
__device__ __forceinline__ void adam_elem_exact(float& p, float& m, float& v, float g, const AdamKExact& k) {
#pragma clang fp contract(off)
  if (k.wd != 0.f) g = __builtin_fmaf(k.wd, p, g);
  m = __builtin_fmaf(k.omb1, g - m, m);
  v = __builtin_fmaf(k.omb2 * g, g, v * k.b2);
  const float denom = sqrtf(v) / k.bc2_sqrt + k.eps;  // correctly rounded: hipcc's default
  p = p + (k.neg_step_size * m) / denom;              // -fhip-fp32-correctly-rounded-divide-sqrt
}

// the m, v half of adam_elem0 / adam_elem at g = 0 (wd only enters through g, which m and v see as
// g + wd p: with wd != 0 a p-only replay is not possible, and the CSR catch-up does not use it then)
__device__ __forceinline__ void adam_mv0(float& m, float& v, const AdamK& k) {
#pragma clang fp contract(off)
  m = m - k.omb1 * m;
  v = v * k.b2;
}

// last_step[j] of a W1t row: bits 0-23 the steps applied to m and v, bits 24-29 how many steps further p is
// (set by the CSR catch-up, which moves p alone: the forward reads only p, and the update that follows in the
// same step replays m and v itself, so the catch-up stores 4 B per element instead of 12); 0 in bits 24-29
// means p is where m and v are. Steps stay below 2^24 (hvae_adam_lazy's table length).
constexpr int kStepBits = 24;
constexpr int32_t kStepMask = (1 << kStepBits) - 1;
constexpr int kPAheadMax = 63;
__device__ __forceinline__ int ls_mv(int32_t ls) { return ls & kStepMask; }
__device__ __forceinline__ int ls_p(int32_t ls) { return (ls & kStepMask) + ((ls >> kStepBits) & kPAheadMax); }

// Deferred updates (hvae_adam_lazy_defer, ABI 5): bit 30 of last_step[j] marks a row whose step-t update -- its
// gradient row rows[pend_slot[j] * ld], times coef -- has been recorded but not applied yet; the low 30 bits keep
// their meaning (the steps m, v and p had before it). The header of the recorded step lives in device memory.
constexpr int32_t kPendBit = 1 << 30;
struct PendHdr {
  int64_t t;          // the recorded step (0: nothing was ever recorded)
  const float* rows;  // its gradient rows
  int64_t ld;         // their stride (H)
  float coef;         // its clip multiplier
  int32_t n;          // its gradient rows: pend_item[0 : n]
};
static_assert(sizeof(PendHdr) == 32, "hvae_adam_pend.hdr is 32 bytes");

struct AdamArgs {
  double lr, b1, b2, eps, wd;
  const int64_t* step_dev;
  const float* coef_dev;
};

__device__ __forceinline__ AdamKExact adam_consts_exact(const AdamArgs& a) {
  const int64_t t = load_step(a.step_dev) + 1;
  const double bc1 = 1.0 - pow(a.b1, (double)t);
  const double bc2 = 1.0 - pow(a.b2, (double)t);
  AdamKExact k;
  k.neg_step_size = (float)(-(a.lr / bc1));
  k.bc2_sqrt = (float)sqrt(bc2);
  k.omb1 = (float)(1.0 - a.b1);
  k.b2 = (float)a.b2;
  k.omb2 = (float)(1.0 - a.b2);
  k.eps = (float)a.eps;
  k.wd = (float)a.wd;
  return k;
}

__device__ __forceinline__ AdamK adam_consts(const AdamArgs& a) {
  const int64_t t = load_step(a.step_dev) + 1;
  const float2 c = adam_step_consts(a.lr, a.b1, a.b2, t);
  AdamK k;
  k.lr_over_bc1 = c.x;
  k.inv_bc2_sqrt = c.y;
  k.omb1 = (float)(1.0 - a.b1);
  k.b2 = (float)a.b2;
  k.omb2 = (float)(1.0 - a.b2);
  k.eps = (float)a.eps;
  k.wd = (float)a.wd;
  return k;
}


// ---- exact lazy Adam for W1t -------------------------------------------------
// torch's Adam moves every row each step, gradient or not: with g = 0 a row's
// (p, m, v) evolve by a fixed per-step map that depends only on the step's bias
// corrections. Rows outside the batch are therefore left as they are and the
// missed steps are replayed -- the identical float operations in the identical
// order, so the result is bitwise the eager one -- when the row is next read:
// before the forward of a batch that contains it (catch-up of the batch rows),
// in the update (rows merged from other ranks), and at an epoch end / state
// read (flush of all rows). last_step[j] = steps already applied to row j;
// tab[t] = (lr / bc1_t, 1 / sqrt(bc2_t)) of step t, written by the step's update.
__device__ __forceinline__ AdamK adam_consts_tab(const AdamArgs& a, float2 c) {
  AdamK k;
  k.lr_over_bc1 = c.x;
  k.inv_bc2_sqrt = c.y;
  k.omb1 = (float)(1.0 - a.b1);
  k.b2 = (float)a.b2;
  k.omb2 = (float)(1.0 - a.b2);
  k.eps = (float)a.eps;
  k.wd = (float)a.wd;
  return k;
}

// Column-parallel row updates: a block covers rpb rows x h4s float4 columns (thread t -> row t / h4s,
// column t % h4s, columns past h4s looped), so a row's replay work is spread over H/4 threads instead
// of one wave and the kernel fills the machine. The threads of a row read last_step[j] at the start of
// a group and one of them advances it after a barrier, so no thread sees a half-updated row.
struct RowMap {
  int rpb, h4s;
};
static inline RowMap row_map(int64_t H) {
  const int h4 = (int)(H / 4);
  RowMap r;
  r.h4s = h4 < 256 ? h4 : 256;
  r.rpb = 256 / r.h4s;
  return r;
}

// float4 column i of a row: replay steps (from, to] with g = 0 (constants from the step table,
// loaded kTabAhead at a time), then, if `step`, one more step with constants kx and gradient gx. Split into load /
// math / store so that the row loops below can keep U row groups' loads in flight together.
struct ColState {
  float4 p, m, v;
};
__device__ __forceinline__ ColState col_load(const float* p, const float* m, const float* v, int64_t i) {
  return ColState{reinterpret_cast<const float4*>(p)[i], reinterpret_cast<const float4*>(m)[i],
                  reinterpret_cast<const float4*>(v)[i]};
}
__device__ __forceinline__ void col_store(float* p, float* m, float* v, int64_t i, const ColState& c) {
  reinterpret_cast<float4*>(p)[i] = c.p;
  reinterpret_cast<float4*>(m)[i] = c.m;
  reinterpret_cast<float4*>(v)[i] = c.v;
}
// m, v at step `from`, p at step `pstep` >= from (the CSR catch-up moves p ahead alone, below): steps from + 1 ..
// pstep move m and v only, the rest all three -- the same float operations on m and v either way
constexpr int kTabAhead = 4;  // step-table entries loaded ahead per replay round
__device__ __forceinline__ void col_math_lazy(const AdamArgs& a, const float2* __restrict__ tab, ColState& cs, int from,
                                              int pstep, int to, bool step, const AdamK& kx, float4 gx) {
  float4 &pp = cs.p, &mm = cs.m, &vv = cs.v;
  for (int s0 = from + 1; s0 <= to; s0 += kTabAhead) {
    float2 c[kTabAhead];
#pragma unroll
    for (int u = 0; u < kTabAhead; ++u) c[u] = (s0 + u <= to) ? tab[s0 + u] : make_float2(0.f, 1.f);
#pragma unroll
    for (int u = 0; u < kTabAhead; ++u) {
      if (s0 + u > to) break;
      const AdamK k = adam_consts_tab(a, c[u]);
      if (s0 + u <= pstep) {
        adam_mv0(mm.x, vv.x, k);
        adam_mv0(mm.y, vv.y, k);
        adam_mv0(mm.z, vv.z, k);
        adam_mv0(mm.w, vv.w, k);
      } else if (k.wd == 0.f) {
        adam_elem0(pp.x, mm.x, vv.x, k);
        adam_elem0(pp.y, mm.y, vv.y, k);
        adam_elem0(pp.z, mm.z, vv.z, k);
        adam_elem0(pp.w, mm.w, vv.w, k);
      } else {
        adam_elem(pp.x, mm.x, vv.x, 0.f, k);
        adam_elem(pp.y, mm.y, vv.y, 0.f, k);
        adam_elem(pp.z, mm.z, vv.z, 0.f, k);
        adam_elem(pp.w, mm.w, vv.w, 0.f, k);
      }
    }
  }
  if (step) {
    adam_elem(pp.x, mm.x, vv.x, gx.x, kx);
    adam_elem(pp.y, mm.y, vv.y, gx.y, kx);
    adam_elem(pp.z, mm.z, vv.z, gx.z, kx);
    adam_elem(pp.w, mm.w, vv.w, gx.w, kx);
  }
}
__device__ __forceinline__ void col_math(const AdamArgs& a, const float2* __restrict__ tab, ColState& cs, int from,
                                         int to, bool step, const AdamK& kx, float4 gx) {
  col_math_lazy(a, tab, cs, from, from, to, step, kx, gx);
}
__device__ __forceinline__ void col_update(const AdamArgs& a, const float2* __restrict__ tab, float* __restrict__ p,
                                           float* __restrict__ m, float* __restrict__ v, int64_t i, int from, int to,
                                           bool step, const AdamK& kx, float4 gx) {
  ColState c = col_load(p, m, v, i);
  col_math(a, tab, c, from, to, step, kx, gx);
  col_store(p, m, v, i, c);
}

static inline AdamArgs to_args(const hvae_adam* c) {
  AdamArgs a;
  a.lr = c->lr; a.b1 = c->beta1; a.b2 = c->beta2; a.eps = c->eps; a.wd = c->weight_decay;
  a.step_dev = c->step_dev;
  a.coef_dev = c->coef_dev;
  return a;
}

}  // namespace hvae
