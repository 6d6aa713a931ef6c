// hvae_latent.hip -- reparameterisation + KL (K5, K9), the loss reduction
// (K8 final, K15) and the materialised-score multinomial loss of the module
// API path.
//
// Reference: src/ml/model.py:157-179 (reparameterize), 259-292
// (vae_loss_function), src/ml/train.py:94-96 (per-batch .item() sums).
#include <algorithm>

#include "hvae_common.h"

namespace hvae {

// 4 rows per 256-thread block, one wave per row, lanes over the latent dim.
__global__ void __launch_bounds__(256) k_reparam_kl_fwd(const float* __restrict__ mu,
                                                        const float* __restrict__ lv, int64_t ld,
                                                        int64_t nb, int64_t L, int train,
                                                        const float* __restrict__ eps_in,
                                                        uint64_t seed, const int64_t* __restrict__ step_dev,
                                                        float* __restrict__ z, float* __restrict__ eps_out,
                                                        float* __restrict__ kl_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t step = load_step(step_dev);
  float kl = 0.f;
  for (int64_t l = lane; l < L; l += 64) {
    const float m = mu[b * ld + l], v = lv[b * ld + l];
    const float ev = expf(v);
    kl += ((1.f + v) - m * m) - ev;
    if (train) {
      const float e = eps_in ? eps_in[b * L + l] : normal_f(seed, step, kTagEps, (uint64_t)(b * L + l));
      if (eps_out) eps_out[b * L + l] = e;
      z[b * L + l] = m + e * expf(0.5f * v);
    } else {
      z[b * L + l] = m;
    }
  }
  kl = wave_sum(kl);
  if (lane == 0) kl_rows[b] = -0.5f * kl;
}

__global__ void k_reparam_kl_bwd(const float* __restrict__ dz, const float* __restrict__ mu,
                                 const float* __restrict__ lv, int64_t ld,
                                 const float* __restrict__ eps, int64_t nb, int64_t L,
                                 float kl_scale_h, const float* __restrict__ kl_scale_dev, int train,
                                 float* __restrict__ dmu, float* __restrict__ dlv, int64_t ldo) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb * L) return;
  const float kl_scale = kl_scale_dev ? *kl_scale_dev : kl_scale_h;
  const int64_t b = i / L, l = i % L;
  const float m = mu[b * ld + l], v = lv[b * ld + l];
  const float g = dz ? dz[i] : 0.f;
  dmu[b * ldo + l] = g + kl_scale * m;
  const float gz = (train && dz) ? g * eps[i] * 0.5f * expf(0.5f * v) : 0.f;
  dlv[b * ldo + l] = gz + kl_scale * 0.5f * (expf(v) - 1.f);
}

__global__ void __launch_bounds__(256) k_loss_finalize(const float* __restrict__ recon_rows,
                                                       const float* __restrict__ kl_rows, int64_t nb,
                                                       float beta, float* __restrict__ out3,
                                                       double* __restrict__ accum3) {
  loss_block_reduce(recon_rows, false, kl_rows, nb, beta, out3, accum3);
}

// Row-wise multinomial NLL over materialised scores (block per row).
__global__ void __launch_bounds__(256) k_nll_rows_fwd(const float* __restrict__ S, int64_t lds,
                                                      const float* __restrict__ X, int64_t ldx,
                                                      int64_t N, float* __restrict__ lse,
                                                      float* __restrict__ recon_rows) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const float* s = S + b * lds;
  const float* x = X + b * ldx;
  float mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < N; i += 256) mx = fmaxf(mx, s[i]);
  mx = wave_max(mx);
  __shared__ float redm[4];
  if ((threadIdx.x & 63) == 0) redm[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
  float se = 0.f, n = 0.f, dot = 0.f;
  for (int64_t i = threadIdx.x; i < N; i += 256) {
    const float v = s[i], xv = x[i];
    se += expf(v - mx);
    n += xv;
    dot += xv * v;
  }
  se = block_sum<256>(se, red);
  n = block_sum<256>(n, red);
  dot = block_sum<256>(dot, red);
  if (threadIdx.x == 0) {
    const float l = mx + logf(se);
    lse[b] = l;
    recon_rows[b] = n * l - dot;
  }
}

__global__ void __launch_bounds__(256) k_nll_rows_bwd(const float* __restrict__ S, int64_t lds,
                                                      const float* __restrict__ X, int64_t ldx,
                                                      const float* __restrict__ lse, int64_t N,
                                                      float scale, float* __restrict__ dS,
                                                      int64_t ldd) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  const float* x = X + b * ldx;
  float n = 0.f;
  for (int64_t i = threadIdx.x; i < N; i += 256) n += x[i];
  n = block_sum<256>(n, red);
  const float l = lse[b];
  for (int64_t i = threadIdx.x; i < N; i += 256)
    dS[b * ldd + i] = scale * (n * expf(S[b * lds + i] - l) - x[i]);
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_reparam_kl_fwd(const float* mu, const float* logvar, int64_t ld, int64_t nb,
                                   int64_t L, int train, const float* eps_in, uint64_t seed,
                                   const int64_t* step_dev, float* z, float* eps_out,
                                   float* kl_rows, void* stream) {
  HVAE_REQUIRE(mu && logvar && z && kl_rows && ld >= L && L > 0, "hvae_reparam_kl_fwd: bad args");
  if (nb == 0) return HVAE_OK;
  k_reparam_kl_fwd<<<(unsigned)cdiv(nb, 4), 256, 0, as_stream(stream)>>>(
      mu, logvar, ld, nb, L, train, eps_in, seed, step_dev, z, eps_out, kl_rows);
  HVAE_LAUNCH_CHECK("k_reparam_kl_fwd");
  return HVAE_OK;
}

extern "C" int hvae_reparam_kl_bwd(const float* dz, const float* mu, const float* logvar, int64_t ld,
                                   const float* eps, int64_t nb, int64_t L, float kl_scale,
                                   const float* kl_scale_dev, int train, float* dmu, float* dlogvar,
                                   int64_t ld_out, void* stream) {
  HVAE_REQUIRE(mu && logvar && dmu && dlogvar && ld >= L && ld_out >= L, "hvae_reparam_kl_bwd: bad args");
  HVAE_REQUIRE(!(train && dz) || eps, "hvae_reparam_kl_bwd: train backward needs eps");
  if (nb == 0) return HVAE_OK;
  k_reparam_kl_bwd<<<(unsigned)cdiv(nb * L, 256), 256, 0, as_stream(stream)>>>(
      dz, mu, logvar, ld, eps, nb, L, kl_scale, kl_scale_dev, train, dmu, dlogvar, ld_out);
  HVAE_LAUNCH_CHECK("k_reparam_kl_bwd");
  return HVAE_OK;
}

// AnnealedVAE.get_current_beta + step_annealing (src/ml/model.py:312-327) for one train step, in double as
// the reference's Python floats; contraction off so that beta_min + progress * span rounds as Python does
__global__ void k_anneal_beta(int64_t* __restrict__ anneal_step, double beta_min, double beta_max,
                              int64_t anneal_steps, int64_t nb, float* __restrict__ out2) {
#pragma clang fp contract(off)
  if (threadIdx.x != 0) return;
  const int64_t s = *anneal_step;
  const double beta = s >= anneal_steps ? beta_max
                                        : beta_min + ((double)s / (double)anneal_steps) * (beta_max - beta_min);
  out2[0] = (float)beta;
  out2[1] = (float)(beta / (double)nb);
  *anneal_step = s + 1;
}

extern "C" int hvae_anneal_beta(int64_t* anneal_step, double beta_min, double beta_max, int64_t anneal_steps,
                                int64_t nb, float* out2, void* stream) {
  HVAE_REQUIRE(anneal_step && out2 && nb > 0 && anneal_steps >= 0, "hvae_anneal_beta: bad args");
  k_anneal_beta<<<1, 64, 0, as_stream(stream)>>>(anneal_step, beta_min, beta_max, anneal_steps, nb, out2);
  HVAE_LAUNCH_CHECK("k_anneal_beta");
  return HVAE_OK;
}

extern "C" int hvae_loss_finalize(const float* recon_rows, const float* kl_rows, int64_t nb,
                                  float beta, float* out3, double* accum3, void* stream) {
  HVAE_REQUIRE(recon_rows && kl_rows && out3 && nb > 0, "hvae_loss_finalize: bad args");
  k_loss_finalize<<<1, 256, 0, as_stream(stream)>>>(recon_rows, kl_rows, nb, beta, out3, accum3);
  HVAE_LAUNCH_CHECK("k_loss_finalize");
  return HVAE_OK;
}

extern "C" int hvae_nll_rows_fwd(const float* S, int64_t lds, const float* X, int64_t ldx, int64_t nb,
                                 int64_t N, float* lse, float* recon_rows, void* stream) {
  HVAE_REQUIRE(S && X && lse && recon_rows && lds >= N && ldx >= N && N > 0, "hvae_nll_rows_fwd: bad args");
  if (nb == 0) return HVAE_OK;
  k_nll_rows_fwd<<<(unsigned)nb, 256, 0, as_stream(stream)>>>(S, lds, X, ldx, N, lse, recon_rows);
  HVAE_LAUNCH_CHECK("k_nll_rows_fwd");
  return HVAE_OK;
}

extern "C" int hvae_nll_rows_bwd(const float* S, int64_t lds, const float* X, int64_t ldx,
                                 const float* lse, int64_t nb, int64_t N, float scale, float* dS,
                                 int64_t ldd, void* stream) {
  HVAE_REQUIRE(S && X && lse && dS && lds >= N && ldx >= N && ldd >= N, "hvae_nll_rows_bwd: bad args");
  if (nb == 0) return HVAE_OK;
  k_nll_rows_bwd<<<(unsigned)nb, 256, 0, as_stream(stream)>>>(S, lds, X, ldx, lse, N, scale, dS, ldd);
  HVAE_LAUNCH_CHECK("k_nll_rows_bwd");
  return HVAE_OK;
}
