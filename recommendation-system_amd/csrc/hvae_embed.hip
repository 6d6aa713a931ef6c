// hvae_embed.hip -- the pieces the fused step adds for trainable item embeddings (HybridVAE(freeze_embeddings=False),
// reference src/ml/model.py:72-75: E is an nn.Parameter, so loss.backward() gives it the dense gradient
//   dE_i = (1/B) sum_b (n_b softmax(u_b E^T)_i - x_bi) u_b,     n_b = sum_i x_bi        (model.py:198, 281)
// and torch.optim.Adam updates every row of it each step). The executor computes the dense term in item chunks:
// S = U E_c^T (hvae_gemm_f32), S <- (n_b / B) exp(S - lse_b) (hvae_softmax_weights), dE_c = S^T U (hvae_gemm_f32);
// the sparse term reuses the batch's W1 row-gradient plan (the same item segments): hvae_w1_rowgrad_apply with U
// in place of da gives sum_b x_bi u_b per item slot, and hvae_rowgrad_scatter_rows adds -(1/B) of each slot's row
// into dE. Every sum runs in a fixed order.
#include <algorithm>

#include "hvae_common.h"

namespace hvae {

// n_b = sum of the stored values of batch row b, one wave per row (a butterfly: a fixed order)
__global__ void __launch_bounds__(256) k_csr_row_sums(const int64_t* __restrict__ row_ptr,
                                                      const float* __restrict__ vals,
                                                      const int32_t* __restrict__ rows,
                                                      const int64_t* __restrict__ rows_offset, int64_t nb,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t r = batch_row(rows, rows_offset, b);
  float s = 0.f;
  for (int64_t e = row_ptr[r] + lane; e < row_ptr[r + 1]; e += 64) s += vals[e];
  s = wave_sum(s);
  if (lane == 0) out[b] = s;
}

// S[b][c] = alpha * w[b] * exp(S[b][c] - lse[b]) for b < nb, c < ncol (in place)
__global__ void __launch_bounds__(256) k_softmax_weights(float* __restrict__ S, int64_t ld, int64_t nb, int64_t ncol,
                                                         const float* __restrict__ lse, const float* __restrict__ w,
                                                         float alpha) {
  const int64_t total = nb * ncol;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / ncol, c = i % ncol;
    float* p = S + b * ld + c;
    *p = alpha * w[b] * expf(*p - lse[b]);
  }
}

// dst[item_of[s]][:] += alpha * rows[s][:] for the plan's slots s < n_unique (each item once: no two slots share
// an item, so the adds do not race)
__global__ void __launch_bounds__(256) k_rowgrad_scatter_rows(const int32_t* __restrict__ n_unique,
                                                              const int32_t* __restrict__ item_of,
                                                              const float* __restrict__ rows, int64_t width,
                                                              float alpha, float* __restrict__ dst, int64_t ldd) {
  const int64_t w4 = width / 4;
  const int64_t total = (int64_t)(*n_unique) * w4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i / w4, c = i % w4;
    const float4 v = reinterpret_cast<const float4*>(rows + s * width)[c];
    float4* d = reinterpret_cast<float4*>(dst + (int64_t)item_of[s] * ldd) + c;
    float4 o = *d;
    o.x += alpha * v.x; o.y += alpha * v.y; o.z += alpha * v.z; o.w += alpha * v.w;
    *d = o;
  }
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_csr_row_sums(const hvae_csr_batch* x, float* out, void* stream) {
  HVAE_REQUIRE(x && x->row_ptr && x->vals && out && x->nb >= 0, "hvae_csr_row_sums: bad args");
  if (x->nb == 0) return HVAE_OK;
  k_csr_row_sums<<<(unsigned)cdiv(x->nb, 4), 256, 0, as_stream(stream)>>>(x->row_ptr, x->vals, x->rows,
                                                                            x->rows_offset, x->nb, out);
  HVAE_LAUNCH_CHECK("k_csr_row_sums");
  return HVAE_OK;
}

extern "C" int hvae_softmax_weights(float* S, int64_t ld, int64_t nb, int64_t ncol, const float* lse, const float* w,
                                    float alpha, void* stream) {
  HVAE_REQUIRE(S && lse && w && nb >= 0 && ncol >= 0 && ld >= ncol, "hvae_softmax_weights: bad args");
  if (nb == 0 || ncol == 0) return HVAE_OK;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(nb * ncol, 256), 8192));
  k_softmax_weights<<<grid, 256, 0, as_stream(stream)>>>(S, ld, nb, ncol, lse, w, alpha);
  HVAE_LAUNCH_CHECK("k_softmax_weights");
  return HVAE_OK;
}

extern "C" int hvae_rowgrad_scatter_rows(const hvae_rowgrad* rg, int64_t width, float alpha, float* dst, int64_t ldd,
                                         void* stream) {
  HVAE_REQUIRE(rg && rg->n_unique && rg->item_of && rg->rows && dst && width > 0 && width % 4 == 0 && ldd >= width &&
                   ldd % 4 == 0 && ((uintptr_t)dst) % 16 == 0,
               "hvae_rowgrad_scatter_rows: bad args (width, ldd multiples of 4; dst 16-B aligned)");
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(rg->cap * (width / 4), 256), 8192));
  k_rowgrad_scatter_rows<<<grid, 256, 0, as_stream(stream)>>>(rg->n_unique, rg->item_of, rg->rows, width, alpha, dst,
                                                              ldd);
  HVAE_LAUNCH_CHECK("k_rowgrad_scatter_rows");
  return HVAE_OK;
}
