// hvae_encoder_row.h -- the first encoder layer of one batch row (sparse gather of W1t rows, LayerNorm, GELU,
// Dropout) as one wave's work: k_encoder_sparse_fwd (hvae_encoder.hip) and the row-parallel MLP forward
// (hvae_mlp.hip) run it.
#pragma once

#include <type_traits>

#include "hvae_common.h"

namespace hvae {

constexpr float kLnEps = 1e-5f;  // nn.LayerNorm default (src/ml/model.py:115)

// --------------------------------------------------------------------------
// LayerNorm -> GELU -> Dropout epilogue on one row held as NV float4 chunks
// per lane (chunk c = lane + 64 k covers elements 4c .. 4c+3, valid if 4c < H).
template <int NV>
__device__ __forceinline__ void ln_gelu_drop_row(float4 (&acc)[NV], int lane, int64_t H, int64_t row,
                                                 const float* __restrict__ ln_w,
                                                 const float* __restrict__ ln_b, float p_drop,
                                                 float scale, const float* __restrict__ drop_mult,
                                                 uint64_t seed, int64_t step, uint32_t tag,
                                                 int train, float* __restrict__ h_out,
                                                 float* __restrict__ xhat_out,
                                                 float* __restrict__ rstd_out, float* h_lds = nullptr) {
  const float invH = 1.0f / (float)H;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    if (e < H) s += (acc[k].x + acc[k].y) + (acc[k].z + acc[k].w);
  }
  const float mean = wave_sum(s) * invH;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    if (e < H) {
      acc[k].x -= mean; acc[k].y -= mean; acc[k].z -= mean; acc[k].w -= mean;
      q += (acc[k].x * acc[k].x + acc[k].y * acc[k].y) + (acc[k].z * acc[k].z + acc[k].w * acc[k].w);
    }
  }
  const float var = wave_sum(q) * invH;  // biased variance, as nn.LayerNorm
  const float rstd = 1.0f / sqrtf(var + kLnEps);
  if (rstd_out && lane == 0) rstd_out[row] = rstd;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    if (e >= H) continue;
    float4 xh = make_float4(acc[k].x * rstd, acc[k].y * rstd, acc[k].z * rstd, acc[k].w * rstd);
    if (xhat_out) *reinterpret_cast<float4*>(xhat_out + row * H + e) = xh;
    const float4 w = *reinterpret_cast<const float4*>(ln_w + e);
    const float4 b = *reinterpret_cast<const float4*>(ln_b + e);
    float y[4] = {xh.x * w.x + b.x, xh.y * w.y + b.y, xh.z * w.z + b.z, xh.w * w.w + b.w};
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float g = gelu_f(y[i]);
      const uint64_t idx = (uint64_t)(row * H + e + i);
      o[i] = train ? g * dropout_mult(p_drop, scale, drop_mult, idx, seed, step, tag) : g;
    }
    if (h_out) *reinterpret_cast<float4*>(h_out + row * H + e) = make_float4(o[0], o[1], o[2], o[3]);
    if (h_lds) *reinterpret_cast<float4*>(h_lds + e) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// Sparse first layer + epilogue of batch row b, by one wave: a = x_b W1^T + b1 gathered from the item-major
// W1t in entry order, then ln_gelu_drop_row (h also into h_lds [H] when non-NULL).
// WIDE: 8 W1t rows in flight per step (else 4: fewer registers, for callers that hold more state)
template <int NV, bool WIDE = true>
__device__ __forceinline__ void encoder_sparse_row(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col_idx,
    const float* __restrict__ vals, const int32_t* __restrict__ rows,
    const int64_t* __restrict__ rows_offset, int64_t b,
    const float* __restrict__ w1t, const float* __restrict__ b1, const float* __restrict__ ln_w,
    const float* __restrict__ ln_b, int64_t H, float p_drop, float scale,
    const float* __restrict__ drop_mult, uint64_t seed, int64_t step,
    int train, float* __restrict__ h_out, float* __restrict__ xhat_out,
    float* __restrict__ rstd_out, float* h_lds) {
  const int lane = threadIdx.x & 63;
  const int64_t r = batch_row(rows, rows_offset, b);
  const int64_t beg = row_ptr[r], end = row_ptr[r + 1];

  float4 acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    acc[k] = (e < H) ? *reinterpret_cast<const float4*>(b1 + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // Row entries are fetched 64 at a time (one per lane) and broadcast with
  // v_readlane; four item rows are in flight per step for memory parallelism.
  for (int64_t base = beg; base < end; base += 64) {
    const int64_t n = min((int64_t)64, end - base);
    const int my_j = (lane < n) ? col_idx[base + lane] : 0;
    const float my_x = (lane < n) ? vals[base + lane] : 0.f;
    int t = 0;
    // R item rows in flight per step (8, then 4, then one at a time); the sum runs in entry order either way
    auto rows = [&](auto rc) {
      constexpr int R = decltype(rc)::value;
      int j[R];
      float x[R];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        j[u] = __builtin_amdgcn_readlane(my_j, t + u);
        x[u] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_x), t + u));
      }
      float4 w[NV][R];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int64_t e = 4 * (int64_t)(lane + 64 * k);
#pragma unroll
        for (int u = 0; u < R; ++u)
          w[k][u] = e < H ? *reinterpret_cast<const float4*>(w1t + (int64_t)j[u] * H + e) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        if (4 * (int64_t)(lane + 64 * k) >= H) continue;
#pragma unroll
        for (int u = 0; u < R; ++u) {
          acc[k].x += x[u] * w[k][u].x; acc[k].y += x[u] * w[k][u].y;
          acc[k].z += x[u] * w[k][u].z; acc[k].w += x[u] * w[k][u].w;
        }
      }
    };
    if (WIDE)
      for (; t + 8 <= n; t += 8) rows(std::integral_constant<int, 8>{});
    for (; t + 4 <= n; t += 4) rows(std::integral_constant<int, 4>{});
    for (; t < n; ++t) {
      const int j = __builtin_amdgcn_readlane(my_j, t);
      const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_x), t));
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int64_t e = 4 * (int64_t)(lane + 64 * k);
        if (e >= H) continue;
        const float4 w = *reinterpret_cast<const float4*>(w1t + (int64_t)j * H + e);
        acc[k].x += x * w.x; acc[k].y += x * w.y; acc[k].z += x * w.z; acc[k].w += x * w.w;
      }
    }
  }
  ln_gelu_drop_row<NV>(acc, lane, H, b, ln_w, ln_b, p_drop, scale, drop_mult, seed, step,
                       kTagEncDrop + 0u, train, h_out, xhat_out, rstd_out, h_lds);
}

// The sparse first layer of batch row b split over nsub waves: wave `sub` sums x_e W1t[j_e] over the row's entries
// e = beg + sub, beg + sub + nsub, ... (entry order within the wave, four rows' loads in flight) into acc (no bias).
// The caller adds the waves' partials in sub order and applies ln_gelu_drop_row.
template <int NV>
__device__ __forceinline__ void encoder_row_partial(const int64_t* __restrict__ row_ptr,
                                                    const int32_t* __restrict__ col_idx,
                                                    const float* __restrict__ vals, const int32_t* __restrict__ rows,
                                                    const int64_t* __restrict__ rows_offset, int64_t b,
                                                    const float* __restrict__ w1t, int64_t H, int sub, int nsub,
                                                    float4 (&acc)[NV]) {
  const int lane = threadIdx.x & 63;
  const int64_t r = batch_row(rows, rows_offset, b);
  const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t e0 = beg + sub; e0 < end; e0 += 4 * (int64_t)nsub) {
    int j[4];
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = e0 + (int64_t)u * nsub;
      j[u] = e < end ? col_idx[e] : 0;
      x[u] = e < end ? vals[e] : 0.f;
    }
    float4 wv[4][NV];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int64_t c = 4 * (int64_t)(lane + 64 * k);
        wv[u][k] = (c < H && e0 + (int64_t)u * nsub < end) ? *reinterpret_cast<const float4*>(w1t + (int64_t)j[u] * H + c)
                                                           : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + (int64_t)u * nsub >= end) break;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        acc[k].x += x[u] * wv[u][k].x; acc[k].y += x[u] * wv[u][k].y;
        acc[k].z += x[u] * wv[u][k].z; acc[k].w += x[u] * wv[u][k].w;
      }
    }
  }
}

}  // namespace hvae
