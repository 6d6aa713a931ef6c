// hvae_eval.hip -- batched evaluation scoring and exact ranking (K16).
//
// Reference: RecommendationEvaluator (src/ml/evaluate.py:106-265) scores one
// user at a time in a Python loop (a 1 x N decode per test row, then
// np.argsort). Here a whole batch of test rows is scored at once: the
// 99-negative protocol only needs the 100 candidate scores per row (a gather
// dot against the fp32 E), the full-ranking protocol uses the fp32 score
// matrix and an exact top-K.
#include <algorithm>

#include "hvae_common.h"

namespace hvae {

// One wave per test row, lanes over D, loop over the row's candidates.
__global__ void __launch_bounds__(256) k_score_candidates(const float* __restrict__ U, int64_t ldu,
                                                          const int32_t* __restrict__ user_row,
                                                          const float* __restrict__ E, int64_t D,
                                                          const int32_t* __restrict__ cand, int64_t R,
                                                          int64_t C, float* __restrict__ scores) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* u = U + (int64_t)user_row[r] * ldu;
  for (int64_t c = 0; c < C; ++c) {
    const float* e = E + (int64_t)cand[r * C + c] * D;
    float s = 0.f;
    for (int64_t d = lane; d < D; d += 64) s += u[d] * e[d];
    s = wave_sum(s);
    if (lane == 0) scores[r * C + c] = s;
  }
}

__global__ void k_rank_first(const float* __restrict__ scores, int64_t R, int64_t C, int32_t* __restrict__ rank) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const float s0 = scores[r * C];
  int k = 0;
  for (int64_t c = 1; c < C; ++c) {
    const float s = scores[r * C + c];
    k += (s > s0) || (s == s0);
  }
  rank[r] = k;
}

__global__ void k_mask_seen(float* __restrict__ scores, int64_t ld, const int64_t* __restrict__ row_ptr,
                            const int32_t* __restrict__ col_idx, const int32_t* __restrict__ rows,
                            const int64_t* __restrict__ rows_offset, int64_t R) {
  const int64_t r = blockIdx.x;
  if (r >= R) return;
  const int64_t m = batch_row(rows, rows_offset, r);
  for (int64_t e = row_ptr[m] + threadIdx.x; e < row_ptr[m + 1]; e += blockDim.x)
    scores[r * ld + col_idx[e]] = -INFINITY;
}

// (score desc, index desc) total order: a before b
__device__ __forceinline__ bool before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia > ib);
}

// Exact top-K: K passes, each selecting the best element strictly after the
// previous selection in the total order (no exclusion state needed).
__global__ void __launch_bounds__(256) k_topk(const float* __restrict__ scores, int64_t N, int64_t ld,
                                              int64_t K, int32_t* __restrict__ idx, float* __restrict__ val) {
  __shared__ float rs[4];
  __shared__ int ri[4];
  const int64_t r = blockIdx.x;
  const float* s = scores + r * ld;
  float ls = INFINITY;
  int li = INT_MAX;
  for (int64_t k = 0; k < K; ++k) {
    float bs = -INFINITY;
    int bi = -1;
    for (int64_t i = threadIdx.x; i < N; i += 256) {
      const float v = s[i];
      if (v != v) continue;  // NaN never ranks
      if (before(ls, li, v, (int)i) && (bi < 0 || before(v, (int)i, bs, bi))) { bs = v; bi = (int)i; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float os = __shfl_xor(bs, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (oi >= 0 && (bi < 0 || before(os, oi, bs, bi))) { bs = os; bi = oi; }
    }
    if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = bs; ri[threadIdx.x >> 6] = bi; }
    __syncthreads();
    bs = rs[0]; bi = ri[0];
    for (int w = 1; w < 4; ++w)
      if (ri[w] >= 0 && (bi < 0 || before(rs[w], ri[w], bs, bi))) { bs = rs[w]; bi = ri[w]; }
    __syncthreads();
    if (threadIdx.x == 0) {
      idx[r * K + k] = bi;
      if (val) val[r * K + k] = bs;
    }
    ls = bs;
    li = bi;
    if (bi < 0) { ls = -INFINITY; li = -1; }
  }
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_score_candidates(const float* U, int64_t ldu, const int32_t* user_row, const float* E32,
                                     int64_t D, const int32_t* cand, int64_t R, int64_t C, float* scores,
                                     void* stream) {
  HVAE_REQUIRE(R >= 0 && ldu >= D && D > 0 && C > 0, "hvae_score_candidates: bad args");
  if (R == 0) return HVAE_OK;  // empty outputs may have null data pointers
  HVAE_REQUIRE(U && user_row && E32 && cand && scores, "hvae_score_candidates: null pointer");
  k_score_candidates<<<(unsigned)cdiv(R, 4), 256, 0, as_stream(stream)>>>(U, ldu, user_row, E32, D, cand, R,
                                                                          C, scores);
  HVAE_LAUNCH_CHECK("k_score_candidates");
  return HVAE_OK;
}

extern "C" int hvae_rank_first(const float* scores, int64_t R, int64_t C, int32_t* rank, void* stream) {
  HVAE_REQUIRE(R >= 0 && C > 0, "hvae_rank_first: bad args");
  if (R == 0) return HVAE_OK;
  HVAE_REQUIRE(scores && rank, "hvae_rank_first: null pointer");
  k_rank_first<<<(unsigned)cdiv(R, 256), 256, 0, as_stream(stream)>>>(scores, R, C, rank);
  HVAE_LAUNCH_CHECK("k_rank_first");
  return HVAE_OK;
}

extern "C" int hvae_topk(const float* scores, int64_t R, int64_t N, int64_t ld, const hvae_csr_batch* exclude,
                         int64_t K, int32_t* idx, float* val, void* stream) {
  HVAE_REQUIRE(R >= 0 && ld >= N && K > 0 && K <= N && K <= 1024 && N < INT32_MAX, "hvae_topk: bad args");
  if (R == 0) return HVAE_OK;
  HVAE_REQUIRE(scores && idx, "hvae_topk: null pointer");
  hipStream_t st = as_stream(stream);
  if (exclude) {
    HVAE_REQUIRE(exclude->row_ptr && exclude->col_idx && exclude->nb == R, "hvae_topk: bad exclude");
    // seen items are masked in place (the scores buffer is scratch for the caller)
    k_mask_seen<<<(unsigned)R, 256, 0, st>>>(const_cast<float*>(scores), ld, exclude->row_ptr,
                                            exclude->col_idx, exclude->rows, exclude->rows_offset, R);
    HVAE_LAUNCH_CHECK("k_mask_seen");
  }
  k_topk<<<(unsigned)R, 256, 0, st>>>(scores, N, ld, K, idx, val);
  HVAE_LAUNCH_CHECK("k_topk");
  return HVAE_OK;
}
