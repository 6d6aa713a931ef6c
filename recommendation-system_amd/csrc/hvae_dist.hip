// hvae_dist.hip -- the data-parallel step's packet (no reference counterpart: the reference trainer is
// single-device).
//
// A rank does not ship its first-layer weight gradient rows (one H-float row per distinct item of its batch,
// ~160 MB per rank per step at Syn-10M) but what they are made of: its batch's CSR rows and the gradient of
// the first hidden layer's pre-activation, da [B, H] (8.4 MB at B = 4096, H = 512). Every rank then rebuilds
// the row gradient of the union batch with the same deterministic kernels (hvae_w1_rowgrad), in rank-major
// batch order -- exactly the order one rank would use for the union batch -- so the replicas stay
// bit-identical and the step equals a single-GPU step over W x B users up to the order of the dense
// reductions.
//
// hvae_csr_batch_pack compacts the batch's rows (read in place through x->rows / x->rows_offset from the
// resident CSR) into [row_ptr (int32, from 0) | col_idx | scale * vals]; the union of W packets gathered side
// by side is a CSR batch of W x B rows whose row r * (B + 1) + j pointers are row_ptr_r[j] + r * stride.
#include "hvae_common.h"

namespace hvae {

constexpr int kPackThreads = 1024;
constexpr int kPackMaxRows = 1 << 20;

// row_ptr_out[0..nb] = exclusive prefix sums of the batch's row lengths (one block)
// (clamped to cap, with *overflow = 1, when the batch holds more than cap entries: the packet stays a valid CSR
// of the entries it kept, and the host raises on the flag)
__global__ void __launch_bounds__(kPackThreads) k_pack_rowptr(hvae_csr_batch x, int32_t* __restrict__ row_ptr_out,
                                                              int64_t cap, int32_t* __restrict__ overflow) {
  __shared__ int32_t wsum[kPackThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t per = (x.nb + kPackThreads - 1) / kPackThreads;
  const int64_t r0 = (int64_t)tid * per, r1 = min(x.nb, r0 + per);
  auto row_len = [&](int64_t b) {
    const int64_t r = batch_row(x.rows, x.rows_offset, b);
    return (int32_t)(x.row_ptr[r + 1] - x.row_ptr[r]);
  };
  int32_t mine = 0;
  for (int64_t b = r0; b < r1; ++b) mine += row_len(b);
  // exclusive scan of the per-thread sums: within the wave, then over the 16 waves
  int32_t incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int32_t base = 0;
  for (int j = 0; j < w; ++j) base += wsum[j];
  int32_t run = base + incl - mine;
  for (int64_t b = r0; b < r1; ++b) {  // second pass over the thread's rows (L1/L2-warm)
    row_ptr_out[b] = (int32_t)min((int64_t)run, cap);
    run += row_len(b);
  }
  if (tid == kPackThreads - 1) {
    int32_t tot = 0;
    for (int j = 0; j < kPackThreads / 64; ++j) tot += wsum[j];
    row_ptr_out[x.nb] = (int32_t)min((int64_t)tot, cap);
    if (tot > cap && overflow) *overflow = 1;
  }
}

// the entries: one wave per batch row, lanes over the row's entries (coalesced), up to the row's clamped end
__global__ void __launch_bounds__(256) k_pack_entries(hvae_csr_batch x, const int32_t* __restrict__ row_ptr_out,
                                                      float scale, int32_t* __restrict__ col_out,
                                                      float* __restrict__ vals_out, int64_t cap) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= x.nb) return;
  const int64_t r = batch_row(x.rows, x.rows_offset, b);
  const int64_t src = x.row_ptr[r];
  const int32_t dst = row_ptr_out[b], len = row_ptr_out[b + 1] - dst;
  for (int32_t i = lane; i < len; i += 64) {
    const int64_t d = (int64_t)dst + i;
    if (d < cap) {
      col_out[d] = x.col_idx[src + i];
      vals_out[d] = scale * x.vals[src + i];
    }
  }
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_csr_batch_pack(const hvae_csr_batch* x, float scale, int32_t* row_ptr_out, int32_t* col_out,
                                   float* vals_out, int64_t cap, int32_t* overflow, void* stream) {
  HVAE_REQUIRE(x && x->row_ptr && x->col_idx && x->vals && row_ptr_out && cap >= 0 && (cap == 0 || (col_out && vals_out)),
               "hvae_csr_batch_pack: bad args");
  HVAE_REQUIRE(x->nb >= 0 && x->nb <= kPackMaxRows,
               "hvae_csr_batch_pack: nb = %lld over %d", (long long)x->nb, kPackMaxRows);
  hipStream_t st = as_stream(stream);
  k_pack_rowptr<<<1, kPackThreads, 0, st>>>(*x, row_ptr_out, cap, overflow);
  HVAE_LAUNCH_CHECK("k_pack_rowptr");
  if (x->nb > 0) {
    k_pack_entries<<<(unsigned)cdiv(x->nb, 4), 256, 0, st>>>(*x, row_ptr_out, scale, col_out, vals_out, cap);
    HVAE_LAUNCH_CHECK("k_pack_entries");
  }
  return HVAE_OK;
}
