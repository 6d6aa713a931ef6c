// hvae_encoder.hip -- encoder kernels (K1-K3, K11 partial, K12 of SURVEY §2.1).
//
//   * sparse first layer: a = x W1^T + b1 gathered row-by-row from the
//     item-major W1t [N, H] (one wave per user row, 2 KB item rows at H=512
//     read as float4 per lane), fused with LayerNorm -> GELU -> Dropout;
//   * the same epilogue for dense hidden layers, and its backward;
//   * the row-sparse first-layer weight gradient, built by a deterministic
//     counting sort over the batch nonzeros (no float atomics);
//   * dense [B, N] -> CSR for the module-API path.
//
// Reference: src/ml/model.py:103-127 (_build_encoder), 138-155 (encode).
#include <algorithm>
#include <cstdlib>

#include <type_traits>

#include "hvae_common.h"
#include "hvae_rgplan.h"
#include "hvae_encoder_row.h"

namespace hvae {


// Sparse first layer + epilogue. One wave per batch row (hvae_encoder_row.h), 4 waves per block.
template <int NV>
__global__ void __launch_bounds__(256) k_encoder_sparse_fwd(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ col_idx,
    const float* __restrict__ vals, const int32_t* __restrict__ rows,
    const int64_t* __restrict__ rows_offset, int64_t nb,
    const float* __restrict__ w1t, const float* __restrict__ b1, const float* __restrict__ ln_w,
    const float* __restrict__ ln_b, int64_t H, float p_drop, float scale,
    const float* __restrict__ drop_mult, uint64_t seed, const int64_t* __restrict__ step_dev,
    int train, float* __restrict__ h_out, float* __restrict__ xhat_out,
    float* __restrict__ rstd_out) {
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  encoder_sparse_row<NV>(row_ptr, col_idx, vals, rows, rows_offset, b, w1t, b1, ln_w, ln_b, H, p_drop, scale,
                         drop_mult, seed, load_step(step_dev), train, h_out, xhat_out, rstd_out, nullptr);
}

template <int NV>
__global__ void __launch_bounds__(256) k_ln_gelu_drop_fwd(
    const float* __restrict__ a, const float* __restrict__ ln_w, const float* __restrict__ ln_b,
    int64_t nb, int64_t H, float p_drop, float scale, const float* __restrict__ drop_mult,
    uint64_t seed, const int64_t* __restrict__ step_dev, uint32_t tag, int train,
    float* __restrict__ h_out, float* __restrict__ xhat_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t step = load_step(step_dev);
  float4 acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    acc[k] = (e < H) ? *reinterpret_cast<const float4*>(a + b * H + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  ln_gelu_drop_row<NV>(acc, lane, H, b, ln_w, ln_b, p_drop, scale, drop_mult, seed, step, tag,
                       train, h_out, xhat_out, rstd_out);
}

// Backward of Dropout(GELU(LN(a))). 4 waves x rpw rows per block (rpw = 1 for
// the small train batches, so that the grid is wide; 4 for large ones, so that
// the partial buffer stays short); per-block column partials of
// d(ln_w) = sum dy * xhat, d(ln_b) = sum dy and d(bias) = sum da.
static inline int ln_bwd_rows_per_wave(int64_t nb) { return nb <= 2048 ? 1 : 4; }

template <int NV>
__global__ void __launch_bounds__(256) k_ln_gelu_drop_bwd(
    const float* __restrict__ dh, const float* __restrict__ xhat, const float* __restrict__ rstd,
    const float* __restrict__ ln_w, const float* __restrict__ ln_b, int64_t nb, int64_t H,
    float p_drop, float scale, const float* __restrict__ drop_mult, uint64_t seed,
    const int64_t* __restrict__ step_dev, uint32_t tag, int train, int rpw, float* __restrict__ da,
    float* __restrict__ part /* [nblocks][3][H] */, unsigned* __restrict__ ticket, float* __restrict__ d_ln_w,
    float* __restrict__ d_ln_b, float* __restrict__ d_bias) {
  extern __shared__ __attribute__((aligned(16))) float lds_part[];  // [4 waves][3][H]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t step = load_step(step_dev);
  const float invH = 1.0f / (float)H;
  float4 pg[NV], pb[NV], pa[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) { pg[k] = make_float4(0.f, 0.f, 0.f, 0.f); pb[k] = pg[k]; pa[k] = pg[k]; }

  for (int rr = 0; rr < rpw; ++rr) {
    const int64_t b = ((int64_t)blockIdx.x * rpw + rr) * 4 + w;
    if (b >= nb) break;
    const float rs = rstd[b];
    float4 dxh[NV], xh[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t e = 4 * (int64_t)(lane + 64 * k);
      if (e >= H) { dxh[k] = make_float4(0.f, 0.f, 0.f, 0.f); xh[k] = dxh[k]; continue; }
      const float4 g = *reinterpret_cast<const float4*>(dh + b * H + e);
      xh[k] = *reinterpret_cast<const float4*>(xhat + b * H + e);
      const float4 lw = *reinterpret_cast<const float4*>(ln_w + e);
      const float4 lb = *reinterpret_cast<const float4*>(ln_b + e);
      const float gv[4] = {g.x, g.y, g.z, g.w};
      const float xv[4] = {xh[k].x, xh[k].y, xh[k].z, xh[k].w};
      const float wv[4] = {lw.x, lw.y, lw.z, lw.w};
      const float bv[4] = {lb.x, lb.y, lb.z, lb.w};
      float dy[4], dx[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t idx = (uint64_t)(b * H + e + i);
        const float dm = train ? dropout_mult(p_drop, scale, drop_mult, idx, seed, step, tag) : 1.f;
        dy[i] = gv[i] * dm * gelu_grad_f(xv[i] * wv[i] + bv[i]);
        dx[i] = dy[i] * wv[i];
        s1 += dx[i];
        s2 += dx[i] * xv[i];
      }
      pg[k].x += dy[0] * xv[0]; pg[k].y += dy[1] * xv[1]; pg[k].z += dy[2] * xv[2]; pg[k].w += dy[3] * xv[3];
      pb[k].x += dy[0]; pb[k].y += dy[1]; pb[k].z += dy[2]; pb[k].w += dy[3];
      dxh[k] = make_float4(dx[0], dx[1], dx[2], dx[3]);
    }
    const float m1 = wave_sum(s1) * invH, m2 = wave_sum(s2) * invH;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t e = 4 * (int64_t)(lane + 64 * k);
      if (e >= H) continue;
      float4 o;
      o.x = rs * (dxh[k].x - m1 - xh[k].x * m2);
      o.y = rs * (dxh[k].y - m1 - xh[k].y * m2);
      o.z = rs * (dxh[k].z - m1 - xh[k].z * m2);
      o.w = rs * (dxh[k].w - m1 - xh[k].w * m2);
      *reinterpret_cast<float4*>(da + b * H + e) = o;
      pa[k].x += o.x; pa[k].y += o.y; pa[k].z += o.z; pa[k].w += o.w;
    }
  }
  // combine the 4 waves' column partials in a fixed order
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int64_t e = 4 * (int64_t)(lane + 64 * k);
    if (e >= H) continue;
    *reinterpret_cast<float4*>(lds_part + (w * 3 + 0) * H + e) = pg[k];
    *reinterpret_cast<float4*>(lds_part + (w * 3 + 1) * H + e) = pb[k];
    *reinterpret_cast<float4*>(lds_part + (w * 3 + 2) * H + e) = pa[k];
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < 3 * H; i += blockDim.x) {
    const float v = ((lds_part[i] + lds_part[3 * H + i]) + lds_part[6 * H + i]) + lds_part[9 * H + i];
    if (ticket) st_shared_f(&part[(int64_t)blockIdx.x * 3 * H + i], v);
    else part[(int64_t)blockIdx.x * 3 * H + i] = v;
  }
  // short grids: the last block to finish sums the partials (same order as k_ln_part_reduce)
  if (!ticket || !last_block_arrives(ticket, gridDim.x)) return;
  // coherent loads batched 8 partials deep (a serial chain would pay the full latency per partial)
  const int np = gridDim.x;
  for (int64_t i = threadIdx.x; i < 3 * H; i += blockDim.x) {
    float s = 0.f;
    int p = 0;
    for (; p + 8 <= np; p += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = ld_shared_f(&part[(int64_t)(p + j) * 3 * H + i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; p < np; ++p) s += ld_shared_f(&part[(int64_t)p * 3 * H + i]);
    if (i < H) d_ln_w[i] = s;
    else if (i < 2 * H) d_ln_b[i - H] = s;
    else if (d_bias) d_bias[i - 2 * H] = s;
  }
}

// Sum the per-block partials [nparts][3][H] -> (d_ln_w, d_ln_b, d_bias), fixed order:
// 64 columns per block, 4 groups of partials (p = g mod 4) per column, loads batched
// 8 deep, the groups combined in order through LDS.
__global__ void __launch_bounds__(256) k_ln_part_reduce(const float* __restrict__ part, int64_t nparts, int64_t H,
                                                        float* __restrict__ d_ln_w, float* __restrict__ d_ln_b,
                                                        float* __restrict__ d_bias) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + cl;
  float s = 0.f;
  if (i < 3 * H) {
    int64_t p = g;
    for (; p + 28 < nparts; p += 32) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(p + 4 * j) * 3 * H + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; p < nparts; p += 4) s += part[p * 3 * H + i];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g != 0 || i >= 3 * H) return;
  const float t = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
  if (i < H) d_ln_w[i] = t;
  else if (i < 2 * H) d_ln_b[i - H] = t;
  else if (d_bias) d_bias[i - 2 * H] = t;
}

// --------------------------------------------------------------------------
// dense [B, N] -> CSR (row order preserved)
__global__ void __launch_bounds__(256) k_dense_row_count(const float* __restrict__ x, int64_t N,
                                                         int64_t* __restrict__ cnt) {
  __shared__ float red[4];
  const int64_t b = blockIdx.x;
  float c = 0.f;
  for (int64_t i = threadIdx.x; i < N; i += 256) c += (x[b * N + i] != 0.f) ? 1.f : 0.f;
  c = block_sum<256>(c, red);
  if (threadIdx.x == 0) cnt[b] = (int64_t)c;
}

// Single-block exclusive scan of n int64 counts in place -> row_ptr[0..n].
__global__ void __launch_bounds__(1024) k_scan_i64(int64_t* __restrict__ v, int64_t n) {
  __shared__ int64_t sh[1024];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < n; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t val = (i < n) ? v[i] : 0;
    sh[threadIdx.x] = val;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int64_t t = (threadIdx.x >= o) ? sh[threadIdx.x - o] : 0;
      __syncthreads();
      sh[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < n) v[i] = carry + sh[threadIdx.x] - val;
    __syncthreads();
    if (threadIdx.x == 1023) carry += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) v[n] = carry;
}

__global__ void __launch_bounds__(256) k_dense_compact(const float* __restrict__ x, int64_t N,
                                                       const int64_t* __restrict__ row_ptr,
                                                       int32_t* __restrict__ col, float* __restrict__ val,
                                                       int64_t cap) {
  __shared__ int wcnt[4];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t pos = row_ptr[b];
  for (int64_t base = 0; base < N; base += 256) {
    const int64_t i = base + threadIdx.x;
    const float v = (i < N) ? x[b * N + i] : 0.f;
    const bool nz = v != 0.f;
    const uint64_t m = __ballot(nz);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += wcnt[k];
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (nz) {
      const int64_t p = pos + off + before;
      if (p < cap) { col[p] = (int32_t)i; val[p] = v; }
    }
    pos += tot;
    __syncthreads();
  }
}

// --------------------------------------------------------------------------
// Row-sparse W1 gradient (K12): counting sort of the batch nonzeros by item.
constexpr int kScanItemsPerBlock = 4096;  // 256 threads x 16 items

__global__ void __launch_bounds__(256) k_rg_count(const int64_t* __restrict__ row_ptr,
                                                  const int32_t* __restrict__ col_idx,
                                                  const int32_t* __restrict__ rows,
    const int64_t* __restrict__ rows_offset, int64_t nb,
                                                  int32_t* __restrict__ cnt, unsigned long long* __restrict__ lb_state,
                                                  int64_t lb_words) {
  // the next launch's look-back state (k_rg_scan_lb): status words and its block-id counter start at zero
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lb_words; i += (int64_t)gridDim.x * blockDim.x)
    lb_state[i] = 0ull;
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t r = batch_row(rows, rows_offset, b);
  for (int64_t e = row_ptr[r] + lane; e < row_ptr[r + 1]; e += 64) atomicAdd(&cnt[col_idx[e]], 1);
}

// One-pass scan of the per-item counts (decoupled look-back): slots in ascending item order for the
// items with cnt > 0, their segment offsets, n_unique and seg_off[n_unique]. A block takes the next
// 4096 items in the order blocks start (block id from an atomic counter, so every block it waits for
// has already started), publishes its aggregate (#items, #entries), then sums its predecessors'
// words back to the first inclusive prefix and publishes its own. A status word is
// [2-bit status | 31-bit items | 31-bit entries] (status 1 aggregate, 2 inclusive prefix), read and
// written with agent-scope atomics, so no separate data needs fencing. Replaces three launches
// (block totals, their scan, the block scans).
__device__ __forceinline__ unsigned long long lb_word(unsigned st, long long f, long long c) {
  return ((unsigned long long)st << 62) | ((unsigned long long)f << 31) | (unsigned long long)c;
}

__global__ void __launch_bounds__(256) k_rg_scan_lb(int32_t* __restrict__ cnt, int64_t N,
                                                    unsigned long long* __restrict__ state, int64_t nblk,
                                                    int32_t* __restrict__ slot_of, int32_t* __restrict__ item_of,
                                                    int32_t* __restrict__ seg_off, int64_t cap,
                                                    int32_t* __restrict__ n_unique) {
  __shared__ int sf[256], sc[256];
  __shared__ int s_bid;
  __shared__ long long s_pf, s_pc;
  unsigned* ctr = reinterpret_cast<unsigned*>(state + nblk);
  if (threadIdx.x == 0) s_bid = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int bid = s_bid;
  const int64_t base = (int64_t)bid * kScanItemsPerBlock + threadIdx.x * 16;
  int c[16];
  int nf = 0, nc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t j = base + i;
    c[i] = (j < N) ? cnt[j] : 0;
    nf += c[i] > 0;
    nc += c[i];
  }
  sf[threadIdx.x] = nf;
  sc[threadIdx.x] = nc;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int tf = (threadIdx.x >= o) ? sf[threadIdx.x - o] : 0;
    const int tc = (threadIdx.x >= o) ? sc[threadIdx.x - o] : 0;
    __syncthreads();
    sf[threadIdx.x] += tf;
    sc[threadIdx.x] += tc;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const long long tf = sf[255], tc = sc[255];
    long long pf = 0, pc = 0;
    if (bid == 0) {
      __hip_atomic_store(&state[0], lb_word(2u, tf, tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&state[bid], lb_word(1u, tf, tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int j = bid - 1; j >= 0; --j) {
        unsigned long long v;
        do {
          v = __hip_atomic_load(&state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } while ((v >> 62) == 0ull);
        pf += (long long)((v >> 31) & 0x7fffffffull);
        pc += (long long)(v & 0x7fffffffull);
        if ((v >> 62) == 2ull) break;
      }
      __hip_atomic_store(&state[bid], lb_word(2u, pf + tf, pc + tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_pf = pf;
    s_pc = pc;
    if (bid == nblk - 1) {
      *n_unique = (int32_t)(pf + tf);
      if (pf + tf <= cap) seg_off[pf + tf] = (int32_t)(pc + tc);
    }
  }
  __syncthreads();
  int64_t slot = s_pf + sf[threadIdx.x] - nf;
  int64_t off = s_pc + sc[threadIdx.x] - nc;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (c[i] > 0) {
      const int64_t j = base + i;
      if (slot < cap) {
        slot_of[j] = (int32_t)slot;
        item_of[slot] = (int32_t)j;
        seg_off[slot] = (int32_t)off;
      }
      cnt[j] = 0;  // leave the histogram zeroed for the next batch
      ++slot;
      off += c[i];
    }
  }
}

// Small catalogs (N <= kSmallScanItems): scan1 + scan2 + scan3 in one block,
// chunk by chunk with a running carry (one launch instead of three).
constexpr int64_t kSmallScanItems = 64 * 1024;


// 1024 threads x 4 items per chunk; wave shuffles + one LDS pass per chunk.
__global__ void __launch_bounds__(1024) k_rg_scan_small(int32_t* __restrict__ cnt, int64_t N,
                                                        int32_t* __restrict__ slot_of, int32_t* __restrict__ item_of,
                                                        int32_t* __restrict__ seg_off, int64_t cap,
                                                        int32_t* __restrict__ n_unique) {
  __shared__ int wf[16], wc[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t carry_f = 0, carry_c = 0;
  for (int64_t base0 = 0; base0 < N; base0 += 4096) {
    const int64_t base = base0 + threadIdx.x * 4;
    int c[4];
    int nf = 0, nc = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t j = base + i;
      c[i] = (j < N) ? cnt[j] : 0;
      nf += c[i] > 0;
      nc += c[i];
    }
    const int xf = wave_incl_scan(nf, lane), xc = wave_incl_scan(nc, lane);
    if (lane == 63) { wf[w] = xf; wc[w] = xc; }
    __syncthreads();
    int pf = 0, pc = 0, tf = 0, tc = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k < w) { pf += wf[k]; pc += wc[k]; }
      tf += wf[k];
      tc += wc[k];
    }
    int64_t slot = carry_f + pf + xf - nf;
    int64_t off = carry_c + pc + xc - nc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (c[i] > 0) {
        const int64_t j = base + i;
        if (slot < cap) {
          slot_of[j] = (int32_t)slot;
          item_of[slot] = (int32_t)j;
          seg_off[slot] = (int32_t)off;
        }
        cnt[j] = 0;
        ++slot;
        off += c[i];
      }
    }
    carry_f += tf;
    carry_c += tc;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *n_unique = (int32_t)carry_f;
    if (carry_f <= cap) seg_off[carry_f] = (int32_t)carry_c;
  }
}

// Whole plan in one block for small batches (hvae_rgplan.h): one launch of the shared block body.
__global__ void __launch_bounds__(1024) k_rg_plan_small(const int64_t* __restrict__ row_ptr,
                                                        const int32_t* __restrict__ col_idx,
                                                        const float* __restrict__ vals,
                                                        const int32_t* __restrict__ rows,
                                                        const int64_t* __restrict__ rows_offset, int64_t nb,
                                                        int32_t* __restrict__ slot_of, int32_t* __restrict__ item_of,
                                                        int32_t* __restrict__ seg_off,
                                                        int32_t* __restrict__ contrib_row,
                                                        float* __restrict__ contrib_val,
                                                        int32_t* __restrict__ contrib_slot,
                                                        int32_t* __restrict__ n_unique) {
  __shared__ unsigned long long key[kPlanSmallCap];
  __shared__ float kv[kPlanSmallCap];
  __shared__ int roff[kPlanSmallRows + 1];
  __shared__ int64_t rbeg[kPlanSmallRows];
  __shared__ int wsum[16];
  rg_plan_small_block(row_ptr, col_idx, vals, rows, rows_offset, nb, slot_of, item_of, seg_off, contrib_row,
                      contrib_val, contrib_slot, n_unique, key, kv, roff, rbeg, wsum);
}

__global__ void __launch_bounds__(256) k_rg_scatter(const int64_t* __restrict__ row_ptr,
                                                    const int32_t* __restrict__ col_idx,
                                                    const float* __restrict__ vals,
                                                    const int32_t* __restrict__ rows,
    const int64_t* __restrict__ rows_offset, int64_t nb,
                                                    const int32_t* __restrict__ slot_of,
                                                    const int32_t* __restrict__ seg_off,
                                                    int32_t* __restrict__ fill,
                                                    int32_t* __restrict__ contrib_row,
                                                    float* __restrict__ contrib_val, int64_t cap) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int64_t r = batch_row(rows, rows_offset, b);
  for (int64_t e = row_ptr[r] + lane; e < row_ptr[r + 1]; e += 64) {
    const int s = slot_of[col_idx[e]];
    const int64_t pos = (int64_t)seg_off[s] + atomicAdd(&fill[s], 1);
    if (pos < cap) {
      contrib_row[pos] = (int32_t)b;
      contrib_val[pos] = vals[e];
    }
  }
}

// Sort every item segment's contributions by batch row (keys are unique within
// a segment: a CSR row holds an item at most once), in place; record each
// contribution's slot; re-zero the fill counters.
//   len <= 64          one wave, bitonic network in registers
//   len > 64, nb <= kRankRows   one block: rank = popcount of a batch-row bitmap
//                      below the key (O(len + nb/32)), via a staging copy in `stage`
//   otherwise          one block, bitonic in LDS (len <= kSegSortCap) or an
//                      in-place selection sort (never met at the path's batch sizes)
constexpr int kSegSortCap = 4096;
constexpr int kRankRows = 32768;
__global__ void __launch_bounds__(256) k_rg_sort(const int32_t* __restrict__ n_unique,
                                                 const int32_t* __restrict__ seg_off, int32_t* __restrict__ fill,
                                                 int32_t* __restrict__ contrib_row, float* __restrict__ contrib_val,
                                                 int32_t* __restrict__ contrib_slot, int2* __restrict__ stage,
                                                 int64_t nb) {
  __shared__ int key[kSegSortCap];
  __shared__ float kval[kSegSortCap];
  __shared__ unsigned bm[kRankRows / 32];
  __shared__ int pre[kRankRows / 32];
  __shared__ int red[8];
  const int nu = *n_unique;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (int s = gw; s < nu; s += nw) {
    const int beg = seg_off[s], len = seg_off[s + 1] - beg;
    if (lane == 0) fill[s] = 0;
    for (int i = lane; i < len; i += 64) contrib_slot[beg + i] = s;
    if (len <= 1 || len > 64) continue;
    int k_ = lane < len ? contrib_row[beg + lane] : 0x7fffffff;
    float v_ = lane < len ? contrib_val[beg + lane] : 0.f;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const int pk = __shfl_xor(k_, j);
        const float pv = __shfl_xor(v_, j);
        const bool keep_min = ((lane & k) == 0) == ((lane & j) == 0);
        if (keep_min ? (pk < k_) : (pk > k_)) { k_ = pk; v_ = pv; }
      }
    if (lane < len) { contrib_row[beg + lane] = k_; contrib_val[beg + lane] = v_; }
  }
  const int words = (int)((nb + 31) / 32);
  for (int s = blockIdx.x; s < nu; s += gridDim.x) {
    const int beg = seg_off[s], len = seg_off[s + 1] - beg;
    if (len <= 64) continue;  // block-uniform
    __syncthreads();
    if (nb <= kRankRows) {
      for (int w = threadIdx.x; w < words; w += 256) bm[w] = 0u;
      __syncthreads();
      for (int i = threadIdx.x; i < len; i += 256) {
        const int b = contrib_row[beg + i];
        stage[beg + i] = make_int2(b, __float_as_int(contrib_val[beg + i]));
        atomicOr(&bm[b >> 5], 1u << (b & 31));
      }
      __syncthreads();
      // exclusive prefix of the word popcounts (each thread owns a run of consecutive words)
      const int per = (words + 255) / 256;
      const int w0 = threadIdx.x * per;
      int c = 0;
      for (int w = w0; w < min(words, w0 + per); ++w) c += __popc(bm[w]);
      int incl = c;  // inclusive scan over the block
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (lane == 63) red[threadIdx.x >> 6] = incl;
      __syncthreads();
      int wbase = 0;
      for (int q = 0; q < (threadIdx.x >> 6); ++q) wbase += red[q];
      int run = wbase + incl - c;
      for (int w = w0; w < min(words, w0 + per); ++w) { pre[w] = run; run += __popc(bm[w]); }
      __syncthreads();
      for (int i = threadIdx.x; i < len; i += 256) {
        const int2 e = stage[beg + i];
        const int b = e.x;
        const int rank = pre[b >> 5] + __popc(bm[b >> 5] & ((1u << (b & 31)) - 1u));
        contrib_row[beg + rank] = b;
        contrib_val[beg + rank] = __int_as_float(e.y);
      }
    } else if (len <= kSegSortCap) {
      int p2 = 128;
      while (p2 < len) p2 <<= 1;
      for (int i = threadIdx.x; i < p2; i += 256) {
        key[i] = (i < len) ? contrib_row[beg + i] : 0x7fffffff;
        kval[i] = (i < len) ? contrib_val[beg + i] : 0.f;
      }
      __syncthreads();
      for (int k = 2; k <= p2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
          for (int i = threadIdx.x; i < p2; i += 256) {
            const int ixj = i ^ j;
            if (ixj > i) {
              const bool up = (i & k) == 0;
              const int a = key[i], c = key[ixj];
              if ((a > c) == up) {
                key[i] = c; key[ixj] = a;
                const float t = kval[i]; kval[i] = kval[ixj]; kval[ixj] = t;
              }
            }
          }
          __syncthreads();
        }
      }
      for (int i = threadIdx.x; i < len; i += 256) { contrib_row[beg + i] = key[i]; contrib_val[beg + i] = kval[i]; }
    } else {
      for (int i = 0; i < len - 1; ++i) {  // selection sort, one block
        int best = 0x7fffffff, at = -1;
        for (int j = i + threadIdx.x; j < len; j += 256) {
          const int k = contrib_row[beg + j];
          if (k < best) { best = k; at = j; }
        }
        for (int o = 32; o > 0; o >>= 1) {
          const int ob = __shfl_xor(best, o), oa = __shfl_xor(at, o);
          if (ob < best) { best = ob; at = oa; }
        }
        __syncthreads();
        if (lane == 0) { key[threadIdx.x >> 6] = best; key[4 + (threadIdx.x >> 6)] = at; }
        __syncthreads();
        if (threadIdx.x == 0) {
          int bb = key[0], ba = key[4];
          for (int q = 1; q < 4; ++q)
            if (key[q] < bb) { bb = key[q]; ba = key[4 + q]; }
          const float tv = contrib_val[beg + ba];
          contrib_row[beg + ba] = contrib_row[beg + i];
          contrib_val[beg + ba] = contrib_val[beg + i];
          contrib_row[beg + i] = bb;
          contrib_val[beg + i] = tv;
        }
        __syncthreads();
      }
    }
  }
}

// Row gather rows[s, :] = sum over segment s (ascending batch row) of x * da[b, :],
// over the sorted contribution list in chunks of CH (8..64, sized so that the
// chunks give ~2K waves): one wave per chunk, lane i
// holds contribution i of the chunk, NV float4 columns per lane. A run of one
// segment that is the whole segment is written to its row; a run cut by a chunk
// edge goes to the chunk's head (run starts the chunk) or tail partial, stored
// agent-coherent; the wave then takes a ticket on the segment (fill[s], zero after
// the plan), and the wave that draws the segment's last ticket adds its chunks'
// partials up in chunk order (the first chunk's head or tail, then the heads) into
// the row and re-zeroes the ticket -- the same sums in the same order as a separate
// pass would, in one launch. Loads are batched 8 contributions deep.
// The clip's share of a W1 gradient row, taken while the row is in registers: each lane's sum of its x^2 in fp64,
// then the four lanes of a quad added by two DPP exchanges (no LDS round trips: a whole-wave shuffle reduction per
// row cost the apply 11-13 us at B = 4096), and lane 4 g stores quad g's sum: 16 fp64 partials per row
// (kRowSqParts), which the clip adds up in a fixed order.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
template <int NV>
__device__ __forceinline__ void row_sumsq(const float4 (&v)[NV], int lane, int64_t H, double* dst) {
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < NV; ++k)
    if (4 * (int64_t)(lane + 64 * k) < H)
      q += ((double)v[k].x * v[k].x + (double)v[k].y * v[k].y) + ((double)v[k].z * v[k].z + (double)v[k].w * v[k].w);
  q += dpp_d<0xB1>(q);  // quad_perm [1, 0, 3, 2]
  q += dpp_d<0x4E>(q);  // quad_perm [2, 3, 0, 1]
  if ((lane & 3) == 0) dst[lane >> 2] = q;
}

template <int NV>
__global__ void __launch_bounds__(256) k_rg_apply(const int32_t* __restrict__ n_unique,
                                                  const int32_t* __restrict__ seg_off,
                                                  const int32_t* __restrict__ contrib_row,
                                                  const float* __restrict__ contrib_val,
                                                  const int32_t* __restrict__ contrib_slot,
                                                  const float* __restrict__ da, int64_t H, int CH,
                                                  float* __restrict__ out_rows, float* __restrict__ part,
                                                  int32_t* __restrict__ ticket, double* __restrict__ rowsq) {
  const int nu = *n_unique;
  const int total = seg_off[nu];
  const int nchunks = (total + CH - 1) / CH;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (int c = gw; c < nchunks; c += nw) {
    const int c0 = c * CH, n = min(CH, total - c0);
    const int mb = lane < n ? contrib_row[c0 + lane] : 0;
    const float mx = lane < n ? contrib_val[c0 + lane] : 0.f;
    const int ms = lane < n ? contrib_slot[c0 + lane] : -1;
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    int run_lo = 0;
    for (int i0 = 0; i0 < n; i0 += 8) {
      float4 d[8][NV];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int b = __shfl(mb, i0 + j);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const int64_t col = 4 * (int64_t)(lane + 64 * k);
          d[j][k] = (i0 + j < n && col < H) ? *reinterpret_cast<const float4*>(da + (int64_t)b * H + col)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j;
        if (i >= n) break;
        const float x = __shfl(mx, i);
        const int si = __shfl(ms, i);
        const int snext = __shfl(ms, min(i + 1, 63));
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          acc[k].x += x * d[j][k].x; acc[k].y += x * d[j][k].y;
          acc[k].z += x * d[j][k].z; acc[k].w += x * d[j][k].w;
        }
        if (i == n - 1 || snext != si) {  // end of a run (wave-uniform)
          const int lo = c0 + run_lo, hi = c0 + i + 1;
          const int beg = seg_off[si], end = seg_off[si + 1];
          if (lo == beg && hi == end) {
            float* dst = out_rows + (int64_t)si * H;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
              const int64_t col = 4 * (int64_t)(lane + 64 * k);
              if (col < H) *reinterpret_cast<float4*>(dst + col) = acc[k];
            }
            if (rowsq) row_sumsq<NV>(acc, lane, H, rowsq + (int64_t)si * kRowSqParts);
          } else {
            const __amdgpu_buffer_rsrc_t prs = coherent_rsrc(part);
            const uint32_t dst = (uint32_t)((run_lo == 0 ? 2 * c : 2 * c + 1) * H) * 4u;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
              const int64_t col = 4 * (int64_t)(lane + 64 * k);
              if (col < H) st_sc1_f4(prs, dst + (uint32_t)col * 4u, acc[k]);
            }
            __builtin_amdgcn_s_waitcnt(0);  // this wave's partial has reached the coherence point
            const int ca = beg / CH, cb = (end - 1) / CH;
            int tk = 0;
            // The hand-off is MI355X_MICROARCH's measured valid form (sc1 16-B stores, every storing wave's
            // vmcnt(0) before its agent-scope ticket add, the last taker's sc1 16-B loads after its add returned);
            // the last taker adds an agent acquire (an L1 invalidate, no L2 writeback) so the ordering holds under
            // the HIP memory model too. An acq_rel add costs every chunk an L2 writeback: Syn-1M
            // rowgrad_apply 50 -> 96 us (profiles/r03_full_bench_syn1m.json).
            if (lane == 0) tk = __hip_atomic_fetch_add(ticket + si, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tk = __shfl(tk, 0, 64);
            if (tk == cb - ca) {  // the segment's last chunk to finish: its partials, in chunk order
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
              const __amdgpu_buffer_rsrc_t prs = coherent_rsrc(part);
              const uint32_t first = (uint32_t)((2 * ca + (beg % CH == 0 ? 0 : 1)) * H) * 4u;
              float4 tot[NV];
#pragma unroll
              for (int k = 0; k < NV; ++k) {
                const int64_t col = 4 * (int64_t)(lane + 64 * k);
                tot[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (col >= H) continue;
                float4 sum = ld_sc1_f4(prs, first + (uint32_t)col * 4u);
                for (int cc = ca + 1; cc <= cb; ++cc) {
                  const float4 v = ld_sc1_f4(prs, (uint32_t)((2 * cc) * H + col) * 4u);
                  sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
                }
                *reinterpret_cast<float4*>(out_rows + (int64_t)si * H + col) = sum;
                tot[k] = sum;
              }
              if (rowsq) row_sumsq<NV>(tot, lane, H, rowsq + (int64_t)si * kRowSqParts);
              if (lane == 0) __hip_atomic_store(ticket + si, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
#pragma unroll
          for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
          run_lo = i + 1;
        }
      }
    }
  }
}

// Small batches (the one-block plan): one wave per segment sums its contributions in ascending
// batch row straight into the segment's row (no chunk partials, no span pass). Loads batched 8 deep.
template <int NV>
__global__ void __launch_bounds__(256) k_rg_apply_seg(const int32_t* __restrict__ n_unique,
                                                      const int32_t* __restrict__ seg_off,
                                                      const int32_t* __restrict__ contrib_row,
                                                      const float* __restrict__ contrib_val,
                                                      const float* __restrict__ da, int64_t H,
                                                      float* __restrict__ out_rows, double* __restrict__ rowsq) {
  const int nu = *n_unique;
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  for (int s = gw; s < nu; s += nw) {
    const int beg = seg_off[s], len = seg_off[s + 1] - beg;
    float4 acc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < len; i0 += 64) {
      const int n = min(64, len - i0);
      const int mb = lane < n ? contrib_row[beg + i0 + lane] : 0;
      const float mx = lane < n ? contrib_val[beg + i0 + lane] : 0.f;
      for (int j0 = 0; j0 < n; j0 += 8) {
        float4 d[8][NV];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = __shfl(mb, min(j0 + j, 63));
#pragma unroll
          for (int k = 0; k < NV; ++k) {
            const int64_t col = 4 * (int64_t)(lane + 64 * k);
            d[j][k] = (j0 + j < n && col < H) ? *reinterpret_cast<const float4*>(da + (int64_t)b * H + col)
                                              : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = (j0 + j < n) ? __shfl(mx, min(j0 + j, 63)) : 0.f;
#pragma unroll
          for (int k = 0; k < NV; ++k) {
            acc[k].x += x * d[j][k].x; acc[k].y += x * d[j][k].y;
            acc[k].z += x * d[j][k].z; acc[k].w += x * d[j][k].w;
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int64_t col = 4 * (int64_t)(lane + 64 * k);
      if (col < H) *reinterpret_cast<float4*>(out_rows + (int64_t)s * H + col) = acc[k];
    }
    if (rowsq) row_sumsq<NV>(acc, lane, H, rowsq + (int64_t)s * kRowSqParts);
  }
}

__global__ void k_rg_to_dense(const int32_t* __restrict__ n_unique, const int32_t* __restrict__ item_of,
                              const float* __restrict__ rows, int64_t H, float* __restrict__ dense,
                              int64_t ld) {
  const int nu = *n_unique;
  for (int s = blockIdx.x; s < nu; s += gridDim.x) {
    const int64_t j = item_of[s];
    for (int64_t h = threadIdx.x; h < H; h += blockDim.x) dense[j * ld + h] = rows[(int64_t)s * H + h];
  }
}

}  // namespace hvae

using namespace hvae;

// ------------------------------------------------------------- launchers ---
#define HVAE_NV_DISPATCH(H, KERNEL_CALL)                                        \
  do {                                                                          \
    const int64_t nv_ = cdiv((H), 256);                                         \
    if (nv_ <= 1) { constexpr int NV = 1; KERNEL_CALL; }                        \
    else if (nv_ <= 2) { constexpr int NV = 2; KERNEL_CALL; }                   \
    else if (nv_ <= 4) { constexpr int NV = 4; KERNEL_CALL; }                   \
    else if (nv_ <= 8) { constexpr int NV = 8; KERNEL_CALL; }                   \
    else HVAE_FAIL(HVAE_ERR_UNSUPPORTED, "hidden width %lld > 2048 unsupported", (long long)(H)); \
  } while (0)

static int check_hidden(int64_t H) {
  HVAE_REQUIRE(H > 0 && H % 4 == 0, "hidden width %lld must be a positive multiple of 4",
               (long long)H);
  return HVAE_OK;
}

extern "C" int hvae_encoder_fwd(const hvae_csr_batch* x, const float* w1t, const float* b1,
                                const float* ln_w, const float* ln_b, int64_t H, float p_drop,
                                const float* drop_mult, uint64_t seed, const int64_t* step_dev,
                                int train, float* h_out, float* xhat_out, float* rstd_out,
                                void* stream) {
  HVAE_REQUIRE(x && x->row_ptr && w1t && b1 && ln_w && ln_b && h_out, "hvae_encoder_fwd: null arg");
  if (int rc = check_hidden(H)) return rc;
  if (x->nb == 0) return HVAE_OK;
  HVAE_REQUIRE(x->col_idx && x->vals, "hvae_encoder_fwd: null CSR arrays");
  const float scale = (p_drop < 1.f) ? 1.0f / (1.0f - p_drop) : 0.f;
  const unsigned grid = (unsigned)cdiv(x->nb, 4);
  ProbeScope probe("encoder_fwd", as_stream(stream));
  HVAE_NV_DISPATCH(H, (k_encoder_sparse_fwd<NV><<<grid, 256, 0, as_stream(stream)>>>(
                          x->row_ptr, x->col_idx, x->vals, x->rows, x->rows_offset, x->nb, w1t, b1, ln_w, ln_b, H,
                          p_drop, scale, drop_mult, seed, step_dev, train, h_out, xhat_out,
                          rstd_out)));
  HVAE_LAUNCH_CHECK("k_encoder_sparse_fwd");
  return HVAE_OK;
}

extern "C" int hvae_ln_gelu_drop_fwd(const float* a, const float* ln_w, const float* ln_b,
                                     int64_t nb, int64_t H, float p_drop, const float* drop_mult,
                                     uint64_t seed, const int64_t* step_dev, uint32_t layer,
                                     int train, float* h_out, float* xhat_out, float* rstd_out,
                                     void* stream) {
  HVAE_REQUIRE(a && ln_w && ln_b && h_out, "hvae_ln_gelu_drop_fwd: null arg");
  if (int rc = check_hidden(H)) return rc;
  if (nb == 0) return HVAE_OK;
  const float scale = (p_drop < 1.f) ? 1.0f / (1.0f - p_drop) : 0.f;
  const unsigned grid = (unsigned)cdiv(nb, 4);
  HVAE_NV_DISPATCH(H, (k_ln_gelu_drop_fwd<NV><<<grid, 256, 0, as_stream(stream)>>>(
                          a, ln_w, ln_b, nb, H, p_drop, scale, drop_mult, seed, step_dev,
                          kTagEncDrop + layer, train, h_out, xhat_out, rstd_out)));
  HVAE_LAUNCH_CHECK("k_ln_gelu_drop_fwd");
  return HVAE_OK;
}

extern "C" size_t hvae_ln_gelu_drop_bwd_workspace(int64_t nb, int64_t H) {
  return (size_t)cdiv(nb, 4 * ln_bwd_rows_per_wave(nb)) * 3 * (size_t)H * sizeof(float);
}

extern "C" int hvae_ln_gelu_drop_bwd(const float* dh, const float* xhat, const float* rstd,
                                     const float* ln_w, const float* ln_b, int64_t nb, int64_t H,
                                     float p_drop, const float* drop_mult, uint64_t seed,
                                     const int64_t* step_dev, uint32_t layer, int train, float* da,
                                     float* d_ln_w, float* d_ln_b, float* d_bias, void* ws, size_t ws_bytes,
                                     void* stream) {
  HVAE_REQUIRE(dh && xhat && rstd && ln_w && ln_b && da && d_ln_w && d_ln_b,
               "hvae_ln_gelu_drop_bwd: null arg");
  if (int rc = check_hidden(H)) return rc;
  if (nb == 0) {
    HVAE_HIP(hipMemsetAsync(d_ln_w, 0, H * sizeof(float), as_stream(stream)));
    HVAE_HIP(hipMemsetAsync(d_ln_b, 0, H * sizeof(float), as_stream(stream)));
    if (d_bias) HVAE_HIP(hipMemsetAsync(d_bias, 0, H * sizeof(float), as_stream(stream)));
    return HVAE_OK;
  }
  const size_t need = hvae_ln_gelu_drop_bwd_workspace(nb, H);
  if (ws_bytes < need || !ws)
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae_ln_gelu_drop_bwd: workspace %zu < %zu", ws_bytes, need);
  const float scale = (p_drop < 1.f) ? 1.0f / (1.0f - p_drop) : 0.f;
  const int rpw = ln_bwd_rows_per_wave(nb);
  const int64_t nparts = cdiv(nb, 4 * rpw);
  const size_t lds = (size_t)12 * H * sizeof(float);
  unsigned* ticket = nullptr;  // fused final reduction when the partial count is small
  if (nparts <= 64 && !(ticket = ticket_slice())) return HVAE_ERR_HIP;
  HVAE_REQUIRE(lds <= 64 * 1024, "hvae_ln_gelu_drop_bwd: H too large (<= 1364)");
  ProbeScope probe("ln_bwd", as_stream(stream));
  HVAE_NV_DISPATCH(H, (k_ln_gelu_drop_bwd<NV><<<(unsigned)nparts, 256, lds, as_stream(stream)>>>(
                          dh, xhat, rstd, ln_w, ln_b, nb, H, p_drop, scale, drop_mult, seed,
                          step_dev, kTagEncDrop + layer, train, rpw, da, (float*)ws, ticket, d_ln_w, d_ln_b,
                          d_bias)));
  HVAE_LAUNCH_CHECK("k_ln_gelu_drop_bwd");
  if (!ticket) {
    k_ln_part_reduce<<<(unsigned)cdiv(3 * H, 64), 256, 0, as_stream(stream)>>>((const float*)ws, nparts,
                                                                                 H, d_ln_w, d_ln_b, d_bias);
    HVAE_LAUNCH_CHECK("k_ln_part_reduce");
  }
  return HVAE_OK;
}

extern "C" size_t hvae_dense_to_csr_workspace(int64_t, int64_t) { return 0; }

extern "C" int hvae_dense_to_csr(const float* x, int64_t B, int64_t N, int64_t* row_ptr,
                                 int32_t* col_idx, float* vals, int64_t cap, void*, size_t,
                                 void* stream) {
  HVAE_REQUIRE(row_ptr && B >= 0 && N >= 0, "hvae_dense_to_csr: bad args");
  HVAE_REQUIRE(N < (int64_t)INT32_MAX, "hvae_dense_to_csr: N too large");
  if (B == 0) {
    HVAE_HIP(hipMemsetAsync(row_ptr, 0, sizeof(int64_t), as_stream(stream)));
    return HVAE_OK;
  }
  HVAE_REQUIRE(x && col_idx && vals, "hvae_dense_to_csr: null arg");
  k_dense_row_count<<<(unsigned)B, 256, 0, as_stream(stream)>>>(x, N, row_ptr);
  HVAE_LAUNCH_CHECK("k_dense_row_count");
  k_scan_i64<<<1, 1024, 0, as_stream(stream)>>>(row_ptr, B);
  HVAE_LAUNCH_CHECK("k_scan_i64");
  k_dense_compact<<<(unsigned)B, 256, 0, as_stream(stream)>>>(x, N, row_ptr, col_idx, vals, cap);
  HVAE_LAUNCH_CHECK("k_dense_compact");
  return HVAE_OK;
}

extern "C" size_t hvae_w1_rowgrad_workspace(int64_t n_items) {
  return (size_t)(cdiv(n_items, kScanItemsPerBlock) + 1) * sizeof(int64_t);  // look-back words + block counter
}

namespace hvae {
int rg_plan_sorted(const hvae_csr_batch* x, const hvae_rowgrad* rg, hipStream_t st);
int64_t rgsort_scratch_floats(int64_t cap, int64_t N);
}  // namespace hvae
static int env_flag_ab(const char* name, int dflt) {
  const char* v = ab_getenv(name);
  return (v && *v) ? (atoi(v) != 0 ? 1 : 0) : dflt;
}

static int rg_check(const hvae_rowgrad* rg) {
  HVAE_REQUIRE(rg && rg->cnt && rg->slot_of && rg->item_of && rg->seg_off && rg->fill && rg->contrib_row &&
                   rg->contrib_val && rg->rows && rg->n_unique,
               "hvae_w1_rowgrad: null rowgrad buffer");
  return HVAE_OK;
}

static unsigned rg_grid(const hvae_rowgrad* rg) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(rg->cap, 4), 2048));
}

extern "C" int hvae_w1_rowgrad_plan(const hvae_csr_batch* x, const hvae_rowgrad* rg, void* ws, size_t ws_bytes,
                                    void* stream) {
  HVAE_REQUIRE(x && x->row_ptr, "hvae_w1_rowgrad_plan: null batch");
  if (int rc = rg_check(rg)) return rc;
  HVAE_REQUIRE(rg->n_items == x->n_items, "hvae_w1_rowgrad: n_items mismatch");
  const int64_t N = x->n_items;
  const size_t need = hvae_w1_rowgrad_workspace(N);
  if (ws_bytes < need || !ws)
    HVAE_FAIL(HVAE_ERR_WORKSPACE, "hvae_w1_rowgrad: workspace %zu < %zu", ws_bytes, need);
  hipStream_t st = as_stream(stream);
  if (x->nb == 0) {
    HVAE_HIP(hipMemsetAsync(rg->n_unique, 0, sizeof(int32_t), st));
    return HVAE_OK;
  }
  if (rg->cap <= kPlanSmallCap && x->nb <= kPlanSmallRows) {  // the whole plan in one block
    HVAE_REQUIRE(rg->contrib_slot, "hvae_w1_rowgrad_plan: null contrib_slot");
    ProbeScope probe("rowgrad_plan", st);
    k_rg_plan_small<<<1, 1024, 0, st>>>(x->row_ptr, x->col_idx, x->vals, x->rows, x->rows_offset, x->nb,
                                        rg->slot_of, rg->item_of, rg->seg_off, rg->contrib_row, rg->contrib_val,
                                        rg->contrib_slot, rg->n_unique);
    HVAE_LAUNCH_CHECK("k_rg_plan_small");
    return HVAE_OK;
  }
  // the sorted plan (hvae_rgsort.hip): one stable radix sort instead of per-item atomics: 3.6x faster at data
  // parallelism's W = 8 union (782 -> 216 us), 1.5x at one rank's batch (121 -> 79 us,
  // profiles/r03_rowgrad_sorted_vs_atomic.jsonl). Round 3 kept the atomic plan below 150 K entries because the
  // step measured slower with the sort at Syn-1M (1.20 -> 1.30 ms) -- but that step was host-bound on a per-step
  // sort of all row lengths in the run loop (fixed in round 6); with the host ahead of the device the sorted plan
  // runs Syn-1M in 1.061-1.064 ms against 1.141 and the Syn-10M shard in 10.95-10.97 against 11.01-11.02
  // (profiles/r06_rowgrad_sorted_ab.jsonl), so it now serves every batch past the one-block plan's reach from
  // kSortedPlanMinCap entries. HVAE_RG_SORTED (A/B build): 1 always sorted, 0 never.
  constexpr int64_t kSortedPlanMinCap = 32768;
  const int sorted_ab = env_flag_ab("HVAE_RG_SORTED", -1);
  if (sorted_ab == 1 || (sorted_ab == -1 && rg->cap >= kSortedPlanMinCap)) {
    const int rc = rg_plan_sorted(x, rg, st);
    if (rc != HVAE_ERR_UNSUPPORTED) return rc;
  }
  const unsigned rgrid = (unsigned)cdiv(x->nb, 4);
  const bool small_scan = N <= kSmallScanItems;
  const int64_t nblk = cdiv(N, kScanItemsPerBlock);
  HVAE_REQUIRE(N < (1ll << 31) && rg->cap < (1ll << 31), "hvae_w1_rowgrad_plan: N or cap >= 2^31");
  unsigned long long* lb = (unsigned long long*)ws;
  k_rg_count<<<rgrid, 256, 0, st>>>(x->row_ptr, x->col_idx, x->rows, x->rows_offset, x->nb, rg->cnt, lb,
                                    small_scan ? 0 : nblk + 1);
  HVAE_LAUNCH_CHECK("k_rg_count");
  if (small_scan) {
    k_rg_scan_small<<<1, 1024, 0, st>>>(rg->cnt, N, rg->slot_of, rg->item_of, rg->seg_off, rg->cap, rg->n_unique);
    HVAE_LAUNCH_CHECK("k_rg_scan_small");
  } else {
    k_rg_scan_lb<<<(unsigned)nblk, 256, 0, st>>>(rg->cnt, N, lb, nblk, rg->slot_of, rg->item_of, rg->seg_off,
                                                rg->cap, rg->n_unique);
    HVAE_LAUNCH_CHECK("k_rg_scan_lb");
  }
  k_rg_scatter<<<rgrid, 256, 0, st>>>(x->row_ptr, x->col_idx, x->vals, x->rows, x->rows_offset, x->nb, rg->slot_of,
                                      rg->seg_off, rg->fill, rg->contrib_row, rg->contrib_val,
                                      rg->cap);
  HVAE_LAUNCH_CHECK("k_rg_scatter");
  HVAE_REQUIRE(rg->part && rg->part_floats >= 2 * rg->cap, "hvae_w1_rowgrad_plan: part scratch too small");
  k_rg_sort<<<rg_grid(rg), 256, 0, st>>>(rg->n_unique, rg->seg_off, rg->fill, rg->contrib_row, rg->contrib_val,
                                         rg->contrib_slot, (int2*)rg->part, x->nb);
  HVAE_LAUNCH_CHECK("k_rg_sort");
  return HVAE_OK;
}

static int rg_chunk(int64_t cap) {
  int ch = 8;
  while (ch < 64 && cap / ch > 2048) ch *= 2;
  return ch;
}

extern "C" int64_t hvae_rowgrad_part_floats(int64_t cap, int64_t H) {
  // the apply's chunk partials, the atomic plan's long-segment staging, or the sorted plan's scratch (keys of up
  // to 2^30 items: the largest rocPRIM temporary)
  return std::max<int64_t>({2 * (cap / rg_chunk(cap) + 1) * H, 2 * cap, rgsort_scratch_floats(cap, 1ll << 30)});
}

extern "C" int hvae_w1_rowgrad_apply(const float* da, int64_t H, const hvae_rowgrad* rg, void* stream) {
  HVAE_REQUIRE(da, "hvae_w1_rowgrad_apply: null da");
  if (int rc = rg_check(rg)) return rc;
  if (int rc = check_hidden(H)) return rc;
  HVAE_REQUIRE(rg->contrib_slot && rg->part && rg->part_floats >= hvae_rowgrad_part_floats(rg->cap, H),
               "hvae_w1_rowgrad_apply: part scratch too small for H");
  hipStream_t st = as_stream(stream);
  ProbeScope probe("rowgrad_apply", st);
  double* rowsq = rg->rowsq;
  if (const char* e = ab_getenv("HVAE_ROWSQ")) if (std::atoi(e) == 0) rowsq = nullptr;  // A/B: the clip reads rows
  if (rg->cap <= kPlanSmallCap) {
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(rg->cap, 4), 1024));
    HVAE_NV_DISPATCH(H, (k_rg_apply_seg<NV><<<grid, 256, 0, st>>>(rg->n_unique, rg->seg_off, rg->contrib_row,
                                                                  rg->contrib_val, da, H, rg->rows, rowsq)));
    HVAE_LAUNCH_CHECK("k_rg_apply_seg");
    return HVAE_OK;
  }
  const int ch = rg_chunk(rg->cap);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(cdiv(rg->cap, ch), 4), 4096));
  HVAE_NV_DISPATCH(H, (k_rg_apply<NV><<<grid, 256, 0, st>>>(rg->n_unique, rg->seg_off, rg->contrib_row,
                                                            rg->contrib_val, rg->contrib_slot, da, H, ch, rg->rows,
                                                            rg->part, rg->fill, rowsq)));
  HVAE_LAUNCH_CHECK("k_rg_apply");
  return HVAE_OK;
}

extern "C" int hvae_w1_rowgrad(const hvae_csr_batch* x, const float* da, int64_t H,
                               const hvae_rowgrad* rg, void* ws, size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(x && x->row_ptr && da && rg, "hvae_w1_rowgrad: null arg");
  if (int rc = check_hidden(H)) return rc;
  if (int rc = hvae_w1_rowgrad_plan(x, rg, ws, ws_bytes, stream)) return rc;
  if (x->nb == 0) return HVAE_OK;
  return hvae_w1_rowgrad_apply(da, H, rg, stream);
}

extern "C" int hvae_rowgrad_to_dense(const hvae_rowgrad* rg, int64_t H, float* dense, int64_t ld,
                                     void* stream) {
  HVAE_REQUIRE(rg && dense && ld >= H, "hvae_rowgrad_to_dense: bad args");
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(rg->cap, 2048));
  k_rg_to_dense<<<grid, 256, 0, as_stream(stream)>>>(rg->n_unique, rg->item_of, rg->rows, H, dense, ld);
  HVAE_LAUNCH_CHECK("k_rg_to_dense");
  return HVAE_OK;
}
