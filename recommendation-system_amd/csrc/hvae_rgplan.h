// hvae_rgplan.h -- the W1 row-gradient plan of a small batch as one block's work (shared by k_rg_plan_small in
// hvae_encoder.hip and the extra block of the row-parallel MLP forward in hvae_mlp.hip).
#pragma once

#include "hvae_common.h"

namespace hvae {

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// Whole plan in one block for small batches (rg->cap <= kPlanSmallCap nonzeros): the batch's
// (item, batch row) pairs are gathered into LDS, bitonic-sorted by item then row, and the slots,
// segments and sorted contributions are read off the sorted list -- the same outputs as
// count / scan / scatter / sort, in one launch and without touching the per-item counters.
constexpr int kPlanSmallCap = 4096;
constexpr int kPlanSmallRows = 4096;

// exclusive block scan of v over 1024 threads (result + total)
__device__ __forceinline__ int block_excl_scan_1024(int v, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int incl = wave_incl_scan(v, lane);
  __syncthreads();
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int pre = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k < w) pre += wsum[k];
    total += wsum[k];
  }
  return pre + incl - v;
}

// Run by one block of 1024 threads: k_rg_plan_small, or the extra block of hvae_mlp_fwd_rows' launch. LDS:
// key [kPlanSmallCap], kv [kPlanSmallCap], roff [kPlanSmallRows + 1], rbeg [kPlanSmallRows], wsum [16].
__device__ __forceinline__ void rg_plan_small_block(const int64_t* __restrict__ row_ptr,
                                                    const int32_t* __restrict__ col_idx,
                                                    const float* __restrict__ vals,
                                                    const int32_t* __restrict__ rows,
                                                    const int64_t* __restrict__ rows_offset, int64_t nb,
                                                    int32_t* __restrict__ slot_of, int32_t* __restrict__ item_of,
                                                    int32_t* __restrict__ seg_off, int32_t* __restrict__ contrib_row,
                                                    float* __restrict__ contrib_val,
                                                    int32_t* __restrict__ contrib_slot,
                                                    int32_t* __restrict__ n_unique, unsigned long long* key,
                                                    float* kv, int* roff, int64_t* rbeg, int* wsum) {
  const int tid = threadIdx.x;
  const int nbi = (int)nb;
  // row lengths -> exclusive offsets (4 rows per thread)
  int len4[4], tot4 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = tid * 4 + i;
    len4[i] = 0;
    if (b < nbi) {
      const int64_t r = batch_row(rows, rows_offset, b);
      const int64_t beg = row_ptr[r];
      rbeg[b] = beg;
      len4[i] = (int)(row_ptr[r + 1] - beg);
    }
    tot4 += len4[i];
  }
  int T = 0;
  int o = block_excl_scan_1024(tot4, wsum, T);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = tid * 4 + i;
    if (b < nbi) roff[b] = o;
    o += len4[i];
  }
  if (tid == 0) roff[nbi] = T;
  __syncthreads();
  int P = 64;
  while (P < T) P <<= 1;
  // entries: key = item << 32 | batch row; the row of entry e by binary search in roff
  for (int e = tid; e < P; e += 1024) {
    if (e < T) {
      int lo = 0, hi = nbi - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (roff[mid] <= e) lo = mid; else hi = mid - 1;
      }
      const int64_t src = rbeg[lo] + (e - roff[lo]);
      key[e] = ((unsigned long long)(uint32_t)col_idx[src] << 32) | (uint32_t)lo;
      kv[e] = vals[src];
    } else {
      key[e] = ~0ull;
      kv[e] = 0.f;
    }
  }
  __syncthreads();
  if (P <= 1024) {
    // one element per thread: distances < 64 in registers (wave shuffles), larger ones through LDS
    const int lane = tid & 63;
    unsigned long long a = tid < P ? key[tid] : ~0ull;
    float av = tid < P ? kv[tid] : 0.f;
    for (int k = 2; k <= P; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        unsigned long long b;
        float bv;
        if (j < 64) {
          const uint32_t lo = __shfl_xor((uint32_t)a, j, 64), hi = __shfl_xor((uint32_t)(a >> 32), j, 64);
          b = ((unsigned long long)hi << 32) | lo;
          bv = __shfl_xor(av, j, 64);
        } else {
          __syncthreads();
          key[tid] = a;
          kv[tid] = av;
          __syncthreads();
          b = key[tid ^ j];
          bv = kv[tid ^ j];
        }
        const bool keep_min = ((tid & k) == 0) == ((tid & j) == 0);
        if (keep_min ? (b < a) : (b > a)) { a = b; av = bv; }
      }
    (void)lane;
    __syncthreads();
    if (tid < P) { key[tid] = a; kv[tid] = av; }
    __syncthreads();
  } else
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += 1024) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const unsigned long long a = key[i], c = key[ixj];
          if ((a > c) == up) {
            key[i] = c; key[ixj] = a;
            const float t = kv[i]; kv[i] = kv[ixj]; kv[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  // segment heads -> slots (4 consecutive entries per thread)
  int f4[4], nf = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid * 4 + i;
    f4[i] = (e < T) && (e == 0 || (key[e] >> 32) != (key[e - 1] >> 32));
    nf += f4[i];
  }
  int NU = 0;
  int sl = block_excl_scan_1024(nf, wsum, NU) - 1;  // slot of the entry before this thread's first
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = tid * 4 + i;
    if (e >= T) break;
    sl += f4[i];
    const int item = (int)(key[e] >> 32);
    if (f4[i]) {
      item_of[sl] = item;
      seg_off[sl] = e;
      slot_of[item] = sl;
    }
    contrib_row[e] = (int32_t)(key[e] & 0xffffffffu);
    contrib_val[e] = kv[e];
    contrib_slot[e] = sl;
  }
  if (tid == 0) {
    *n_unique = NU;
    seg_off[NU] = T;
  }
}


// LDS bytes of rg_plan_small_block
constexpr size_t kPlanSmallLds = (size_t)kPlanSmallCap * (8 + 4) + (size_t)(kPlanSmallRows + 1) * 4 +
                                 (size_t)kPlanSmallRows * 8 + 16 * 4;

}  // namespace hvae
