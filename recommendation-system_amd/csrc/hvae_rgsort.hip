// hvae_rgsort.hip -- the W1 row-gradient plan by one stable radix sort (rocPRIM) instead of per-item atomics.
//
// The plan (hvae_w1_rowgrad_plan, hvae_encoder.hip) turns a batch's CSR entries into per-item segments of
// contributions sorted by batch row: item_of / seg_off / slot_of / n_unique, and contrib_row / contrib_val /
// contrib_slot in (item, batch row) order. The atomic plan (count, look-back scan, scatter, per-segment sort)
// serialises on the popular items' counters: a Zipf catalogue puts thousands of a batch's entries on one item,
// and the data-parallel union batch (W x B rows) multiplies that by W (plan + apply 181 us at W = 1, 1,181 us at
// W = 8 at the Syn-10M shard, profiles/r02_union_rowgrad_cost.jsonl). Here:
//   1. the batch rows' entry offsets (one-block scan of the row lengths);
//   2. one wave per batch row writes key = item, value = entry position p (entries in batch-row order), and
//      the entry's batch row and value beside p; positions past the batch's total get the key N (sorts last);
//   3. rocprim::radix_sort_pairs over the key bits of N: stable, so each item's entries stay in ascending batch
//      row -- the order the atomic plan's segment sort produces;
//   4. segment heads (key changes) and their inclusive scan give each entry its slot;
//   5. one pass writes contrib_row / contrib_val / contrib_slot, and at each head item_of, seg_off, slot_of;
//      the last entry writes n_unique and seg_off[n_unique].
// The outputs equal the atomic plan's bitwise (tests/test_gpu_kernels.py compares them), so the apply and the
// lazy Adam downstream are unchanged. Scratch: the rowgrad's `part` buffer (the apply's chunk partials, free
// while the plan runs), sized by hvae_rowgrad_part_floats.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "hvae_common.h"

namespace hvae {

static int key_bits(int64_t N) {
  int b = 1;
  while ((1ll << b) <= N) ++b;  // keys 0 .. N (N = the padding key)
  return b;
}

// scratch layout (uint32 words) for a plan of capacity cap over at most nb_max batch rows
struct RgSortLayout {
  size_t pfx, keys, perm, row_of, val_of, keys_s, perm_s, head, segid, temp, total_words;
  size_t temp_bytes;
};

static RgSortLayout rgsort_layout(int64_t cap, int64_t N) {
  RgSortLayout L{};
  const size_t c = (size_t)cap;
  auto al = [](size_t w) { return (w + 63) / 64 * 64; };  // 256-B aligned regions
  size_t o = 0;
  L.pfx = o; o += al(c + 1);  // batch rows <= cap + 1 (checked at the call)
  L.keys = o; o += al(c);
  L.perm = o; o += al(c);
  L.row_of = o; o += al(c);
  L.val_of = o; o += al(c);
  L.keys_s = o; o += al(c);
  L.perm_s = o; o += al(c);
  L.head = o; o += al(c);
  L.segid = o; o += al(c);
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (const unsigned*)nullptr, (unsigned*)nullptr,
                            (const unsigned*)nullptr, (unsigned*)nullptr, (unsigned)c, 0, key_bits(N));
  (void)rocprim::inclusive_scan(nullptr, scan_bytes, (const unsigned*)nullptr, (unsigned*)nullptr, (unsigned)c,
                          rocprim::plus<unsigned>());
  L.temp_bytes = std::max(sort_bytes, scan_bytes);
  L.temp = o; o += al((L.temp_bytes + 3) / 4);
  L.total_words = o;
  return L;
}

// 1. exclusive prefix of the batch rows' entry counts (one block; nb <= cap + 1)
__global__ void __launch_bounds__(1024) k_rgs_rowscan(const int64_t* __restrict__ row_ptr,
                                                      const int32_t* __restrict__ rows,
                                                      const int64_t* __restrict__ rows_offset, int64_t nb,
                                                      uint32_t* __restrict__ pfx) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t b = base + tid;
    uint32_t len = 0;
    if (b < nb) {
      const int64_t r = batch_row(rows, rows_offset, b);
      len = (uint32_t)(row_ptr[r + 1] - row_ptr[r]);
    }
    uint32_t incl = len;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t wb = 0;
    for (int q = 0; q < w; ++q) wb += wsum[q];
    const uint32_t c0 = carry;
    if (b < nb) pfx[b] = c0 + wb + incl - len;
    __syncthreads();
    if (tid == 1023) carry = c0 + wb + incl;
    __syncthreads();
  }
  if (tid == 0) pfx[nb] = carry;
}

// 2. keys / values in batch-row order; padding keys past the total
__global__ void __launch_bounds__(256) k_rgs_fill(const int64_t* __restrict__ row_ptr,
                                                  const int32_t* __restrict__ col_idx,
                                                  const float* __restrict__ vals, const int32_t* __restrict__ rows,
                                                  const int64_t* __restrict__ rows_offset, int64_t nb,
                                                  const uint32_t* __restrict__ pfx, int64_t cap, uint32_t pad_key,
                                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ perm,
                                                  uint32_t* __restrict__ row_of, float* __restrict__ val_of) {
  const uint32_t total = min((int64_t)pfx[nb], cap);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    perm[i] = (uint32_t)i;
    if (i >= total) keys[i] = pad_key;
  }
  const int lane = threadIdx.x & 63;
  for (int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); b < nb; b += (int64_t)gridDim.x * 4) {
    const int64_t r = batch_row(rows, rows_offset, b);
    const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
    const uint32_t p0 = pfx[b];
    for (int64_t e = beg + lane; e < end; e += 64) {
      const int64_t p = (int64_t)p0 + (e - beg);
      if (p >= cap) break;
      keys[p] = (uint32_t)col_idx[e];
      row_of[p] = (uint32_t)b;
      val_of[p] = vals[e];
    }
  }
}

// 4a. segment heads of the sorted keys (padding entries are no heads)
__global__ void __launch_bounds__(256) k_rgs_heads(const uint32_t* __restrict__ keys_s, const uint32_t* __restrict__ pfx,
                                                   int64_t nb, int64_t cap, uint32_t* __restrict__ head) {
  const int64_t total = min((int64_t)pfx[nb], cap);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i < total && (i == 0 || keys_s[i] != keys_s[i - 1])) ? 1u : 0u;
}

// 5. the plan's outputs
__global__ void __launch_bounds__(256) k_rgs_emit(const uint32_t* __restrict__ keys_s,
                                                  const uint32_t* __restrict__ perm_s,
                                                  const uint32_t* __restrict__ segid, const uint32_t* __restrict__ pfx,
                                                  int64_t nb, int64_t cap, const uint32_t* __restrict__ row_of,
                                                  const float* __restrict__ val_of, int32_t* __restrict__ slot_of,
                                                  int32_t* __restrict__ item_of, int32_t* __restrict__ seg_off,
                                                  int32_t* __restrict__ contrib_row, float* __restrict__ contrib_val,
                                                  int32_t* __restrict__ contrib_slot, int32_t* __restrict__ n_unique) {
  const int64_t total = min((int64_t)pfx[nb], cap);
  if (total == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *n_unique = 0;
      seg_off[0] = 0;
    }
    return;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t sg = segid[i];  // inclusive count of heads: the slot is sg - 1
    const int32_t s = (int32_t)sg - 1;
    const uint32_t p = perm_s[i];
    contrib_slot[i] = s;
    contrib_row[i] = (int32_t)row_of[p];
    contrib_val[i] = val_of[p];
    const uint32_t key = keys_s[i];
    if (i == 0 || keys_s[i - 1] != key) {
      item_of[s] = (int32_t)key;
      seg_off[s] = (int32_t)i;
      slot_of[key] = s;
    }
    if (i == total - 1) {
      *n_unique = (int32_t)sg;
      seg_off[sg] = (int32_t)total;
    }
  }
}

int64_t rgsort_scratch_floats(int64_t cap, int64_t N) { return (int64_t)rgsort_layout(cap, N).total_words; }

// the sorted plan; returns HVAE_ERR_UNSUPPORTED (nothing launched) when the scratch cannot hold it, so the caller
// runs the atomic plan instead
int rg_plan_sorted(const hvae_csr_batch* x, const hvae_rowgrad* rg, hipStream_t st) {
  const int64_t N = x->n_items, cap = rg->cap, nb = x->nb;
  if (nb + 1 > cap + 1 || cap >= (1ll << 31) || N >= (1ll << 31) - 1 || !rg->part) return HVAE_ERR_UNSUPPORTED;
  const RgSortLayout L = rgsort_layout(cap, N);
  if ((int64_t)L.total_words > rg->part_floats) return HVAE_ERR_UNSUPPORTED;
  uint32_t* w = reinterpret_cast<uint32_t*>(rg->part);
  uint32_t *pfx = w + L.pfx, *keys = w + L.keys, *perm = w + L.perm, *row_of = w + L.row_of;
  float* val_of = reinterpret_cast<float*>(w + L.val_of);
  uint32_t *keys_s = w + L.keys_s, *perm_s = w + L.perm_s, *head = w + L.head, *segid = w + L.segid;
  void* temp = w + L.temp;
  ProbeScope probe("rowgrad_plan", st);
  k_rgs_rowscan<<<1, 1024, 0, st>>>(x->row_ptr, x->rows, x->rows_offset, nb, pfx);
  HVAE_LAUNCH_CHECK("k_rgs_rowscan");
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(std::max(cap, nb * 4), 256), 4096));
  k_rgs_fill<<<g, 256, 0, st>>>(x->row_ptr, x->col_idx, x->vals, x->rows, x->rows_offset, nb, pfx, cap,
                                (uint32_t)N, keys, perm, row_of, val_of);
  HVAE_LAUNCH_CHECK("k_rgs_fill");
  size_t tb = L.temp_bytes;
  if (rocprim::radix_sort_pairs(temp, tb, keys, keys_s, perm, perm_s, (unsigned)cap, 0, key_bits(N), st) !=
      hipSuccess)
    HVAE_FAIL(HVAE_ERR_HIP, "hvae_w1_rowgrad_plan: radix sort failed");
  k_rgs_heads<<<g, 256, 0, st>>>(keys_s, pfx, nb, cap, head);
  HVAE_LAUNCH_CHECK("k_rgs_heads");
  tb = L.temp_bytes;
  if (rocprim::inclusive_scan(temp, tb, head, segid, (unsigned)cap, rocprim::plus<unsigned>(), st) != hipSuccess)
    HVAE_FAIL(HVAE_ERR_HIP, "hvae_w1_rowgrad_plan: segment scan failed");
  k_rgs_emit<<<g, 256, 0, st>>>(keys_s, perm_s, segid, pfx, nb, cap, row_of, val_of, rg->slot_of, rg->item_of,
                                rg->seg_off, rg->contrib_row, rg->contrib_val, rg->contrib_slot, rg->n_unique);
  HVAE_LAUNCH_CHECK("k_rgs_emit");
  return HVAE_OK;
}

}  // namespace hvae
