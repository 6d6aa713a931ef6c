// hvae_topk.hip -- fused exact top-K over all items (full-ranking eval, /recommend core; K16 of SURVEY §2.1).
//
// Reference: RecommendationEvaluator.get_user_recommendations (src/ml/evaluate.py:137-147), HybridVAE.recommend
// (src/ml/model.py:236-256) and the /recommend handler (src/api/server.py:115-183) score ALL N items of a user
// in fp32 (u E^T), mask the seen ones to -inf and take np.argsort(scores)[::-1][:top_k]. Here the [R, N] score
// matrix never exists. With K_u = K + |seen_u| (seen items excluded) or K, s the fp32 score, s~ the bf16 MFMA
// score and eps_u >= |s~ - s| for every item of user u:
//
//   k_topk_seed        s~ of a strided sample of <= 4096 items per user (128 tiles of 32), and
//   k_topk_seed_select per user the K_u-th largest sample score r: t = r - eps_u <= T, the K_u-th largest fp32
//                      score over all items (K_u sample items have s >= r - eps_u); t is the user's starting bound;
//   k_topk_scan        one sweep of s~ over E (32 items x 32 users per 32x32x16 chain, E's fragments straight from
//                      global memory, u in registers). An item is a candidate when s~ >= t - eps_u: every true
//                      top-K_u item has s >= T >= t, hence s~ >= t - eps_u, so the candidates are a superset. The
//                      bound tightens during the sweep: a wave keeps, per user, a min-heap (LDS) of its K_u largest
//                      per-tile maxima of s~ (K_u distinct items, so root - eps_u <= T too) and publishes it with an
//                      atomic max per user (a larger t is still a lower bound, and a stale read only loosens the
//                      filter, so no ordering between blocks is needed);
//   k_topk_select      one block per user: exact fp32 rescore of the candidates against fp32 E (the score the
//                      reference ranks), seen items dropped, bitonic sort by (score desc, item desc) -- the order
//                      hvae_topk uses -- and the first K out.
// eps_u = ||u|| max||E|| (2^-7 + 2^-16 + 4 D 2^-24) x 1.02 (bf16 rounding of u and E, each off by up to 2^-8
// relative, so a product by up to 2^-7 + 2^-16; fp32 accumulation on both
// sides). Users whose candidate lists overflow (or that have fewer than K unseen items, or K_u > 256) are flagged
// and left to the caller's exact path.
#include <climits>

#include <cstdlib>

#include "hvae_common.h"

namespace hvae {

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int kTkHeap = 256;    // per-user heap capacity (K_u <= 256)
// LDS heaps of one wave's 32 users sit cap + 1 floats apart, so that the same slot of every user's heap is on a
// different bank (a stride of cap floats put the 32 lanes' root reads on one bank: 32-way conflicts every tile)
constexpr int kTkHeapPad = 1;
constexpr int kTkSegCap = 256;  // candidates per (user, wave instance, lane half)
constexpr int kTkMaxCand = 4096;
constexpr int kTkMaxSeen = 2048;
constexpr int kTkSeedTiles = 128;
constexpr int kTkSeed = kTkSeedTiles * 32;

__device__ __forceinline__ uint32_t tk_pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
// float <-> int with the same order (for atomicMax on signed ints)
__device__ __forceinline__ int tk_ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}
__device__ __forceinline__ float tk_unord(int i) { return __int_as_float(i >= 0 ? i : (i ^ 0x7FFFFFFF)); }

struct TkScanArgs {
  const float* U;
  int64_t ldu;
  const bf16_t* E;         // bf16 [N, D] row-major
  const float* e_maxnorm;  // max_i ||E32_i||
  int64_t R, N;
  const int64_t* ex_row_ptr;  // exclude: CSR of the R users (nullable)
  const int32_t* ex_rows;
  const int64_t* ex_rows_offset;
  int K;
  int splits;
  int64_t tiles_per_split;
  int* g_tau;          // [R] ordered-int lower bound t of the K_u-th fp32 score
  float* g_eps;        // [R] eps_u
  float* seed;         // [R][kTkSeed] sampled bf16 scores
  int32_t* cand;       // [R][nseg][kTkSegCap]
  int32_t* cand_cnt;   // [R][nseg]
  int nseg;            // segments per user: splits * 8 (wave_users 0) or splits * 2 (wave_users 1)
  int wave_users;      // 1: a block's 4 waves take 4 user groups over the same tiles (E read once per block
                       // from L2, the repeats served by the CU's L1); 0: one user group, waves split the tiles
  int tau_mask;        // other waves' bounds are read every tau_mask + 1 tiles (a power of two minus one)
};

__device__ __forceinline__ int tk_ku(const TkScanArgs& a, int64_t r) {
  int ku = a.K;
  if (a.ex_row_ptr) {
    const int64_t m = batch_row(a.ex_rows, a.ex_rows_offset, r);
    ku += (int)(a.ex_row_ptr[m + 1] - a.ex_row_ptr[m]);
  }
  return ku;
}

// One wave's 32 users: u in registers as bf16 MFMA B fragments, in a permuted k order (group g of 64 k's,
// step j, lane half h -> k = 64 g + 32 h + 8 j .. + 7, the same order for E's A fragments, so a lane reads
// 64 contiguous bytes of an E row per group), and S~^T tiles of 32 items.
template <int D>
struct TkScorer {
  static constexpr int NG = D / 64;
  uint4 uf[NG][4];
  float eps;
  int h, col;

  __device__ __forceinline__ void load(const TkScanArgs& a, int64_t user, bool live, int lane) {
    h = lane >> 5;
    col = lane & 31;
    float usq = 0.f;
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f), y = x;
        if (live) {
          const float* p = a.U + user * a.ldu + 64 * g + 32 * h + 8 * j;
          x = *reinterpret_cast<const float4*>(p);
          y = *reinterpret_cast<const float4*>(p + 4);
        }
        usq += (x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w) + (y.x * y.x + y.y * y.y) +
               (y.z * y.z + y.w * y.w);
        uf[g][j] = make_uint4(tk_pack_bf16x2(x.x, x.y), tk_pack_bf16x2(x.z, x.w), tk_pack_bf16x2(y.x, y.y),
                              tk_pack_bf16x2(y.z, y.w));
        __builtin_amdgcn_sched_barrier(0);
      }
    usq += __shfl_xor(usq, 32, 64);
    eps = sqrtf(usq) * (*a.e_maxnorm) * (0x1p-7f + 0x1p-16f + 4.0f * D * 0x1p-24f) * 1.02f;
  }

  // S~^T of tile t: lane (col = user, h) holds items 32 t + (r & 3) + 8 (r >> 2) + 4 h; past N: -inf
  __device__ __forceinline__ f32x16_t score(const TkScanArgs& a, int64_t t) const {
    f32x16_t s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    const int64_t row = min(t * 32 + col, a.N - 1);  // rows past N: clamped, masked below
    const unsigned char* er = reinterpret_cast<const unsigned char*>(a.E) + row * (int64_t)(D * 2) + 64 * h;
    uint4 ea[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) ea[0][j] = *reinterpret_cast<const uint4*>(er + 16 * j);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      if (g + 1 < NG) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ea[(g + 1) & 1][j] = *reinterpret_cast<const uint4*>(er + 128 * (g + 1) + 16 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, ea[g & 1][j]),
                                                   __builtin_bit_cast(bf16x8_t, uf[g][j]), s, 0, 0, 0);
    }
    if (t * 32 + 32 > a.N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h >= a.N) s[r] = -INFINITY;
    }
    return s;
  }
};

// seed pass: s~ of sample tiles j * stride (j < nsample) -> seed[user][32 j + item in tile]; eps_u -> g_eps
template <int D>
__global__ void __launch_bounds__(256) k_topk_seed(TkScanArgs a, int64_t stride, int nsample) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t user = (int64_t)blockIdx.x * 32 + (lane & 31);
  const bool live = user < a.R;
  TkScorer<D> sc;
  sc.load(a, user, live, lane);
  if (live && w == 0 && sc.h == 0) a.g_eps[user] = sc.eps;
  for (int j = w; j < nsample; j += 4) {
    const f32x16_t s = sc.score(a, j * stride);
    if (live) {
#pragma unroll
      for (int r = 0; r < 16; ++r) a.seed[user * kTkSeed + 32 * j + (r & 3) + 8 * (r >> 2) + 4 * sc.h] = s[r];
    }
  }
}

// per user: t = (K_u-th largest sample s~) - eps_u, or the lowest bound when the sample holds fewer than K_u items
__global__ void __launch_bounds__(256) k_topk_seed_select(TkScanArgs a, int nsample) {
  __shared__ float v[kTkSeed];
  const int64_t r = blockIdx.x;
  const int tid = threadIdx.x;
  const int n = nsample * 32;
  const int ku = tk_ku(a, r);
  int P2 = 1;
  while (P2 < n) P2 <<= 1;
  for (int i = tid; i < P2; i += 256) v[i] = i < n ? a.seed[r * kTkSeed + i] : -INFINITY;
  __syncthreads();
  for (int k = 2; k <= P2; k <<= 1)  // bitonic, descending
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P2; i += 256) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const float x = v[i], y = v[p];
          if ((y > x) == up) { v[i] = y; v[p] = x; }
        }
      }
      __syncthreads();
    }
  if (tid == 0) {
    const float kth = ku <= n ? v[ku - 1] : -INFINITY;
    a.g_tau[r] = kth > -INFINITY ? tk_ord(kth - a.g_eps[r]) : INT_MIN;
  }
}

// The per-tile selection of one wave's 32 users (shared by both scans): the heap of per-tile maxima (the pair's
// h == 0 lane), the bound t (own heap root - eps_u, other waves' via the atomic max), candidate emission.
struct TkSelect {
  float* hp;
  int cap, ku, h, sgw;
  int64_t user, seg;
  bool live;
  float eps, tau;
  int cnt = 0;
  __device__ __forceinline__ TkSelect(const TkScanArgs& a, float* heap, int cap_, int64_t user_, bool live_, int h_,
                                      float eps_, int ku_, int sgw_)
      : hp(heap), cap(cap_), ku(ku_ <= cap_ ? ku_ : 0), h(h_), sgw(sgw_), user(user_), live(live_), eps(eps_) {
    if (h == 0)
      for (int i = 0; i < cap; ++i) hp[i] = -INFINITY;
    tau = live ? tk_unord(a.g_tau[user]) : -INFINITY;  // bound t; the filter is s~ >= t - eps_u
    seg = (user * a.nseg + sgw + h) * kTkSegCap;
  }
  __device__ __forceinline__ void consume(const TkScanArgs& a, const f32x16_t& s, int64_t t, int64_t j) {
    float m = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) m = fmaxf(m, s[r]);
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    if (h == 0 && ku > 0 && m > hp[0]) {  // replace the root, sift down
      int i = 0;
      while (true) {
        const int l = 2 * i + 1;
        if (l >= ku) break;
        const int rr = l + 1;
        const int c = (rr < ku && hp[rr] < hp[l]) ? rr : l;
        if (hp[c] >= m) break;
        hp[i] = hp[c];
        i = c;
      }
      hp[i] = m;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the h == 0 lane's writes land before the pair reads
    const float root = ku > 0 ? hp[0] : -INFINITY;
    // a tighter own bound is published without waiting for the atomic's return; other waves' bounds are read
    // every tau_mask + 1 tiles (a returned atomic holds the wave for a device round trip). A stale bound only
    // loosens the filter, so neither needs ordering.
    if (live && root - eps > tau) {
      tau = root - eps;
      __hip_atomic_fetch_max(a.g_tau + user, tk_ord(tau), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (live && (j & a.tau_mask) == a.tau_mask)
      tau = fmaxf(tau, tk_unord(atomicMax(a.g_tau + user, INT_MIN)));  // other waves' bounds
    if (live) {
      const float thr = tau - eps;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (s[r] >= thr) {
          if (cnt < kTkSegCap) a.cand[seg + cnt] = (int32_t)(t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h);
          ++cnt;
        }
    }
  }
};

template <int D>
__global__ void __launch_bounds__(256) k_topk_scan(TkScanArgs a) {
  extern __shared__ float heap_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = blockIdx.x % a.splits;
  const int64_t user = a.wave_users ? (int64_t)(blockIdx.x / a.splits) * 128 + 32 * w + (lane & 31)
                                    : (int64_t)(blockIdx.x / a.splits) * 32 + (lane & 31);
  const bool live = user < a.R;
  const int64_t ntiles = (a.N + 31) / 32;
  const int64_t t0 = (int64_t)split * a.tiles_per_split;
  const int64_t t1 = min(ntiles, t0 + a.tiles_per_split);
  // this wave's tiles: t0 + tw, t0 + tw + ts, ... (every tile of the split with wave_users)
  const int tw = a.wave_users ? 0 : w, ts = a.wave_users ? 1 : 4;
  const int64_t nw = t1 > t0 + tw ? (t1 - t0 - tw + ts - 1) / ts : 0;
  const int sgw = a.wave_users ? split * 2 : (split * 4 + w) * 2;  // the wave's first segment of the user
  TkScorer<D> sc;
  sc.load(a, user, live, lane);
  const int h = sc.h;
  const int ku = live ? min(tk_ku(a, user), kTkHeap) : 0;  // K_u > kTkHeap: flagged by k_topk_select
  const float eps = sc.eps;

  TkSelect sel(a, heap_lds + (size_t)(w * 32 + (lane & 31)) * (kTkHeap + kTkHeapPad), kTkHeap, user, live, h, eps, ku,
               sgw);
  for (int64_t j = 0; j < nw; ++j) {
    const int64_t t = t0 + tw + ts * j;
    sel.consume(a, sc.score(a, t), t, j);
  }
  const int cnt = sel.cnt;
  if (live) a.cand_cnt[user * a.nseg + sgw + h] = cnt;
}


// ---- LDS-staged scan (D a multiple of 128): a block's 4 waves take 4 groups of 32 users over the same tiles;
// each 32-item E tile arrives once per block by LDS-DMA (three-slot ring, the decoder's image and piece map,
// one barrier per tile) and the 32x32x16 A operands are ds_read_b128 row reads of it. Per-user heaps of up to
// tkl_heap - 1 tile maxima (a user with K_u beyond it keeps the seed / other waves' bound, which is still valid).
// ring slots and heap capacity per D (LDS: slots x the tile + 4 waves x 32 users x the heap): d = 768 keeps two
// slots (the next tile's DMA overlaps the current tile's MFMAs) so that K_u up to 64 keeps its heap
template <int D>
constexpr int tkl_ns() { return D >= 768 ? 2 : 3; }
template <int D>
constexpr int tkl_heap() { return D >= 768 ? 64 : 128; }
template <int D>
constexpr int tkl_lds_bytes() { return tkl_ns<D>() * ((D / 128) * 8192) + 4 * 32 * tkl_heap<D>() * 4; }

__device__ __forceinline__ uint32_t tk_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
template <int n>
__device__ __forceinline__ void tk_wait_vmcnt() {
  static_assert(n >= 0 && n < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14));
}

template <int D>
__global__ void __launch_bounds__(256) k_topk_scan_lds(TkScanArgs a) {
  constexpr int NSEG = D / 128, TB = NSEG * 8192, PW = NSEG * 8 / 4, NS = tkl_ns<D>(), KS = D / 16;
  constexpr int HC = tkl_heap<D>() - 1;  // heap capacity = stride: odd, so the 32 users' slots fall on 32 banks
  static_assert(D % 128 == 0 && tkl_lds_bytes<D>() <= 160 * 1024, "k_topk_scan_lds shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  float* heaps = reinterpret_cast<float*>(lds + NS * TB);
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = blockIdx.x % a.splits;
  const int64_t user = (int64_t)(blockIdx.x / a.splits) * 128 + 32 * w + col;
  const bool live = user < a.R;
  const int64_t ntiles = (a.N + 31) / 32;
  const int64_t t0 = (int64_t)split * a.tiles_per_split;
  const int64_t t1 = min(ntiles, t0 + a.tiles_per_split);
  const int64_t nt = t1 > t0 ? t1 - t0 : 0;
  const float emax = *a.e_maxnorm;  // before any LDS-DMA is in flight

  // u as the B operand: lane holds U[user][16 ks + 8 h .. + 7]
  uint4 uf[KS];
  float usq = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f), y = x;
    if (live) {
      x = *reinterpret_cast<const float4*>(a.U + user * a.ldu + 16 * ks + 8 * h);
      y = *reinterpret_cast<const float4*>(a.U + user * a.ldu + 16 * ks + 8 * h + 4);
    }
    usq += (x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w) + (y.x * y.x + y.y * y.y) + (y.z * y.z + y.w * y.w);
    uf[ks] = make_uint4(tk_pack_bf16x2(x.x, x.y), tk_pack_bf16x2(x.z, x.w), tk_pack_bf16x2(y.x, y.y),
                        tk_pack_bf16x2(y.z, y.w));
    __builtin_amdgcn_sched_barrier(0);  // a few k-steps' loads in flight, not all (register peak)
  }
  usq += __shfl_xor(usq, 32, 64);
  const float eps = sqrtf(usq) * emax * (0x1p-7f + 0x1p-16f + 4.0f * D * 0x1p-24f) * 1.02f;
  const int ku = live ? tk_ku(a, user) : 0;

  // LDS-DMA (the decoder's version-2 image: 8-row x 32-column subtiles, 2-bit chunk XOR)
  int vlane[2];
#pragma unroll
  for (int pb = 0; pb < 2; ++pb) {
    const int row = 8 * pb + ((lane >> 2) & 7);
    vlane[pb] = ((lane >> 2) & 7) * (D * 2) + 64 * (lane >> 5) + 16 * ((lane & 3) ^ ((row >> 2) & 3));
  }
  // the resource covers this split's items only (its extent is a 32-bit byte count: a whole E of more than
  // 2^31 bytes would wrap, and the bounds check would then read real items as zeros); tile offsets are split-relative
  const int64_t i_end = min(a.N, t1 * 32);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(a.E) + t0 * 32 * D, (short)0, (int)(i_end > t0 * 32 ? (i_end - t0 * 32) * D * 2 : 0),
      0x00020000);
  const uint32_t ring0 = tk_lds_addr(lds) + (uint32_t)(w * PW * 1024);
  auto issue_pieces = [&](uint32_t soff, int slot_i, int i0, int i1, bool fresh) {
    const uint32_t lb = ring0 + (uint32_t)(slot_i * TB);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int p = w * PW + i;  // wave-uniform; PW need not be a multiple of 4 here, so p's own bits
      const uint32_t so = soff + (uint32_t)(8 * ((p >> 1) & 3) * (D * 2) + 256 * (p >> 3) + 128 * (p & 1));
      const int vo = ((p >> 1) & 1) ? vlane[1] : vlane[0];
      if (fresh && i == i0)
        asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                     :: "s"(lb + (uint32_t)(i * 1024)), "v"(vo), "s"(rsrc), "s"(so) : "memory");
    }
  };
  auto tile_soff = [&](int64_t t) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)((t - t0) * (int64_t)(32 * D * 2)));
  };
  auto barrier = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int laneA0 = ((col >> 3) << 11) + ((col & 7) << 6) + (((0 + h) ^ ((col >> 2) & 3)) << 4);
  const int laneA1 = ((col >> 3) << 11) + ((col & 7) << 6) + (((2 + h) ^ ((col >> 2) & 3)) << 4);

  TkSelect sel(a, heaps + (w * 32 + col) * HC, HC, user, live, h, eps, ku, split * 2);
  if (nt > 0) {
    issue_pieces(tile_soff(t0), 0, 0, PW, true);
    if (NS == 3) issue_pieces(tile_soff(min(t0 + 1, t1 - 1)), 1, 0, PW, true);
  }
  for (int64_t j = 0; j < nt; ++j) {
    const int64_t t = t0 + j;
    const int cur = (int)(j % NS), s_dma = (int)((j + NS - 1) % NS);
    // tile t has landed (three slots: issued two iterations back, younger ops may stay in flight; two slots:
    // issued in the previous iteration, so everything is waited for)
    if constexpr (NS == 3) tk_wait_vmcnt<PW>();
    else tk_wait_vmcnt<0>();
    barrier();  // every wave's pieces of t; every wave is done with the slot the next DMA reuses
    const uint32_t soff_dma = tile_soff(min(t + NS - 1, t1 - 1));
    const unsigned char* b0 = lds + cur * TB + laneA0;
    const unsigned char* b1 = lds + cur * TB + laneA1;
    auto rdA = [&](int ks) {
      const int grp = ks >> 1;
      return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(((ks & 1) ? b1 : b0) + ((grp >> 2) << 13) +
                                                                          ((grp & 3) << 9)));
    };
    f32x16_t s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    bf16x8_t an[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) an[q] = rdA(q);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16x8_t c = an[ks & 3];
      if (ks + 4 < KS) an[ks & 3] = rdA(ks + 4);
      s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c, __builtin_bit_cast(bf16x8_t, uf[ks]), s, 0, 0, 0);
      if ((ks & 1) == 1 && (ks >> 1) < PW) issue_pieces(soff_dma, s_dma, ks >> 1, (ks >> 1) + 1, ks == 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (KS / 2 < PW) issue_pieces(soff_dma, s_dma, KS / 2, PW, false);
    if (t * 32 + 32 > a.N) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h >= a.N) s[r] = -INFINITY;
    }
    sel.consume(a, s, t, j);
  }
  tk_wait_vmcnt<0>();  // the LDS-DMA lands before the block's LDS is released
  if (live) a.cand_cnt[user * a.nseg + split * 2 + h] = sel.cnt;
}

// (score desc, item desc): a before b
__device__ __forceinline__ bool tk_before(float sa, int ia, float sb, int ib) {
  return sa > sb || (sa == sb && ia > ib);
}

struct TkSelArgs {
  const float* U;
  int64_t ldu;
  const float* E32;
  int64_t R, N, D;
  const int64_t* ex_row_ptr;
  const int32_t* ex_col;
  const int32_t* ex_rows;
  const int64_t* ex_rows_offset;
  int K;
  const int32_t* cand;
  const int32_t* cand_cnt;
  int nseg;
  int32_t* idx;  // [R, K]
  float* val;    // [R, K] (nullable)
  int32_t* flag; // [R]
};

template <int NK>  // D / 64
__global__ void __launch_bounds__(256) k_topk_select(TkSelArgs a) {
  __shared__ float ss[kTkMaxCand];
  __shared__ int si[kTkMaxCand];
  __shared__ int seen[kTkMaxSeen];
  __shared__ int s_off[1025];
  __shared__ int s_bad;
  const int64_t r = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int nseen = 0;
  int64_t m = 0;
  if (a.ex_row_ptr) {
    m = batch_row(a.ex_rows, a.ex_rows_offset, r);
    nseen = (int)(a.ex_row_ptr[m + 1] - a.ex_row_ptr[m]);
  }
  // candidate offsets per segment (nseg <= 1024)
  if (tid == 0) {
    int tot = 0, bad = 0;
    for (int sgi = 0; sgi < a.nseg; ++sgi) {
      const int c = a.cand_cnt[r * a.nseg + sgi];
      bad |= c > kTkSegCap;
      s_off[sgi] = tot;
      tot += min(c, kTkSegCap);
    }
    s_off[a.nseg] = tot;
    bad |= tot > kTkMaxCand || nseen > kTkMaxSeen || a.K + nseen > kTkHeap || tot < a.K;
    s_bad = bad;
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) a.flag[r] = 1;
    return;
  }
  const int C = s_off[a.nseg];
  // seen items, sorted ascending (bitonic over the next power of two)
  int P2s = 1;
  while (P2s < nseen) P2s <<= 1;
  for (int i = tid; i < P2s; i += 256) seen[i] = i < nseen ? a.ex_col[a.ex_row_ptr[m] + i] : INT_MAX;
  __syncthreads();
  for (int k = 2; k <= P2s; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P2s; i += 256) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const int x = seen[i], y = seen[p];
          if ((x > y) == up) { seen[i] = y; seen[p] = x; }
        }
      }
      __syncthreads();
    }
  // gather the candidates
  for (int sgi = 0; sgi < a.nseg; ++sgi) {
    const int o = s_off[sgi], n = s_off[sgi + 1] - o;
    for (int i = tid; i < n; i += 256) si[o + i] = a.cand[(r * a.nseg + sgi) * kTkSegCap + i];
  }
  __syncthreads();
  // exact fp32 rescore: 16 lanes per candidate, 4 candidates per wave pass; lane g of a group owns float4
  // columns g + 16 k (k < NK) of u (in registers) and of the candidate's E row, all NK loads in flight; the sum
  // is over k in order, then a fixed xor tree over the group (deterministic)
  const float* u = a.U + r * a.ldu;
  const int g = lane & 15, slot = lane >> 4;
  float4 u4[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) u4[k] = *reinterpret_cast<const float4*>(u + 4 * (g + 16 * k));
  for (int c0 = w * 4; c0 < C; c0 += 16) {
    const int c = c0 + slot;
    const int it = c < C ? si[c] : 0;
    const float4* e = reinterpret_cast<const float4*>(a.E32 + (int64_t)it * (16 * 4 * NK));
    float4 e4[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) e4[k] = e[g + 16 * k];
    float sdot = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k)
      sdot += (u4[k].x * e4[k].x + u4[k].y * e4[k].y) + (u4[k].z * e4[k].z + u4[k].w * e4[k].w);
    sdot += __shfl_xor(sdot, 8, 64);
    sdot += __shfl_xor(sdot, 4, 64);
    sdot += __shfl_xor(sdot, 2, 64);
    sdot += __shfl_xor(sdot, 1, 64);
    if (g == 0 && c < C) {
      int lo = 0, hi = nseen;  // binary search in the sorted seen list
      while (lo < hi) {
        const int md = (lo + hi) >> 1;
        if (seen[md] < it) lo = md + 1;
        else hi = md;
      }
      const bool is_seen = lo < nseen && seen[lo] == it;
      ss[c] = (is_seen || sdot != sdot) ? -INFINITY : sdot;
    }
  }
  __syncthreads();
  int P2 = 1;
  while (P2 < C) P2 <<= 1;
  for (int i = C + tid; i < P2; i += 256) { ss[i] = -INFINITY; si[i] = -1; }
  __syncthreads();
  // bitonic sort, "before" first
  for (int k = 2; k <= P2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P2; i += 256) {
        const int p = i ^ j;
        if (p > i) {
          const bool up = (i & k) == 0;
          const float x = ss[i], y = ss[p];
          const int xi = si[i], yi = si[p];
          if (tk_before(y, yi, x, xi) == up) { ss[i] = y; si[i] = yi; ss[p] = x; si[p] = xi; }
        }
      }
      __syncthreads();
    }
  // fewer than K finite candidates (seen items ate the shortlist): the exact path decides
  if (tid == 0) a.flag[r] = !(ss[a.K - 1] > -INFINITY);
  for (int i = tid; i < a.K; i += 256) {
    a.idx[r * a.K + i] = si[i];
    if (a.val) a.val[r * a.K + i] = ss[i];
  }
}

static int tk_lds_scan(int64_t D) {  // HVAE_TOPK_LDS=0 keeps the global-load scan (A/B)
  const char* v = ab_getenv("HVAE_TOPK_LDS");
  return D % 128 == 0 && ((v && *v) ? (atoi(v) != 0) : 1);
}

static int tk_wave_users() {  // HVAE_TOPK_WAVE_USERS=0 selects the tile-split mapping (A/B)
  const char* v = ab_getenv("HVAE_TOPK_WAVE_USERS");
  return (v && *v) ? (atoi(v) != 0) : 1;
}

// a split's bf16 slice of E must stay below 2^31 bytes (the LDS scan's buffer resource extent is 32-bit)
constexpr int64_t kTkSplitBytes = (int64_t)1 << 30;

static int tk_splits(int64_t R, int64_t N, int64_t D, int wave_users) {
  const int64_t groups = std::max<int64_t>(1, cdiv(R, wave_users ? 128 : 32));  // R = 0: a workspace query
  const int64_t tiles = cdiv(N, 32);
  int64_t s = std::max<int64_t>(1, cdiv(256, groups));  // ~256 blocks (one per CU: 128 KiB of heaps each)
  s = std::min<int64_t>(s, std::max<int64_t>(1, tiles / (wave_users ? 4 : 16)));  // >= 4 tiles per wave
  s = std::max<int64_t>(s, cdiv(tiles * 32 * D * 2, kTkSplitBytes));  // large E: enough splits for the extent
  s = std::min<int64_t>(s, wave_users ? 512 : 128);  // nseg <= 1024
  return (int)s;
}

}  // namespace hvae

using namespace hvae;

extern "C" size_t hvae_topk_fused_workspace(int64_t R, int64_t N, int64_t D, int64_t K) {
  const int wu = tk_lds_scan(D) ? 1 : tk_wave_users();
  const int s = tk_splits(R, N, D, wu);
  const size_t nseg = (size_t)s * (wu ? 2 : 8);
  return 256 + (size_t)R * 8 + (size_t)R * nseg * 4 + (size_t)R * nseg * kTkSegCap * 4 + (size_t)R * kTkSeed * 4;
}

// HVAE_TK_TAU_PERIOD (A/B, read at every call; a power of two): tiles between reads of the other waves' bounds
static int tk_tau_mask() {
  const char* e = ab_getenv("HVAE_TK_TAU_PERIOD");
  int p = e ? std::atoi(e) : 8;
  if (p < 1 || (p & (p - 1)) != 0) p = 8;
  return p - 1;
}

extern "C" int hvae_topk_fused(const float* U, int64_t ldu, const void* E_bf16, const float* E32,
                               const float* e32_maxnorm, int64_t N, int64_t D, const hvae_csr_batch* exclude,
                               int64_t R, int64_t K, int32_t* idx, float* val, int32_t* flag, void* ws,
                               size_t ws_bytes, void* stream) {
  HVAE_REQUIRE(R >= 0 && ldu >= D && K > 0 && K <= kTkHeap && K <= N && N < INT32_MAX, "hvae_topk_fused: bad args");
  HVAE_REQUIRE(D == 64 || D == 128 || D == 256 || D == 384 || D == 512 || D == 768,
               "hvae_topk_fused: D must be 64, 128, 256, 384, 512 or 768");
  if (R == 0) return HVAE_OK;  // an empty batch: its (empty) output tensors may have null data pointers
  HVAE_REQUIRE(U && E_bf16 && E32 && e32_maxnorm && idx && flag, "hvae_topk_fused: null pointer");
  HVAE_REQUIRE(ws && ws_bytes >= hvae_topk_fused_workspace(R, N, D, K), "hvae_topk_fused: workspace too small");
  if (exclude)
    HVAE_REQUIRE(exclude->row_ptr && exclude->col_idx && exclude->nb == R, "hvae_topk_fused: bad exclude");
  hipStream_t st = as_stream(stream);
  const bool lds_scan = tk_lds_scan(D);
  const int wu = lds_scan ? 1 : tk_wave_users();
  const int splits = tk_splits(R, N, D, wu);
  const int nseg = splits * (wu ? 2 : 8);
  HVAE_REQUIRE(!lds_scan || cdiv(cdiv(N, 32), splits) * 32 * D * 2 < ((int64_t)1 << 31),
               "hvae_topk_fused: a split of E exceeds 2^31 bytes");
  unsigned char* p = static_cast<unsigned char*>(ws);
  int* g_tau = reinterpret_cast<int*>(p + 256);
  float* g_eps = reinterpret_cast<float*>(g_tau + R);
  int32_t* cnt = reinterpret_cast<int32_t*>(g_eps + R);
  int32_t* cand = cnt + (size_t)R * nseg;
  float* seed = reinterpret_cast<float*>(cand + (size_t)R * nseg * kTkSegCap);
  HVAE_HIP(hipMemsetAsync(cnt, 0, (size_t)R * nseg * 4, st));
  HVAE_HIP(hipMemsetAsync(flag, 0, (size_t)R * 4, st));
  TkScanArgs sa{U, ldu, static_cast<const bf16_t*>(E_bf16), e32_maxnorm, R, N,
                exclude ? exclude->row_ptr : nullptr, exclude ? exclude->rows : nullptr,
                exclude ? exclude->rows_offset : nullptr, (int)K, splits, cdiv(cdiv(N, 32), splits), g_tau, g_eps,
                seed, cand, cnt, nseg, wu, tk_tau_mask()};
  const int64_t ntiles = cdiv(N, 32);
  const int nsample = (int)std::min<int64_t>(ntiles, kTkSeedTiles);
  const int64_t stride = std::max<int64_t>(1, ntiles / nsample);
  const unsigned groups = (unsigned)cdiv(R, 32);  // the seed pass: one block per 32 users
  const unsigned blocks = (unsigned)(cdiv(R, wu ? 128 : 32) * splits);
  const size_t lds = (size_t)4 * 32 * (kTkHeap + kTkHeapPad) * 4;
#define TK_SCAN_LDS(DD)                                                                                 \
  {                                                                                                       \
    constexpr int DL = DD % 128 == 0 ? DD : 128;                                                          \
    HVAE_HIP(hipFuncSetAttribute((const void*)k_topk_scan_lds<DL>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                 tkl_lds_bytes<DL>()));                                                   \
    k_topk_scan_lds<DL><<<blocks, 256, tkl_lds_bytes<DL>(), st>>>(sa);                                   \
  }
  switch (D) {
#define TK_CASE(DD)                                                                                       \
  case DD:                                                                                                \
    k_topk_seed<DD><<<groups, 256, 0, st>>>(sa, stride, nsample);                                        \
    HVAE_LAUNCH_CHECK("k_topk_seed");                                                                     \
    k_topk_seed_select<<<(unsigned)R, 256, 0, st>>>(sa, nsample);                                         \
    HVAE_LAUNCH_CHECK("k_topk_seed_select");                                                              \
    if (DD % 128 == 0 && lds_scan) {                                                                      \
      TK_SCAN_LDS(DD)                                                                                     \
    } else {                                                                                              \
      HVAE_HIP(hipFuncSetAttribute((const void*)k_topk_scan<DD>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                   (int)lds));                                                            \
      k_topk_scan<DD><<<blocks, 256, lds, st>>>(sa);                                                      \
    }                                                                                                     \
    HVAE_LAUNCH_CHECK("k_topk_scan");                                                                     \
    break;
    TK_CASE(64) TK_CASE(128) TK_CASE(256) TK_CASE(384) TK_CASE(512) TK_CASE(768)
#undef TK_CASE
#undef TK_SCAN_LDS
  }
  TkSelArgs la{U, ldu, E32, R, N, D, exclude ? exclude->row_ptr : nullptr, exclude ? exclude->col_idx : nullptr,
               exclude ? exclude->rows : nullptr, exclude ? exclude->rows_offset : nullptr, (int)K, cand, cnt, nseg,
               idx, val, flag};
  switch (D) {
    case 64: k_topk_select<1><<<(unsigned)R, 256, 0, st>>>(la); break;
    case 128: k_topk_select<2><<<(unsigned)R, 256, 0, st>>>(la); break;
    case 256: k_topk_select<4><<<(unsigned)R, 256, 0, st>>>(la); break;
    case 384: k_topk_select<6><<<(unsigned)R, 256, 0, st>>>(la); break;
    case 512: k_topk_select<8><<<(unsigned)R, 256, 0, st>>>(la); break;
    default: k_topk_select<12><<<(unsigned)R, 256, 0, st>>>(la); break;
  }
  HVAE_LAUNCH_CHECK("k_topk_select");
  return HVAE_OK;
}
