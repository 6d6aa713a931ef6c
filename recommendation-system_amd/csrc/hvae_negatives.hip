// hvae_negatives.hip -- the 99-negative protocol's sampler, on the host, draw for draw the reference's.
//
// RecommendationEvaluator.evaluate_user_with_negatives (src/ml/evaluate.py:149-185) draws, per test row,
//   available = np.where(mask)[0]   (items neither seen by the user in training nor the test item, ascending)
//   negatives = available if len(available) < n else np.random.choice(available, n, replace=False)
// from numpy's global legacy RandomState. Legacy choice without p and without replacement is
// permutation(len(available))[:n] (numpy/random/mtrand.pyx, RandomState.choice), and permutation(k) is a
// Fisher-Yates shuffle of arange(k): for i = k - 1 .. 1, j = random_interval(i), swap (mtrand.pyx
// _shuffle_raw); random_interval(max) masks 32-bit MT19937 outputs down to the smallest 2^b - 1 >= max and
// rejects values above max (numpy/random/src/distributions/distributions.c). Every row therefore consumes
// ~1.3 len(available) outputs of the one global stream, in row order, which is what makes the reference's
// evaluation host-bound (one Python-level choice per row). Here the same stream runs in C++ over all rows at
// once: the caller passes numpy's MT19937 state (np.random.get_state(): 624 key words and the position) and
// gets it back advanced exactly as the per-row choices would have left it, so the negatives -- and every
// later draw of the process -- are the reference's. tests/test_negatives_cpu.py checks both against numpy.
// Host code only: the device pass of this translation unit compiles nothing.
#ifndef __HIP_DEVICE_COMPILE__
#include <immintrin.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "hvae_common.h"

// The row's draw loop and the generator have an AVX-512 form (both the GPU box's EPYC and this image's build
// host have it), picked at run time; every other x86-64 runs the scalar form. HVAE_NEG_SCALAR=1 forces the
// scalar form (the tests run both).
#define HVAE_AVX512 __attribute__((target("avx512f,avx512vl,popcnt")))
#define HVAE_INLINE inline __attribute__((always_inline))

namespace {

constexpr int kMtN = 624, kMtM = 397;
constexpr uint32_t kMtA = 0x9908b0dfu, kMtUp = 0x80000000u, kMtLo = 0x7fffffffu;

HVAE_INLINE uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t far) {
  const uint32_t y = (a & kMtUp) | (b & kMtLo);
  return far ^ (y >> 1) ^ ((0u - (y & 1u)) & kMtA);
}
HVAE_INLINE uint32_t mt_temper(uint32_t y) {  // numpy's mt19937_next32 tempering
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}

struct Mt19937 {
  uint32_t key[kMtN];  // numpy's state words (untempered)
  uint32_t out[kMtN];  // the block's tempered outputs
  int pos;
};

// numpy's mt19937_gen (the next block of 624 words) followed by the block's tempering. The loops carry no
// dependence closer than 227 words, so each vectorises; the body is inlined into a scalar-ISA and an AVX-512
// caller.
HVAE_INLINE void mt_refill_body(Mt19937& mt) {
  uint32_t* k = mt.key;
  for (int i = 0; i < kMtN - kMtM; ++i) k[i] = mt_twist(k[i], k[i + 1], k[i + kMtM]);
  for (int i = kMtN - kMtM; i < kMtN - 1; ++i) k[i] = mt_twist(k[i], k[i + 1], k[i + (kMtM - kMtN)]);
  k[kMtN - 1] = mt_twist(k[kMtN - 1], k[0], k[kMtM - 1]);
  for (int i = 0; i < kMtN; ++i) mt.out[i] = mt_temper(k[i]);
  mt.pos = 0;
}
HVAE_INLINE void mt_temper_body(Mt19937& mt) {
  for (int i = 0; i < kMtN; ++i) mt.out[i] = mt_temper(mt.key[i]);
}
void mt_refill(Mt19937& mt) { mt_refill_body(mt); }
void mt_temper_all(Mt19937& mt) { mt_temper_body(mt); }
HVAE_AVX512 HVAE_INLINE __m512i mt_twist16(const uint32_t* a, const uint32_t* far) {
  const __m512i x = _mm512_loadu_si512(a), x1 = _mm512_loadu_si512(a + 1);
  const __m512i y = _mm512_or_si512(_mm512_and_si512(x, _mm512_set1_epi32((int)kMtUp)),
                                    _mm512_and_si512(x1, _mm512_set1_epi32((int)kMtLo)));
  const __m512i odd = _mm512_sub_epi32(_mm512_setzero_si512(), _mm512_and_si512(y, _mm512_set1_epi32(1)));
  return _mm512_xor_si512(_mm512_xor_si512(_mm512_loadu_si512(far), _mm512_srli_epi32(y, 1)),
                          _mm512_and_si512(odd, _mm512_set1_epi32((int)kMtA)));
}
// The same block 16 words at a time (the compiler leaves the second loop at 4 lanes). A 16-word group reads
// the 16 words after it still unchanged and, in the second loop, words 227 back that are already new.
HVAE_AVX512 void mt_refill_avx512(Mt19937& mt) {
  uint32_t* k = mt.key;
  int i = 0;
  for (; i + 16 <= kMtN - kMtM; i += 16) _mm512_storeu_si512(k + i, mt_twist16(k + i, k + i + kMtM));
  for (; i < kMtN - kMtM; ++i) k[i] = mt_twist(k[i], k[i + 1], k[i + kMtM]);
  for (; i + 16 <= kMtN - 1; i += 16) _mm512_storeu_si512(k + i, mt_twist16(k + i, k + i + (kMtM - kMtN)));
  for (; i < kMtN - 1; ++i) k[i] = mt_twist(k[i], k[i + 1], k[i + (kMtM - kMtN)]);
  k[kMtN - 1] = mt_twist(k[kMtN - 1], k[0], k[kMtM - 1]);
  mt_temper_body(mt);
  mt.pos = 0;
}
HVAE_AVX512 void mt_temper_all_avx512(Mt19937& mt) { mt_temper_body(mt); }

// One word of random_interval's rejection loop, branchless: the masked word v is taken (j = v, i -= 1) when
// v <= i, else skipped (~25 % of the words are rejected at random, which a branch mispredicts at ~8 ns an
// element).
template <bool STORE>
HVAE_INLINE void draw_word(uint32_t w, uint32_t m, int32_t& i, int32_t& k, int32_t* js) {
  const uint32_t v = w & m;
  const int32_t take = v <= (uint32_t)i;
  if (STORE) js[k] = (int32_t)v;
  k += take;
  i -= take;
}

// A row's draws j(i) = random_interval(i) for i = A - 1 .. 1 in stream order (js[A - 1 - i] when STORE; the
// count-only form just advances the stream past them). The mask is fixed between powers of two, and a run of
// words that cannot take i below the next power is processed without a bound check.
template <bool STORE>
void draw_row_scalar(Mt19937& mt, int32_t A, int32_t* js) {
  int32_t i = A - 1, k = 0;
  while (i >= 1) {
    const uint32_t m = 0xffffffffu >> __builtin_clz((uint32_t)i);
    const int32_t lo = (int32_t)(m >> 1);  // i keeps this mask while i > lo
    while (i > lo) {
      if (mt.pos == kMtN) mt_refill(mt);
      const int p0 = mt.pos, n = std::min(kMtN - p0, i - lo);
      const uint32_t* w = mt.out + p0;
      for (int q = 0; q < n; ++q) draw_word<STORE>(w[q], m, i, k, js);
      mt.pos = p0 + n;
    }
  }
}

// The same draws, 16 or 32 words at a time. Word q of a group meets an i in [i0 - q, i0] (i0: i at the
// group's start), so a masked word v <= i0 - q is taken whatever the words before it did and a word v > i0 is
// rejected; only v in (i0 - q, i0] depends on the words before it. A group with none of those (almost every
// group while i is large: the band averages 8 or 16 of 2^b values) takes popcount(v <= i0) words at once, its
// taken words compressed into js in order. The loop-carried chain (broadcast, compare, popcount, subtract)
// is the cost, so words go 32 at a time; a 32-word group that fails runs as two 16-word groups, and a 16-word
// group that fails runs the scalar chain. A group never crosses the next power of two (the mask changes
// there), and one that crosses the end of the generator's block is staged.
template <bool STORE>
HVAE_AVX512 HVAE_INLINE void draw_group16(const uint32_t* w, __m512i vm, uint32_t m, int32_t& i, int32_t& k,
                                          int32_t* js) {
  const __m512i iota = _mm512_set_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
  const __m512i v = _mm512_and_si512(_mm512_loadu_si512(w), vm), vi = _mm512_set1_epi32(i);
  const __mmask16 le = _mm512_cmple_epu32_mask(v, vi);
  const __mmask16 sure = _mm512_cmple_epu32_mask(v, _mm512_sub_epi32(vi, iota));
  if (__builtin_expect(le == sure, 1)) {
    if (STORE) _mm512_storeu_si512(js + k, _mm512_maskz_compress_epi32(le, v));
    const int32_t t = __builtin_popcount((unsigned)le);
    k += t;
    i -= t;
  } else {
    for (int q = 0; q < 16; ++q) draw_word<STORE>(w[q], m, i, k, js);
  }
}

template <bool STORE>
HVAE_AVX512 HVAE_INLINE void draw_group32(const uint32_t* w, __m512i vm, uint32_t m, int32_t& i, int32_t& k,
                                          int32_t* js) {
  const __m512i iota = _mm512_set_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
  const __m512i va = _mm512_and_si512(_mm512_loadu_si512(w), vm);
  const __m512i vb = _mm512_and_si512(_mm512_loadu_si512(w + 16), vm);
  const __m512i vi = _mm512_set1_epi32(i), sa = _mm512_sub_epi32(vi, iota);
  const __m512i sb = _mm512_sub_epi32(sa, _mm512_set1_epi32(16));
  const __mmask16 la = _mm512_cmple_epu32_mask(va, vi), lb = _mm512_cmple_epu32_mask(vb, vi);
  const __mmask16 ua = _mm512_cmple_epu32_mask(va, sa), ub = _mm512_cmple_epu32_mask(vb, sb);
  if (__builtin_expect((la == ua) & (lb == ub), 1)) {
    const int32_t ta = __builtin_popcount((unsigned)la), tb = __builtin_popcount((unsigned)lb);
    if (STORE) {
      _mm512_storeu_si512(js + k, _mm512_maskz_compress_epi32(la, va));
      _mm512_storeu_si512(js + k + ta, _mm512_maskz_compress_epi32(lb, vb));
    }
    k += ta + tb;
    i -= ta + tb;
  } else {
    draw_group16<STORE>(w, vm, m, i, k, js);
    draw_group16<STORE>(w + 16, vm, m, i, k, js);
  }
}

template <bool STORE>
HVAE_AVX512 void draw_row_avx512(Mt19937& mt, int32_t A, int32_t* js) {
  int32_t i = A - 1, k = 0;
  int p = mt.pos;
  while (i >= 1) {
    const uint32_t m = 0xffffffffu >> __builtin_clz((uint32_t)i);
    const int32_t lo = (int32_t)(m >> 1);  // i keeps this mask while i > lo
    const __m512i vm = _mm512_set1_epi32((int)m);
    while (i > lo) {
      if (p == kMtN) {
        mt_refill_avx512(mt);
        p = 0;
      }
      if (i - lo >= 32) {  // the group cannot take i to lo
        if (__builtin_expect(p + 32 <= kMtN, 1)) {
          draw_group32<STORE>(mt.out + p, vm, m, i, k, js);
          p += 32;
        } else {  // the block's last words and the next block's first
          uint32_t st[32];
          const int L = kMtN - p;
          std::memcpy(st, mt.out + p, sizeof(uint32_t) * L);
          mt_refill_avx512(mt);
          std::memcpy(st + L, mt.out, sizeof(uint32_t) * (32 - L));
          draw_group32<STORE>(st, vm, m, i, k, js);
          p = 32 - L;
        }
      } else if (i - lo >= 16 && p + 16 <= kMtN) {
        draw_group16<STORE>(mt.out + p, vm, m, i, k, js);
        p += 16;
      } else {
        draw_word<STORE>(mt.out[p++], m, i, k, js);
      }
    }
  }
  mt.pos = p;
}

// The swaps replayed backwards for the n_neg leading positions only (rows are independent here). The value
// that ends at position q < n_neg is the one at src[q] before the swaps, found by undoing them from the last
// (i = 1) to the first (i = A - 1); at[] maps a position to the tracked q sitting there (-1: none; int8 up to
// 127 tracked positions, so the map stays in L1, int16 past that), back to all -1 on return.
template <typename At>
void replay_row(int32_t A, int32_t n_neg, const int32_t* js, At* at, int32_t* src) {
  for (int32_t q = 0; q < n_neg; ++q) {
    src[q] = q;
    at[q] = (At)q;
  }
  for (int32_t i = 1; i < A; ++i) {
    const int32_t j = js[A - 1 - i];
    const int32_t a = at[i], b = at[j];
    if (__builtin_expect((a & b) >= 0, 0) && j != i) {  // either position tracked
      if (a >= 0) src[a] = j;
      if (b >= 0) src[b] = i;
      at[i] = (At)b;
      at[j] = (At)a;
    }
  }
  for (int32_t q = 0; q < n_neg; ++q) at[src[q]] = -1;
}

// The ascending items neither in the user's training row nor the test item (np.where(mask)[0]); ex[] is all 0
// on entry and on return. Returns their count.
int32_t available_row(const int64_t* row_ptr, const int32_t* col_idx, int64_t n_items, int32_t u, int32_t t,
                      uint8_t* ex, int32_t* avail) {
  const int64_t b = row_ptr[u], e = row_ptr[u + 1];
  for (int64_t k = b; k < e; ++k) ex[col_idx[k]] = 1;
  ex[t] = 1;
  int32_t A = 0;
  if (avail) {
    for (int32_t i = 0; i < (int32_t)n_items; ++i) {
      avail[A] = i;
      A += ex[i] ^ 1;
    }
  } else {
    int32_t x = 0;
    for (int64_t k = b; k < e; ++k) {
      x += ex[col_idx[k]];  // each distinct item once
      ex[col_idx[k]] = 0;
    }
    x += ex[t];
    A = (int32_t)n_items - x;
  }
  for (int64_t k = b; k < e; ++k) ex[col_idx[k]] = 0;
  ex[t] = 0;
  return A;
}

bool use_avx512() {
  static const bool hw = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl");
  }();
  const char* s = std::getenv("HVAE_NEG_SCALAR");
  return hw && !(s && s[0] == '1');
}

}  // namespace

// Rows go in chunks. The caller's thread runs the one sequential stream over chunk c: per row the count of
// available items and, when a draw happens, a snapshot of the generator (624 words and the position) before
// the row's words are consumed, then the stream advanced past them (the count-only draw: no stores). Up to
// kWorkers threads meanwhile finish chunk c - 1, each row independently: regenerate the row's words from its
// snapshot (the stored draw), list the available items and replay the swaps.
extern "C" int hvae_negatives_legacy(uint32_t* mt_key, int32_t* mt_pos, const int64_t* row_ptr,
                                     int64_t n_users, const int32_t* col_idx, int64_t n_items, const int32_t* users,
                                     const int32_t* tests, int64_t n_rows, int32_t n_neg, int32_t* out,
                                     int32_t* counts) {
  HVAE_REQUIRE(mt_key && mt_pos && row_ptr && n_users >= 0 && n_items > 0 && n_items < (int64_t)1 << 31 && n_rows >= 0 &&
                   n_neg >= 0 && n_neg <= 32767 && (n_rows == 0 || (users && tests && out && counts)),
               "hvae_negatives_legacy: bad args (n_neg <= 32767)");
  HVAE_REQUIRE(*mt_pos >= 0 && *mt_pos <= kMtN, "hvae_negatives_legacy: MT19937 position outside [0, 624]");
  for (int64_t r = 0; r < n_rows; ++r) {
    HVAE_REQUIRE(users[r] >= 0 && users[r] < n_users && tests[r] >= 0 && tests[r] < n_items,
                 "hvae_negatives_legacy: row %lld: bad user / test item", (long long)r);
    for (int64_t k = row_ptr[users[r]]; k < row_ptr[users[r] + 1]; ++k)
      HVAE_REQUIRE(col_idx[k] >= 0 && col_idx[k] < n_items, "hvae_negatives_legacy: item outside [0, n_items)");
  }
  const bool avx = use_avx512();
  Mt19937 mt;
  std::memcpy(mt.key, mt_key, sizeof(mt.key));
  mt.pos = *mt_pos;
  if (avx)
    mt_temper_all_avx512(mt);
  else
    mt_temper_all(mt);
  int kWorkers = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  if (const char* s = std::getenv("HVAE_NEG_WORKERS")) kWorkers = std::max(1, std::min(64, std::atoi(s)));
  constexpr int64_t kChunk = 256;
  struct Snap {
    uint32_t key[kMtN];
    int32_t pos;
  };
  std::vector<Snap> snb[2] = {std::vector<Snap>(kChunk), std::vector<Snap>(kChunk)};
  std::vector<int32_t> Ab[2] = {std::vector<int32_t>(kChunk), std::vector<int32_t>(kChunk)};
  std::vector<uint8_t> ex0((size_t)n_items, 0);
  auto finish = [&](int64_t c0, int64_t nr, const Snap* sn, const int32_t* As) {  // chunk c - 1, in parallel
    auto work = [&](int wk) {
      std::vector<uint8_t> ex((size_t)n_items, 0);
      std::vector<int32_t> avail((size_t)n_items), js((size_t)n_items + 16), src((size_t)n_neg + 1);
      const bool narrow = n_neg <= 127;
      std::vector<int8_t> at8(narrow ? (size_t)n_items : 0, -1);
      std::vector<int16_t> at16(narrow ? 0 : (size_t)n_items, -1);
      Mt19937 g;
      for (int64_t rr = wk; rr < nr; rr += kWorkers) {
        const int64_t r = c0 + rr;
        const int32_t A = available_row(row_ptr, col_idx, n_items, users[r], tests[r], ex.data(), avail.data());
        int32_t* o = out + r * n_neg;
        if (As[rr] < n_neg) {  // every available item, no draw (`available if len(available) < n`)
          std::memcpy(o, avail.data(), sizeof(int32_t) * (size_t)A);
          counts[r] = A;
          continue;
        }
        std::memcpy(g.key, sn[rr].key, sizeof(g.key));
        g.pos = sn[rr].pos;
        if (avx) {
          mt_temper_all_avx512(g);
          draw_row_avx512<true>(g, A, js.data());
        } else {
          mt_temper_all(g);
          draw_row_scalar<true>(g, A, js.data());
        }
        if (narrow)
          replay_row(A, n_neg, js.data(), at8.data(), src.data());
        else
          replay_row(A, n_neg, js.data(), at16.data(), src.data());
        for (int32_t q = 0; q < n_neg; ++q) o[q] = avail[src[q]];
        counts[r] = n_neg;
      }
    };
    std::vector<std::thread> th;
    for (int wk = 1; wk < kWorkers; ++wk) th.emplace_back(work, wk);
    work(0);
    for (auto& x : th) x.join();
  };
  std::thread pending;
  for (int64_t c0 = 0, ci = 0; c0 < n_rows; c0 += kChunk, ci ^= 1) {
    const int64_t nr = std::min(kChunk, n_rows - c0);
    for (int64_t rr = 0; rr < nr; ++rr) {  // the stream, in row order
      const int64_t r = c0 + rr;
      const int32_t A = available_row(row_ptr, col_idx, n_items, users[r], tests[r], ex0.data(), nullptr);
      Ab[ci][rr] = A;
      if (A < n_neg) continue;
      std::memcpy(snb[ci][rr].key, mt.key, sizeof(mt.key));
      snb[ci][rr].pos = mt.pos;
      if (avx)
        draw_row_avx512<false>(mt, A, nullptr);
      else
        draw_row_scalar<false>(mt, A, nullptr);
    }
    if (pending.joinable()) pending.join();  // chunk c - 1 done: its buffers are free again
    pending = std::thread(finish, c0, nr, snb[ci].data(), Ab[ci].data());
  }
  if (pending.joinable()) pending.join();
  std::memcpy(mt_key, mt.key, sizeof(mt.key));
  *mt_pos = mt.pos;
  return HVAE_OK;
}

#endif  // __HIP_DEVICE_COMPILE__
