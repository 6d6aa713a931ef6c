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
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "hvae_common.h"

namespace {

constexpr int kMtN = 624, kMtM = 397;

struct Mt19937 {
  uint32_t key[kMtN];  // numpy's state words (untempered)
  uint32_t out[kMtN];  // the block's tempered outputs
  int pos;

  void gen() {  // the next block of 624 (numpy's mt19937_gen)
    constexpr uint32_t kA = 0x9908b0dfu, kUp = 0x80000000u, kLo = 0x7fffffffu;
    int i = 0;
    for (; i < kMtN - kMtM; ++i) {
      const uint32_t y = (key[i] & kUp) | (key[i + 1] & kLo);
      key[i] = key[i + kMtM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    for (; i < kMtN - 1; ++i) {
      const uint32_t y = (key[i] & kUp) | (key[i + 1] & kLo);
      key[i] = key[i + (kMtM - kMtN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    const uint32_t y = (key[kMtN - 1] & kUp) | (key[0] & kLo);
    key[kMtN - 1] = key[kMtM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    pos = 0;
  }
  void temper_from(int p0) {  // numpy's mt19937_next32 tempering, a block at a time (vectorised)
    for (int i = p0; i < kMtN; ++i) {
      uint32_t y = key[i];
      y ^= y >> 11;
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= y >> 18;
      out[i] = y;
    }
  }
  inline uint32_t next() {
    if (__builtin_expect(pos == kMtN, 0)) {
      gen();
      temper_from(0);
    }
    return out[pos++];
  }
};

}  // namespace

namespace {

// Pass (1) of a row, on the caller's thread (the stream is sequential): the draws j(i) = random_interval(i) for
// i = A - 1 .. 1 in stream order, js[A - 1 - i]. A word is taken (j = word & mask(i), i -= 1) when j <= i,
// else skipped: random_interval's rejection loop without a branch (~25 % of the words are rejected at random,
// which a branch mispredicts at ~8 ns an element). The mask is fixed between powers of two, and a run of
// words that cannot take i below the next power is processed without a bound check, so the loop-carried chain
// is one compare and one subtract per word.
void draw_row(Mt19937& mt, int32_t A, int32_t* js) {
  int32_t i = A - 1, k = 0;
  while (i >= 1) {
    const uint32_t m = 0xffffffffu >> __builtin_clz((uint32_t)i);
    const int32_t lo = (int32_t)(m >> 1);  // i keeps this mask while i > lo
    while (i > lo) {
      if (mt.pos == kMtN) {
        mt.gen();
        mt.temper_from(0);
      }
      const int p0 = mt.pos;
      const int n = std::min(kMtN - p0, i - lo);
      const uint32_t* w = mt.out + p0;
      for (int q = 0; q < n; ++q) {
        const uint32_t v = w[q] & m;
        const int32_t take = v <= (uint32_t)i;
        js[k] = (int32_t)v;
        k += take;
        i -= take;
      }
      mt.pos = p0 + n;
    }
  }
}

// Pass (2) of a row, on a worker (rows are independent here): the swaps replayed backwards for the n_neg
// leading positions only. The value that ends at position q < n_neg is the one at src[q] before the swaps,
// found by undoing them from the last (i = 1) to the first (i = A - 1); at[] maps a position to the tracked q
// sitting there (-1: none; int8, so the map stays in L1), back to all -1 on return.
void replay_row(int32_t A, int32_t n_neg, const int32_t* js, int8_t* at, int32_t* src) {
  for (int32_t q = 0; q < n_neg; ++q) {
    src[q] = q;
    at[q] = (int8_t)q;
  }
  for (int32_t i = 1; i < A; ++i) {
    const int32_t j = js[A - 1 - i];
    const int32_t a = at[i], b = at[j];
    if (__builtin_expect((a & b) >= 0, 0) && j != i) {  // either position tracked
      if (a >= 0) src[a] = j;
      if (b >= 0) src[b] = i;
      at[i] = (int8_t)b;
      at[j] = (int8_t)a;
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

}  // namespace

// Rows go in chunks: the caller's thread draws chunk c (pass 1, the one sequential stream) while up to
// kWorkers threads finish chunk c - 1 (the available list and pass 2 of each row).
extern "C" int hvae_negatives_legacy(uint32_t* mt_key, int32_t* mt_pos, const int64_t* row_ptr,
                                     const int32_t* col_idx, int64_t n_items, const int32_t* users,
                                     const int32_t* tests, int64_t n_rows, int32_t n_neg, int32_t* out,
                                     int32_t* counts) {
  HVAE_REQUIRE(mt_key && mt_pos && row_ptr && n_items > 0 && n_items < (int64_t)1 << 31 && n_rows >= 0 &&
                   n_neg >= 0 && n_neg <= 127 && (n_rows == 0 || (users && tests && out && counts)),
               "hvae_negatives_legacy: bad args (n_neg <= 127)");
  HVAE_REQUIRE(*mt_pos >= 0 && *mt_pos <= kMtN, "hvae_negatives_legacy: MT19937 position outside [0, 624]");
  for (int64_t r = 0; r < n_rows; ++r) {
    HVAE_REQUIRE(users[r] >= 0 && tests[r] >= 0 && tests[r] < n_items,
                 "hvae_negatives_legacy: row %lld: bad user / test item", (long long)r);
    for (int64_t k = row_ptr[users[r]]; k < row_ptr[users[r] + 1]; ++k)
      HVAE_REQUIRE(col_idx[k] >= 0 && col_idx[k] < n_items, "hvae_negatives_legacy: item outside [0, n_items)");
  }
  Mt19937 mt;
  std::memcpy(mt.key, mt_key, sizeof(mt.key));
  mt.pos = *mt_pos;
  mt.temper_from(0);
  const int kWorkers = (int)std::max(1u, std::min(4u, std::thread::hardware_concurrency()));
  // chunk rows: about 32 M draw slots per chunk buffer (two buffers in flight)
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(256, ((int64_t)1 << 25) / n_items));
  std::vector<int32_t> jsb[2] = {std::vector<int32_t>((size_t)(chunk * n_items)),
                                 std::vector<int32_t>((size_t)(chunk * n_items))};
  std::vector<int32_t> Ab[2] = {std::vector<int32_t>((size_t)chunk), std::vector<int32_t>((size_t)chunk)};
  std::vector<uint8_t> ex0((size_t)n_items, 0);
  auto finish = [&](int64_t c0, int64_t nr, const int32_t* js, const int32_t* As) {  // pass 2 of a chunk
    auto work = [&](int wk) {
      std::vector<uint8_t> ex((size_t)n_items, 0);
      std::vector<int32_t> avail((size_t)n_items), src((size_t)n_neg + 1);
      std::vector<int8_t> at((size_t)n_items, -1);
      for (int64_t rr = wk; rr < nr; rr += kWorkers) {
        const int64_t r = c0 + rr;
        const int32_t A = available_row(row_ptr, col_idx, n_items, users[r], tests[r], ex.data(), avail.data());
        int32_t* o = out + r * n_neg;
        if (As[rr] < n_neg) {  // every available item, no draw (`available if len(available) < n`)
          std::memcpy(o, avail.data(), sizeof(int32_t) * (size_t)A);
          counts[r] = A;
          continue;
        }
        replay_row(A, n_neg, js + rr * n_items, at.data(), src.data());
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
  for (int64_t c0 = 0, ci = 0; c0 < n_rows; c0 += chunk, ci ^= 1) {
    const int64_t nr = std::min(chunk, n_rows - c0);
    for (int64_t rr = 0; rr < nr; ++rr) {  // pass 1: the stream, in row order
      const int64_t r = c0 + rr;
      const int32_t A = available_row(row_ptr, col_idx, n_items, users[r], tests[r], ex0.data(), nullptr);
      Ab[ci][rr] = A;
      if (A >= n_neg) draw_row(mt, A, jsb[ci].data() + rr * n_items);
    }
    if (pending.joinable()) pending.join();  // chunk c - 1 done: its buffers are free again
    pending = std::thread(finish, c0, nr, jsb[ci].data(), Ab[ci].data());
  }
  if (pending.joinable()) pending.join();
  std::memcpy(mt_key, mt.key, sizeof(mt.key));
  *mt_pos = mt.pos;
  return HVAE_OK;
}
