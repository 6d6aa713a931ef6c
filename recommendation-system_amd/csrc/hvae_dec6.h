// hvae_dec6.h -- the version-6 bf16 sweep's plan and partial-slot map (hvae_decoder6.hip), shared with the
// finalize in hvae_decoder.hip.
#pragma once

#include "hvae_common.h"

namespace hvae {

constexpr int kDec6D = 768;
constexpr int kDec6Users = 96;  // users per block (per E tile)

// Tasks are (user block u, item split s) in split-major order k = s * nub + u. The first `main` run one per
// block; the X = nub * S - main tasks past them are cut into P pieces each (piece j of excess task e -> slot
// main + e * P + j). A task's partial rows are [slot][kDec6Users].
struct Dec6Plan {
  int nub, S, tps, main, X, P, ntiles, grid, slots;
};

struct Dec6Args {
  const float* U;
  int64_t ldu;
  const bf16_t* E;
  const float* e_maxnorm;
  int64_t nb, N;
  int nub, S, tps, main, X, P, ntiles;
  int* flag;
  float* m;
  float* l;
  float* O;
};

// The user-block's partial slots, in the fixed merge order: its main tasks by split, then each excess task's
// pieces in order.
__host__ __device__ __forceinline__ int dec6_nmain(int nub, int S, int main, int u) {
  return main > u ? min(S, (main - u + nub - 1) / nub) : 0;
}
__host__ __device__ __forceinline__ int dec6_nslots(int nub, int S, int main, int P, int u) {
  const int nm = dec6_nmain(nub, S, main, u);
  return nm + (S - nm) * P;
}
__host__ __device__ __forceinline__ int dec6_slot_of(int nub, int S, int main, int P, int u, int i) {
  const int nm = dec6_nmain(nub, S, main, u);
  if (i < nm) return i * nub + u;
  const int j = i - nm, sp = nm + j / P;
  return main + (sp * nub + u - main) * P + j % P;
}

bool dec6_plan(int64_t nb, int64_t N, Dec6Plan& p);
int dec6_launch(bool with_o, const float* U, int64_t ldu, const void* E, const float* enorm, int64_t nb, int64_t N,
                const Dec6Plan& p, int* flag, float* m, float* l, float* O, hipStream_t st);

}  // namespace hvae
