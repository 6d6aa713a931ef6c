// hvae_common.h -- shared device/host helpers for libhvae (gfx950 / CDNA4 only).
//
// Everything here is written for 64-lane wavefronts (wave = 64 on gfx950) and
// for the launch conventions of the C-ABI in include/hvae.h: raw device
// pointers owned by the caller, a hipStream_t passed as void*, no allocation
// and no host synchronisation inside any launcher (so every launcher can be
// captured into a hipGraph).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <math.h>
#include <stdlib.h>

#include "../../include/hvae.h"

namespace hvae {

// ---------------------------------------------------------------- errors ---
// Thread-local last-error text, returned by hvae_last_error().
void set_error(const char* fmt, ...);

#define HVAE_FAIL(code, ...)                                                   \
  do {                                                                         \
    ::hvae::set_error(__VA_ARGS__);                                            \
    return (code);                                                             \
  } while (0)

#define HVAE_REQUIRE(cond, ...)                                                \
  do {                                                                         \
    if (!(cond)) HVAE_FAIL(HVAE_ERR_ARG, __VA_ARGS__);                         \
  } while (0)

#define HVAE_HIP(call)                                                         \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess)                                                      \
      HVAE_FAIL(HVAE_ERR_HIP, "%s failed: %s (%s:%d)", #call,                  \
                hipGetErrorString(e_), __FILE__, __LINE__);                    \
  } while (0)

// After a <<<>>> launch: surface launch-configuration errors immediately.
#define HVAE_LAUNCH_CHECK(name)                                                \
  do {                                                                         \
    hipError_t e_ = hipGetLastError();                                         \
    if (e_ != hipSuccess)                                                      \
      HVAE_FAIL(HVAE_ERR_HIP, "launch of %s failed: %s", name,                 \
                hipGetErrorString(e_));                                        \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Arrival tickets for "last block finishes the reduction" kernels (one launch
// instead of partials + a second reduce launch). The pool is a device global of
// hvae_abi.hip (zero at code-object load); the last arriving block resets its
// ticket, so tickets are zero between launches. Each launch takes a slice of
// kTicketSlice tickets in rotation, so launches that may run concurrently on
// different streams (the nodes of one captured graph) never share one.
constexpr int kTicketPool = 1 << 16, kTicketSlice = 256;
constexpr int kRowSqParts = HVAE_ROWSQ_PARTS;  // fp64 partial sums of squares per W1 gradient row (hvae_rowgrad.rowsq)
unsigned* ticket_slice();  // nullptr (error set) on failure

// A/B knobs (HVAE_DEC_*, HVAE_TOPK_*, HVAE_TK_*, HVAE_GEMM_* in the environment) are read only by variant builds
// compiled with -DHVAE_AB=1 (scripts/build_ab.sh -> build_var/libhvae_ab.so); the product library ignores the
// environment and always runs its defaults.
#ifndef HVAE_AB
#define HVAE_AB 0
#endif
static inline const char* ab_getenv(const char* name) {
#if HVAE_AB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// Partials exchanged between the blocks of one launch go through agent-coherent
// (sc1) stores and loads: they bypass the per-XCD L2s that plain accesses may
// hit stale, without the whole-L2 writeback / invalidate an agent-scope
// __threadfence() costs on gfx950 (that cost per block is what made a fenced
// version slower than a second launch).
__device__ __forceinline__ void st_shared_f(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_shared_f(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B agent-coherent (sc1) stores and loads through a buffer resource over a wave-uniform base (32-bit byte
// offsets): one fabric write per 16 B where the scalar sc1 store is one per dword (MI355X_MICROARCH: a dword sc1
// store costs ~6x a dwordx4 per byte). Compiler builtins, not inline asm: the compiler then inserts the waits
// the loads need and the wait state a >8-byte store needs before its data registers are rewritten (an inline-asm
// global_store_dwordx4 followed by a VALU write of its data registers stored garbage).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t coherent_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
constexpr int kCpolSc1 = 16;  // buffer cache-policy bits on gfx950: sc1
__device__ __forceinline__ void st_sc1_f4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 x = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, (int)off, 0, kCpolSc1);
}
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kCpolSc1);
  return make_float4(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]), __uint_as_float(x[3]));
}
__device__ __forceinline__ void st_shared_d(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_shared_d(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by every thread of a block after it wrote its partials with
// st_shared_*: true in the one block that arrives last at ticket *t; that block
// then reads every block's partials with ld_shared_*. Each thread waits for its
// own stores to complete (s_waitcnt 0) before the barrier, so all of the
// block's partials have reached the coherence point before thread 0 takes a
// ticket.
__device__ __forceinline__ bool last_block_arrives(unsigned* t, unsigned n_blocks) {
  __shared__ unsigned s_last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old == n_blocks - 1);
    if (s_last) __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last;
}

// Live kernel timing (hvae_probe_arm / hvae_probe_collect): a launcher brackets
// the launch of a named kernel with ProbeScope; when that name is armed (and
// the stream is not capturing) a hipEvent pair is recorded around it on its
// own stream.
void probe_mark(const char* name, hipStream_t st, bool begin);
struct ProbeScope {
  const char* name;
  hipStream_t st;
  ProbeScope(const char* n, hipStream_t s) : name(n), st(s) { probe_mark(name, st, true); }
  ~ProbeScope() { probe_mark(name, st, false); }
};

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// --------------------------------------------------------------- device ----
constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64
// floats. Result valid in every thread.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// Exact (erf) GELU, as torch.nn.GELU() default (approximate='none').
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}
// d/dx GELU(x) = Phi(x) + x * phi(x)
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// ------------------------------------------------------ Philox4x32-10 ------
// Counter-based RNG: every random value is a pure function of
// (seed, step, stream tag, element index), so dropout masks and reparameter-
// isation noise can be regenerated in the backward pass instead of stored, and
// a hipGraph replay advances them through the device-side step counter.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Stream tags (the 4th counter word) so that independent draws never collide.
enum : uint32_t {
  kTagEncDrop = 0x100u,   // + hidden layer index
  kTagProjDrop = 0x200u,
  kTagEps = 0x300u,
};

__device__ __forceinline__ uint32_t rng_u32(uint64_t seed, int64_t step, uint32_t tag, uint64_t idx) {
  const u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)step, tag};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32)).x;
}
// uniform in [0, 1) with 24 random bits
__device__ __forceinline__ float u01(uint32_t r) { return (float)(r >> 8) * (1.0f / 16777216.0f); }

// Dropout multiplier: 0 or 1/(1-p) (torch semantics: keep with prob 1-p and
// scale the survivors). External masks (parity mode) override the RNG.
__device__ __forceinline__ float dropout_mult(float p, float scale, const float* ext, uint64_t i,
                                           uint64_t seed, int64_t step, uint32_t tag) {
  if (ext) return ext[i];
  if (p <= 0.f) return 1.f;
  if (p >= 1.f) return 0.f;
  return (u01(rng_u32(seed, step, tag, i)) >= p) ? scale : 0.f;
}

// Standard normal via Box-Muller from one Philox call.
__device__ __forceinline__ float normal_f(uint64_t seed, int64_t step, uint32_t tag, uint64_t idx) {
  const u32x4 c{(uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)step, tag};
  const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float a = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  const float b = (float)(r.y >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * logf(a)) * cospif(2.0f * b);
}

// Matrix row of batch entry b (hvae_csr_batch.rows / rows_offset).
__device__ __forceinline__ int64_t batch_row(const int32_t* rows, const int64_t* rows_offset, int64_t b) {
  return rows ? (int64_t)rows[(rows_offset ? *rows_offset : 0) + b] : b;
}

__device__ __forceinline__ int64_t load_step(const int64_t* step_dev) {
  return step_dev ? *step_dev : 0;
}

// ------------------------------------------------------------ bf16 ---------
typedef unsigned short bf16_t;
// round-to-nearest-even (inputs here are finite activations/embeddings)
__device__ __host__ __forceinline__ bf16_t f2bf(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}
__device__ __host__ __forceinline__ float bf2f(bf16_t h) {
  uint32_t u = ((uint32_t)h) << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

// Batch means of the loss rows in fp64, the step's (total, recon, kl) and the
// epoch accumulators -- vae_loss_function's reductions (src/ml/model.py:283-292).
// One 256-thread block; shared by k_loss_finalize and the decoder finalize's last
// block (which reads recon rows other blocks just wrote, hence `coherent`).
__device__ __forceinline__ void loss_block_reduce(const float* recon_rows, bool coherent, const float* kl_rows,
                                                  int64_t nb, float beta, float* out3, double* accum3) {
  __shared__ double lred[2][4];
  double r = 0.0, k = 0.0;
  for (int64_t i = threadIdx.x; i < nb; i += 256) {
    r += (double)(coherent ? ld_shared_f(&recon_rows[i]) : recon_rows[i]);
    k += (double)kl_rows[i];
  }
  r = wave_sum_d(r);
  k = wave_sum_d(k);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { lred[0][w] = r; lred[1][w] = k; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double rs = ((lred[0][0] + lred[0][1]) + lred[0][2]) + lred[0][3];
    const double ks = ((lred[1][0] + lred[1][1]) + lred[1][2]) + lred[1][3];
    const float recon = (float)(rs / (double)nb), kl = (float)(ks / (double)nb);
    const float total = recon + beta * kl;
    out3[0] = total; out3[1] = recon; out3[2] = kl;
    if (accum3) {
      accum3[0] += (double)total; accum3[1] += (double)recon; accum3[2] += (double)kl;
    }
  }
}

}  // namespace hvae
