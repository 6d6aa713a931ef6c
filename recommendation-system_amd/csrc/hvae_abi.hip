// hvae_abi.hip -- version / error plumbing of the C ABI and small utility launchers.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "hvae_common.h"

namespace hvae {

static thread_local char g_last_error[1024] = "";

__device__ unsigned g_tickets[kTicketPool];

unsigned* ticket_slice() {
  static unsigned* pools[64] = {};  // per device: the symbol has one instance per device
  static std::atomic<uint64_t> next{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("ticket_slice: no current device");
    return nullptr;
  }
  if (!pools[dev] && hipGetSymbolAddress((void**)&pools[dev], HIP_SYMBOL(g_tickets)) != hipSuccess) {
    set_error("ticket_slice: hipGetSymbolAddress failed");
    return nullptr;
  }
  return pools[dev] + (next.fetch_add(1) % (kTicketPool / kTicketSlice)) * kTicketSlice;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

// ---- live kernel timing
struct Probe {
  char name[64] = "";
  std::vector<hipEvent_t> ev;  // [2 * cap]
  int n = 0, cap = 0;
  bool open = false;
};
static Probe g_probe;
static std::mutex g_probe_mu;

// Head start for an armed launch: one wave that spins ~200 us on the constant 100-MHz clock (a bounded loop)
// before the start event. A hipEvent recorded on a stream the device has drained is stamped before the host has
// enqueued the kernel after it, so on a host-bound (eager) step the pair would time the host's gap too (the fp8
// Syn-10M line's 428-us "adam_catchup" against 115 us in its kernel trace); with the hold in front, the kernel
// is queued behind the start event by the time the event executes.
__global__ void k_probe_hold(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

void probe_mark(const char* name, hipStream_t st, bool begin) {
  if (g_probe.cap == 0) return;  // fast path: nothing armed
  std::lock_guard<std::mutex> lk(g_probe_mu);
  if (g_probe.cap == 0 || strcmp(name, g_probe.name) != 0) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  if (begin) {
    if (g_probe.n >= g_probe.cap) return;
    // a pending launch error of the caller's is left for the caller's own check (hipGetLastError below would
    // clear it): no hold, no bracket
    if (hipPeekAtLastError() != hipSuccess) return;
    k_probe_hold<<<1, 64, 0, st>>>(20000);  // 200 us at 100 MHz
    if (hipGetLastError() != hipSuccess) return;
    if (hipEventRecord(g_probe.ev[2 * g_probe.n], st) == hipSuccess) g_probe.open = true;
  } else if (g_probe.open) {
    if (hipEventRecord(g_probe.ev[2 * g_probe.n + 1], st) == hipSuccess) ++g_probe.n;
    g_probe.open = false;
  }
}

__global__ void k_counter_add(int64_t* c, int64_t d, int64_t* c2, int64_t d2) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *c += d;
    if (c2) *c2 += d2;
  }
}

__global__ void k_cast_bf16(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      ushort4 o;
      o.x = f2bf(v.x); o.y = f2bf(v.y); o.z = f2bf(v.z); o.w = f2bf(v.w);
      *reinterpret_cast<ushort4*>(y + i) = o;
    } else {
      for (int64_t j = i; j < n; ++j) y[j] = f2bf(x[j]);
    }
  }
}

}  // namespace hvae

using namespace hvae;

extern "C" int hvae_version(void) { return HVAE_ABI_VERSION; }

extern "C" int hvae_last_error(char* buf, size_t len) {
  if (!buf || len == 0) return HVAE_ERR_ARG;
  strncpy(buf, g_last_error, len - 1);
  buf[len - 1] = '\0';
  return HVAE_OK;
}

extern "C" int hvae_probe_arm(const char* kernel, int max_launches) {
  std::lock_guard<std::mutex> lk(g_probe_mu);
  for (hipEvent_t e : g_probe.ev) (void)hipEventDestroy(e);
  g_probe.ev.clear();
  g_probe.n = g_probe.cap = 0;
  g_probe.open = false;
  g_probe.name[0] = '\0';
  if (!kernel || max_launches <= 0) return HVAE_OK;
  HVAE_REQUIRE(strlen(kernel) < sizeof(g_probe.name), "hvae_probe_arm: name too long");
  g_probe.ev.resize(2 * (size_t)max_launches);
  for (auto& e : g_probe.ev) HVAE_HIP(hipEventCreate(&e));
  strcpy(g_probe.name, kernel);
  g_probe.cap = max_launches;
  return HVAE_OK;
}

extern "C" int hvae_probe_collect(double* avg_us, int* launches) {
  HVAE_REQUIRE(avg_us && launches, "hvae_probe_collect: null out");
  std::lock_guard<std::mutex> lk(g_probe_mu);
  double tot = 0.0;
  for (int i = 0; i < g_probe.n; ++i) {
    HVAE_HIP(hipEventSynchronize(g_probe.ev[2 * i + 1]));
    float ms = 0.f;
    HVAE_HIP(hipEventElapsedTime(&ms, g_probe.ev[2 * i], g_probe.ev[2 * i + 1]));
    tot += ms;
  }
  *launches = g_probe.n;
  *avg_us = g_probe.n ? tot * 1e3 / g_probe.n : 0.0;
  return HVAE_OK;
}

extern "C" int hvae_counter_add(int64_t* counter, int64_t delta, void* stream) {
  HVAE_REQUIRE(counter, "hvae_counter_add: null counter");
  k_counter_add<<<1, 64, 0, as_stream(stream)>>>(counter, delta, nullptr, 0);
  HVAE_LAUNCH_CHECK("k_counter_add");
  return HVAE_OK;
}

extern "C" int hvae_counters_add(int64_t* a, int64_t da, int64_t* b, int64_t db, void* stream) {
  HVAE_REQUIRE(a, "hvae_counters_add: null counter");
  k_counter_add<<<1, 64, 0, as_stream(stream)>>>(a, da, b, db);
  HVAE_LAUNCH_CHECK("k_counter_add");
  return HVAE_OK;
}

extern "C" int hvae_cast_bf16(const float* x, void* y, int64_t n, void* stream) {
  HVAE_REQUIRE(n >= 0 && (n == 0 || (x && y)), "hvae_cast_bf16: bad args");
  HVAE_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)y % 8) == 0,
               "hvae_cast_bf16: x must be 16-B and y 8-B aligned");
  if (n == 0) return HVAE_OK;
  const int64_t blocks = std::min<int64_t>(cdiv(n, 256 * 4), 4096);
  k_cast_bf16<<<(unsigned)blocks, 256, 0, as_stream(stream)>>>(x, (bf16_t*)y, n);
  HVAE_LAUNCH_CHECK("k_cast_bf16");
  return HVAE_OK;
}
