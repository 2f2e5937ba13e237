// Status reporting and the per-kernel event timer behind the C ABI.
//
// The timer lets bench.py measure each kernel's average launch duration live, on the stream the
// kernel is launched on (torch.cuda.Event only sees torch's current stream): while enabled, every
// launch of an enabled kernel id carries a pair of pre-created hipEvents as its start / stop events
// (pico_launch in common.h).
#include <stdarg.h>
#include <stdio.h>
#include <atomic>
#include <mutex>
#include <vector>
#include "common.h"

#include <cstdlib>

static thread_local char g_err[512] = "";

int pico_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return PICO_EINVAL;
}

int pico_check_launch(const char* op) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: kernel launch failed: %s", op, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

namespace {
struct Pool {
  int capacity = 0;
  int used = 0;  // event pairs recorded
  std::vector<hipEvent_t> ev;
};
std::mutex g_mu;
std::atomic<unsigned> g_mask{0};  // bit k set: kernel id k is being timed
Pool g_pool[PICO_K_COUNT];

void destroy_pool(Pool& p) {
  for (auto e : p.ev) (void)hipEventDestroy(e);
  p.ev.clear();
  p.used = p.capacity = 0;
}
}  // namespace

bool pico_prof_events(int kid, hipEvent_t* start, hipEvent_t* stop) {
  if (!(g_mask.load(std::memory_order_relaxed) & (1u << kid))) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  Pool& p = g_pool[kid];
  if (p.used >= p.capacity) return false;
  *start = p.ev[2 * p.used];
  *stop = p.ev[2 * p.used + 1];
  p.used++;
  return true;
}

namespace {
// knob values: the environment once, at first use (_lib.load() calls pico_select when it loads the library), then
// pico_select
struct SelTable {
  int v[PICO_SEL_COUNT];
  SelTable() {
    static const char* const names[PICO_SEL_COUNT] = {"PICO_ATTN_KVP", "PICO_KVP_WAVES", "PICO_ATTN_GROUPS",
                                                      "PICO_ATTN_FWD"};
    for (int i = 0; i < PICO_SEL_COUNT; ++i) {
      const char* e = getenv(names[i]);
      v[i] = (e && *e) ? atoi(e) : PICO_SEL_AUTO;
    }
  }
};
SelTable& sel_table() {
  static SelTable t;
  return t;
}
}  // namespace

int pico_sel(int knob) { return (knob >= 0 && knob < PICO_SEL_COUNT) ? sel_table().v[knob] : PICO_SEL_AUTO; }


extern "C" {

int pico_abi_version(void) { return PICO_ABI_VERSION; }

int pico_select(int knob, int value) {
  if (knob < 0 || knob >= PICO_SEL_COUNT) return -2;
  const int old = sel_table().v[knob];
  sel_table().v[knob] = value;
  return old;
}

const char* pico_last_error(void) { return g_err; }

int pico_prof_enable(int kernel_id, int capacity) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (kernel_id <= 0) {  // disable everything
    g_mask.store(0);
    for (auto& p : g_pool) destroy_pool(p);
    return 0;
  }
  PICO_REQUIRE(kernel_id < PICO_K_COUNT, "pico_prof_enable: bad kernel id %d", kernel_id);
  PICO_REQUIRE(capacity > 0 && capacity <= (1 << 20), "pico_prof_enable: bad capacity %d", capacity);
  Pool& p = g_pool[kernel_id];
  destroy_pool(p);
  p.ev.resize(2 * (size_t)capacity);
  for (auto& e : p.ev) {
    hipError_t r = hipEventCreate(&e);
    if (r != hipSuccess) {
      pico_set_error("pico_prof_enable: hipEventCreate: %s", hipGetErrorString(r));
      return (int)r;
    }
  }
  p.capacity = capacity;
  g_mask.fetch_or(1u << kernel_id);
  return 0;
}

int pico_prof_collect(int kernel_id, double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_mu);
  PICO_REQUIRE(kernel_id > 0 && kernel_id < PICO_K_COUNT && (g_mask.load() & (1u << kernel_id)),
               "pico_prof_collect: kernel %d is not enabled", kernel_id);
  Pool& p = g_pool[kernel_id];
  double tot = 0.0;
  for (int i = 0; i < p.used; ++i) {
    hipError_t r = hipEventSynchronize(p.ev[2 * i + 1]);
    if (r != hipSuccess) {
      pico_set_error("pico_prof_collect: %s", hipGetErrorString(r));
      return (int)r;
    }
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, p.ev[2 * i], p.ev[2 * i + 1]);
    tot += ms;
  }
  *total_ms = tot;
  *launches = p.used;
  p.used = 0;
  return 0;
}

}  // extern "C"
