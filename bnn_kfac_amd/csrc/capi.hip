// Misc C-ABI entry points of libkfac_hip.so.
#include "kfac_common.h"

extern "C" const char* kfac_strerror(int status) {
  switch (status) {
    case KFAC_OK: return "ok";
    case KFAC_EINVAL: return "invalid argument";
    case KFAC_ELAUNCH: return "HIP kernel launch failed";
    case KFAC_EWORKSPACE: return "workspace too small";
    default: return "unknown kfac status";
  }
}

extern "C" const char* kfac_version(void) { return "bnn_kfac_amd 0.1.0 gfx950"; }

// ------------------------------------------------------------------ knobs
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>

#include "knobs.h"

namespace kfac {
namespace {
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
int env_mode(const char* name) {  // -1 auto, 0 off, 1 forced
  const char* v = getenv(name);
  return v && v[0] == '1' ? 1 : v && v[0] == '0' ? 0 : -1;
}
// read at library load (static initialisation of this object)
Knobs g_knobs = [] {
  Knobs k;
  k.syrk3 = env_mode("KFAC_SYRK3");
  k.tiles_x3 = env_mode("KFAC_TILES_X3");
  k.conv_small = env_int("KFAC_CONV_SMALL", 1) != 0;
  k.conv_k = std::max(0, env_int("KFAC_CONV_K", 0));
  k.conv_x3 = env_int("KFAC_CONV_X3", 1) != 0;
  k.inv_graph = env_int("KFAC_INV_GRAPH", 1) != 0;
  k.inv_lookahead = env_int("KFAC_INV_LOOKAHEAD", 1) != 0;
  k.eig_g = std::max(0, env_int("KFAC_EIG_G", 0));
  k.eig_rb = env_int("KFAC_EIG_RB", 4) == 8 ? 8 : 4;
  return k;
}();
}  // namespace
const Knobs& knobs() { return g_knobs; }
}  // namespace kfac

// The per-call knobs (KFAC_INV_GRAPH, KFAC_INV_LOOKAHEAD, KFAC_EIG_G, KFAC_EIG_RB) may be
// changed between calls; the kernel-selection ones are fixed at load (KFAC_EINVAL).
extern "C" int kfac_set_knob(const char* name, int value) {
  if (!name) return KFAC_EINVAL;
  kfac::Knobs& k = kfac::g_knobs;
  if (!strcmp(name, "KFAC_INV_GRAPH")) k.inv_graph = value != 0;
  else if (!strcmp(name, "KFAC_INV_LOOKAHEAD")) k.inv_lookahead = value != 0;
  else if (!strcmp(name, "KFAC_EIG_G") && value >= 0) k.eig_g = value;
  else if (!strcmp(name, "KFAC_EIG_RB") && (value == 4 || value == 8)) k.eig_rb = value;
  else return KFAC_EINVAL;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  return KFAC_OK;
}

extern "C" int kfac_get_knob(const char* name, int* value) {
  if (!name || !value) return KFAC_EINVAL;
  const kfac::Knobs& k = kfac::g_knobs;
  if (!strcmp(name, "KFAC_SYRK3")) *value = k.syrk3;
  else if (!strcmp(name, "KFAC_TILES_X3")) *value = k.tiles_x3;
  else if (!strcmp(name, "KFAC_CONV_SMALL")) *value = k.conv_small;
  else if (!strcmp(name, "KFAC_CONV_K")) *value = k.conv_k;
  else if (!strcmp(name, "KFAC_CONV_X3")) *value = k.conv_x3;
  else if (!strcmp(name, "KFAC_INV_GRAPH")) *value = k.inv_graph;
  else if (!strcmp(name, "KFAC_INV_LOOKAHEAD")) *value = k.inv_lookahead;
  else if (!strcmp(name, "KFAC_EIG_G")) *value = k.eig_g;
  else if (!strcmp(name, "KFAC_EIG_RB")) *value = k.eig_rb;
  else return KFAC_EINVAL;
  return KFAC_OK;
}

// ------------------------------------------------------------------ profiling
#include <mutex>
#include <vector>

namespace kfac {
namespace {
struct Rec {
  int id;
  hipEvent_t start, stop;
  double work;   // algorithmic flops of the scope, 0 if none
  double bytes;  // algorithmic HBM bytes of the scope, 0 if none
};
std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_open;     // started, waiting for their stop
std::vector<Rec> g_done;     // closed pairs, read lazily
std::vector<hipEvent_t> g_pool;

hipEvent_t take() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

bool prof_on() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_on;
}

void prof_begin(int id, hipStream_t s, double work, double bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return;
  Rec r{id, take(), take(), work, bytes};
  if (!r.start || !r.stop) return;
  (void)hipEventRecord(r.start, s);
  g_open.push_back(r);
}

void prof_end(int id, hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_on) return;
  for (size_t i = g_open.size(); i-- > 0;) {
    if (g_open[i].id == id) {
      (void)hipEventRecord(g_open[i].stop, s);
      g_done.push_back(g_open[i]);
      g_open.erase(g_open.begin() + i);
      return;
    }
  }
}
}  // namespace kfac

using namespace kfac;

extern "C" int kfac_profile_enable(int on) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = on != 0;
  return KFAC_OK;
}

extern "C" int kfac_profile_read_work(int id, double* total_ms, int64_t* launches, double* work,
                                      double* bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  double tot = 0.0, wk = 0.0, by = 0.0;
  int64_t cnt = 0;
  for (const Rec& r : g_done) {
    if (r.id != id) continue;
    if (hipEventSynchronize(r.stop) != hipSuccess) return KFAC_ELAUNCH;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.start, r.stop) != hipSuccess) return KFAC_ELAUNCH;
    tot += ms;
    wk += r.work;
    by += r.bytes;
    ++cnt;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = cnt;
  if (work) *work = wk;
  if (bytes) *bytes = by;
  return KFAC_OK;
}

extern "C" int kfac_profile_read(int id, double* total_ms, int64_t* launches) {
  return kfac_profile_read_work(id, total_ms, launches, nullptr, nullptr);
}

// Every HIP object the library keeps across calls -- the inversion's cached graphs,
// their replay events, the profiling event pool -- released while the HIP runtime
// is still up (the Python binding registers it with atexit).  Later calls rebuild
// what they need, so it is also safe mid-process.
int kfac_release_graphs();  // invert.hip

extern "C" int kfac_release(void) {
  int rc = kfac_release_graphs();
  std::lock_guard<std::mutex> lk(g_mu);
  g_on = false;
  for (const Rec& r : g_open) {
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
  }
  for (const Rec& r : g_done) {
    if (hipEventSynchronize(r.stop) != hipSuccess) rc = KFAC_ELAUNCH;
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
  }
  for (hipEvent_t e : g_pool) (void)hipEventDestroy(e);
  g_open.clear();
  g_done.clear();
  g_pool.clear();
  return rc;
}

// ---------------------------------------------------------------- raw events / streams
// The host side's ordering primitives without torch.cuda's Python objects (each of
// those calls costs the caller's thread 5-10 us; these are one ctypes call each).
extern "C" int kfac_event_create(void** ev) {
  if (!ev) return KFAC_EINVAL;
  return hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(ev), hipEventDisableTiming) == hipSuccess
             ? KFAC_OK
             : KFAC_ELAUNCH;
}
// flags bit 0: an ordering-only event (hipEventDisableSystemFence): no system-scope
// release / acquire when it is recorded or waited on -- for events that only order one
// stream after another on the same device; an event the host synchronizes with before
// reading memory the device wrote keeps kfac_event_create's default
extern "C" int kfac_event_create_ex(void** ev, int flags) {
  if (!ev) return KFAC_EINVAL;
  unsigned f = hipEventDisableTiming;
  if (flags & 1) f |= hipEventDisableSystemFence;
  return hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(ev), f) == hipSuccess ? KFAC_OK : KFAC_ELAUNCH;
}
extern "C" int kfac_event_destroy(void* ev) {
  return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? KFAC_OK : KFAC_ELAUNCH;
}
extern "C" int kfac_event_record(void* ev, kfac_stream_t s) {
  return hipEventRecord((hipEvent_t)ev, (hipStream_t)s) == hipSuccess ? KFAC_OK : KFAC_ELAUNCH;
}
extern "C" int kfac_stream_wait_event(kfac_stream_t s, void* ev) {
  return hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)ev, 0) == hipSuccess ? KFAC_OK : KFAC_ELAUNCH;
}
// 1: every work recorded before the event has completed, 0: not yet, < 0: error
extern "C" int kfac_event_query(void* ev) {
  const hipError_t e = hipEventQuery((hipEvent_t)ev);
  return e == hipSuccess ? 1 : e == hipErrorNotReady ? 0 : KFAC_ELAUNCH;
}
extern "C" int kfac_event_synchronize(void* ev) {
  return hipEventSynchronize((hipEvent_t)ev) == hipSuccess ? KFAC_OK : KFAC_ELAUNCH;
}

extern "C" int kfac_profile_reset(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (const Rec& r : g_done) {
    (void)hipEventSynchronize(r.stop);
    g_pool.push_back(r.start);
    g_pool.push_back(r.stop);
  }
  g_done.clear();
  return KFAC_OK;
}
