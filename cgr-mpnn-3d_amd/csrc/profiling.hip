// Event-based per-kernel-class timing (see profiling.hpp) + its C ABI.
#include <stdio.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "gnn_internal.hpp"
#include "profiling.hpp"
#include "stamps.hpp"

namespace cgr {
namespace {
struct Rec {
  std::string name;
  hipEvent_t a, b;
};
struct Acc {
  long count = 0;
  double total_ms = 0.0;
};
bool g_on = false;
std::vector<Rec*> g_pending;
std::vector<hipEvent_t> g_pool;
std::map<std::string, Acc> g_acc;

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  // timing-only events: no system-scope release when recorded, so a bracket measures the launch
  // and not the write-back of the L2 lines it left dirty (which the default event's release
  // performs before its timestamp; HIP's own advice for timing events)
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

bool prof_enabled() { return g_on; }

void prof_begin(const char* name, hipStream_t st, void** token) {
  Rec* r = new Rec{name, get_event(), get_event()};
  if (!r->a || !r->b) {
    delete r;
    *token = nullptr;
    return;
  }
  (void)hipEventRecord(r->a, st);
  *token = r;
}

void prof_end(void* token, hipStream_t st) {
  Rec* r = static_cast<Rec*>(token);
  (void)hipEventRecord(r->b, st);
  g_pending.push_back(r);
}

#ifdef CGR_STAMPS
// setters of the per-translation-unit stamp buffer pointers (stamps.hpp)
static std::vector<StampSetter>& stamp_setters() {
  static std::vector<StampSetter> v;
  return v;
}
void stamp_register(StampSetter f) { stamp_setters().push_back(f); }
#endif

}  // namespace cgr

using namespace cgr;

extern "C" {

int cgr_profile_enable(int32_t on) {
  g_on = on != 0;
  return 0;
}

int cgr_profile_collect(void) {
  for (Rec* r : g_pending) {
    HIP_RET(hipEventSynchronize(r->b));
    float ms = 0.f;
    HIP_RET(hipEventElapsedTime(&ms, r->a, r->b));
    Acc& a = g_acc[r->name];
    a.count += 1;
    a.total_ms += ms;
    g_pool.push_back(r->a);
    g_pool.push_back(r->b);
    delete r;
  }
  g_pending.clear();
  return 0;
}

void cgr_profile_reset(void) {
  cgr_profile_collect();
  g_acc.clear();
}

int64_t cgr_profile_report(char* buf, int64_t len) {
  std::string s;
  char line[256];
  for (auto& kv : g_acc) {
    snprintf(line, sizeof(line), "%s %ld %.6f\n", kv.first.c_str(), kv.second.count,
             kv.second.total_ms);
    s += line;
  }
  if (buf && len > 0) {
    const size_t n = s.size() < (size_t)(len - 1) ? s.size() : (size_t)(len - 1);
    memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int64_t)s.size() + 1;
}

int cgr_debug_stamps(void* buffer, int64_t records) {
#ifdef CGR_STAMPS
  if (records < 0 || records > 0x7fffffff) {
    set_error("cgr_debug_stamps: records out of range");
    return CGR_ERR_INVALID_ARGUMENT;
  }
  for (StampSetter f : stamp_setters())
    HIP_RET(f(static_cast<unsigned long long*>(buffer), (unsigned int)records));
  return 0;
#else
  (void)buffer;
  (void)records;
  set_error("cgr_debug_stamps: not a stamp build (compile with -DCGR_STAMPS)");
  return CGR_ERR_UNSUPPORTED;
#endif
}

}  // extern "C"
