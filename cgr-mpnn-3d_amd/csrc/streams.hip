#include "streams.hpp"

#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>

#include "common.hpp"
#include "gnn_internal.hpp"

namespace cgr {

namespace {
std::mutex g_mu;
SideStreams* g_side[64] = {nullptr};
}  // namespace

bool single_stream() {
  static const bool on = [] {
    const char* v = getenv("CGR_SINGLE_STREAM");
    return v && v[0] == '1';
  }();
  return on;
}

int unpaired_spin_limit() {
  const char* v = getenv("CGR_UNPAIRED_SPIN_LIMIT");
  return v && v[0] ? atoi(v) : kUnpairedSpinLimit;
}

bool prep_split() {
  const char* v = getenv("CGR_PREP_SPLIT");
  return v && v[0] == '1';
}

// Keyed by the device of the caller's stream (the null stream: the current device).  The side
// stream and its events are created on that device, whatever device is current.  The event ring
// is per device; its users hold SideStreams::mu across each forward / backward enqueue, so
// concurrent host threads on one device serialise their enqueues instead of sharing ring events.
SideStreams* side_streams(hipStream_t main) {
  int dev = 0;
  if (main) {
    hipDevice_t d = 0;
    if (hipStreamGetDevice(main, &d) != hipSuccess) {
      set_error("cgr: hipStreamGetDevice failed");
      return nullptr;
    }
    dev = (int)d;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    set_error("cgr: hipGetDevice failed");
    return nullptr;
  }
  if (dev < 0 || dev >= 64) {
    set_error("cgr: device ordinal out of range");
    return nullptr;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_side[dev]) return g_side[dev];
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) return nullptr;
  struct Restore {
    int d;
    bool on;
    ~Restore() {
      if (on) (void)hipSetDevice(d);
    }
  } restore{cur, cur != dev};
  if (cur != dev && hipSetDevice(dev) != hipSuccess) {
    set_error("cgr: hipSetDevice failed");
    return nullptr;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (main && hipStreamIsCapturing(main, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
    set_error("cgr: first native call on this device happened inside a stream capture; run one "
              "eager step before capturing (side streams/events are created lazily)");
    return nullptr;
  }
  SideStreams* s = new SideStreams();
  // the side stream carries the weight-gradient GEMMs and the x-GEMM beside graph prep, at the
  // default priority: the lowest priority made the step 38 % slower (A/B) -- the side stream is
  // the backward's critical path
  if (hipStreamCreateWithPriority(&s->side, hipStreamNonBlocking, 0) != hipSuccess) {
    set_error("cgr: hipStreamCreate failed");
    delete s;
    return nullptr;
  }
  for (auto& e : s->ev) {
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      set_error("cgr: hipEventCreate failed");
      return nullptr;
    }
  }
  s->next = 0;
  s->err_host = nullptr;
  s->dev_err = nullptr;
  void* h = nullptr;
  if (hipHostMalloc(&h, sizeof(int) * kDevErrWords, hipHostMallocMapped | hipHostMallocCoherent) ==
      hipSuccess) {
    memset(h, 0, sizeof(int) * kDevErrWords);
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, h, 0) == hipSuccess) {
      s->err_host = static_cast<int*>(h);
      s->dev_err = static_cast<int*>(dp);
    } else {
      (void)hipHostFree(h);
    }
  }
  s->adam_gate = nullptr;
  if (s->dev_err) {
    void* g = nullptr;
    if (hipMalloc(&g, 64) == hipSuccess && hipMemset(g, 0, 64) == hipSuccess)
      s->adam_gate = static_cast<int*>(g);
  }
  (void)hipGetLastError();  // a failed pinned allocation only disables the error words
  g_side[dev] = s;
  return s;
}

SideStreams* side_streams_of(int dev) {
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  return g_side[dev];
}

hipError_t depend(SideStreams* s, hipStream_t from, hipStream_t to) {
  hipEvent_t e = s->ev[s->next];
  s->next = (s->next + 1) % 16;
  hipError_t r = hipEventRecord(e, from);
  if (r != hipSuccess) return r;
  return hipStreamWaitEvent(to, e, 0);
}

hipError_t record_point(SideStreams* s, hipStream_t from, hipEvent_t* ev) {
  *ev = s->ev[s->next];
  s->next = (s->next + 1) % 16;
  return hipEventRecord(*ev, from);
}

hipError_t fork_to(SideStreams* s, hipStream_t main, hipStream_t side) {
  return depend(s, main, side);
}

}  // namespace cgr
