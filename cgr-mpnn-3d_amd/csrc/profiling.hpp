// Optional per-kernel-class timing with HIP events recorded on the launch stream (used by
// bench.py to measure the dominant kernel's average duration live; rocprofv3 must agree).
// Disabled by default: a disabled ProfScope costs one branch.  Never enable it while capturing a
// graph (hipEventCreate is not capture-safe).
#pragma once

#include <hip/hip_runtime.h>

namespace cgr {

bool prof_enabled();
void prof_begin(const char* name, hipStream_t st, void** token);
void prof_end(void* token, hipStream_t st);

struct ProfScope {
  void* tok = nullptr;
  hipStream_t st;
  ProfScope(const char* name, hipStream_t s) : st(s) {
    if (prof_enabled()) prof_begin(name, s, &tok);
  }
  void end() {
    if (tok) prof_end(tok, st);
    tok = nullptr;
  }
  ~ProfScope() { end(); }
};

}  // namespace cgr
