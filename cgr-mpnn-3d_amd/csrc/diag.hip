// Process diagnostics of the C ABI (include/cgr_mpnn3d.h, cgr_debug_abort_backtrace): a SIGABRT
// handler that names the aborting thread and prints its NATIVE stack before handing the signal
// on.  Python's faulthandler prints only Python frames, and for a thread without a Python thread
// state (a HIP runtime thread, RCCL's proxy thread, the c10d watchdog) nothing that identifies it
// -- which is all the round-4 RCCL teardown abort record held.
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <mutex>

#include "../../include/cgr_mpnn3d.h"

namespace {
std::mutex g_mu;
bool g_on = false;
struct sigaction g_prev;

void on_abort(int sig, siginfo_t* si, void* uc) {
  char buf[160];
  char name[32] = {0};
  FILE* f = fopen("/proc/thread-self/comm", "r");  // diagnostics: not async-signal-safe, tolerated
  if (f) {
    if (fgets(name, sizeof name, f)) name[strcspn(name, "\n")] = 0;
    fclose(f);
  }
  const int n = snprintf(buf, sizeof buf,
                         "[cgr] SIGABRT in thread %ld (\"%s\", pid %ld); native backtrace:\n",
                         (long)syscall(SYS_gettid), name, (long)getpid());
  if (n > 0) (void)!write(2, buf, (size_t)n);
  void* frames[64];
  const int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  // hand the signal on: the handler that was installed before (faulthandler's Python dump),
  // or the default action
  sigaction(SIGABRT, &g_prev, nullptr);
  if ((g_prev.sa_flags & SA_SIGINFO) && g_prev.sa_sigaction) {
    g_prev.sa_sigaction(sig, si, uc);
  } else if (g_prev.sa_handler != SIG_DFL && g_prev.sa_handler != SIG_IGN) {
    g_prev.sa_handler(sig);
  }
  signal(SIGABRT, SIG_DFL);
  raise(SIGABRT);
}
}  // namespace

extern "C" int cgr_debug_abort_backtrace(int32_t on) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (on && !g_on) {
    void* warm[2];
    (void)backtrace(warm, 2);  // load the unwinder now, not inside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_abort;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_NODEFER;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGABRT, &sa, &g_prev) != 0) return CGR_ERR_HIP;
    g_on = true;
  } else if (!on && g_on) {
    sigaction(SIGABRT, &g_prev, nullptr);
    g_on = false;
  }
  return CGR_OK;
}
