// Diagnostic only (never linked into the product library): a one-wave sampler that records
// (s_memtime, s_memrealtime) pairs every `period` ticks of the 100 MHz real-time clock, launched on
// a stream of its own beside the bench's timed region, so the shader clock the chip held during
// those steps reads as d(s_memtime) / d(s_memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS
// give-back item 6).  Bounded: exactly n samples, then the wave exits.
//   hipcc -O2 --offload-arch=gfx950 -shared -fPIC tools/clock_probe.hip -o tools/_build/libclockprobe.so
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(64) k_clock_sampler(unsigned long long* out, int n,
                                                      unsigned long long period) {
  if (threadIdx.x != 0) return;
  unsigned long long next = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) {
    unsigned long long r;
    do {
      r = __builtin_amdgcn_s_memrealtime();
    } while (r < next);
    unsigned long long s = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    out[2 * i] = s;  // vector stores (global_store), no scalar-cache writes
    out[2 * i + 1] = r;
    next = r + period;
  }
}

extern "C" int clock_probe_launch(void* out, int n, unsigned long long period, void* stream) {
  hipLaunchKernelGGL(k_clock_sampler, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (unsigned long long*)out, n, period);
  return (int)hipGetLastError();
}

// one stamp on the caller's stream between two steps: (s_memtime, s_memrealtime) at entry and
// after `spin` real-time ticks of spinning, so each stamp also reads the shader clock of that moment
__global__ void k_clock_stamp(unsigned long long* out, unsigned long long spin) {
  if (threadIdx.x != 0) return;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long s0 = __builtin_amdgcn_s_memtime();
  unsigned long long r1;
  do {
    r1 = __builtin_amdgcn_s_memrealtime();
  } while (r1 < r0 + spin);
  const unsigned long long s1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  out[0] = r0;
  out[1] = s0;
  out[2] = r1;
  out[3] = s1;
}

extern "C" int clock_probe_stamp(void* out, unsigned long long spin, void* stream) {
  hipLaunchKernelGGL(k_clock_stamp, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (unsigned long long*)out, spin);
  return (int)hipGetLastError();
}
