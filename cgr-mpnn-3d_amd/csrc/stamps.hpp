// In-kernel phase stamps of the split-bf16 NT GEMM (diagnostic builds only: -DCGR_STAMPS).
//
// Workgroup thread 0 notes the shader clock at the phase boundaries of gemm_b3nt_kernel and its
// epilogues (CGR_STAMP(i), i < 7) in LDS; at the end the workgroup synchronises and thread 0 writes
// one record to the buffer set by cgr_debug_stamps (include/cgr_mpnn3d.h) with a plain vector
// store.  The buffer's first 8 bytes are the record counter (one global atomic per workgroup);
// records follow in ticket order, which keeps each launch's workgroups contiguous on a serial
// stream.  Record (16 x u64):
//   [0] tag | grid << 16   [1] blockIdx | smid << 32   [2] realtime at entry   [3] realtime at end
//   [4 + i] shader clock at stamp i (0 = entry, 7 = end; 0 where a phase did not run)
// In the product build every macro is empty and nothing here is compiled.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef CGR_STAMPS

namespace cgr {

// one copy per translation unit (no relocatable device code): each TU registers its setter
static __device__ unsigned long long* g_stamp_buf;
static __device__ unsigned int g_stamp_cap;

typedef hipError_t (*StampSetter)(unsigned long long*, unsigned int);
void stamp_register(StampSetter f);

static hipError_t stamp_set_local(unsigned long long* p, unsigned int cap) {
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &p, sizeof(p));
  if (e != hipSuccess) return e;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_cap), &cap, sizeof(cap));
}
static const int g_stamp_registered = (stamp_register(&stamp_set_local), 0);

__device__ __forceinline__ unsigned long long* stamp_lds() {
  __shared__ unsigned long long s[10];
  return s;
}

__device__ __forceinline__ void stamp_begin() {
  if (threadIdx.x == 0) {
    unsigned long long* s = stamp_lds();
    for (int i = 0; i < 8; ++i) s[i] = 0;
    s[8] = __builtin_amdgcn_s_memrealtime();
    s[0] = __builtin_amdgcn_s_memtime();
  }
}

__device__ __forceinline__ void stamp_at(int i) {
  if (threadIdx.x == 0) stamp_lds()[i] = __builtin_amdgcn_s_memtime();
}

__device__ __forceinline__ void stamp_end(int tag) {
  __syncthreads();
  if (threadIdx.x == 0 && g_stamp_buf != nullptr) {
    unsigned long long* s = stamp_lds();
    s[7] = __builtin_amdgcn_s_memtime();
    const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
    const unsigned int idx = atomicAdd(reinterpret_cast<unsigned int*>(g_stamp_buf), 1u);
    if (idx < g_stamp_cap) {
      unsigned long long* r = g_stamp_buf + 2 + (size_t)idx * 16;
      r[0] = (unsigned long long)tag | ((unsigned long long)gridDim.x << 16);
      r[1] = (unsigned long long)blockIdx.x | ((unsigned long long)__smid() << 32);
      r[2] = s[8];
      r[3] = rt;
      for (int i = 0; i < 8; ++i) r[4 + i] = s[i];
    }
  }
}

// a value of the caller's into slot i (accumulated cycle counts: gemm_b3tni_kernel)
__device__ __forceinline__ void stamp_val(int i, unsigned long long v) { stamp_lds()[i] = v; }
__device__ __forceinline__ unsigned long long stamp_now() { return __builtin_amdgcn_s_memtime(); }

}  // namespace cgr

#define CGR_STAMP_BEGIN() ::cgr::stamp_begin()
#define CGR_STAMP(i) ::cgr::stamp_at(i)
#define CGR_STAMP_END(tag) ::cgr::stamp_end(tag)

#else

#define CGR_STAMP_BEGIN() ((void)0)
#define CGR_STAMP(i) ((void)0)
#define CGR_STAMP_END(tag) ((void)0)

#endif
