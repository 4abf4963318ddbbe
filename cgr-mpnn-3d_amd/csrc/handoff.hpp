// Workgroup-to-workgroup hand-off of the tile-crossing dst segments of the fused layer GEMMs
// (gemm_b3.hpp EpLayerSeg, ep_bwd.hpp EpLayerBwdSeg): the last of a segment's contributing
// workgroups completes it (cdna_hip_programming.md §6 Guideline 16, counter form).
#pragma once

#include "common.hpp"

namespace cgr {

__device__ __forceinline__ void ep_vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The hand-off below rests on gfx950 behaviour (MI355X_MICROARCH.md "Correctness boundaries",
// valid forms of the sc1 hand-off): agent-scope relaxed atomic stores / loads are the
// write-through / L2-bypassing forms, and vmcnt counts stores.  Refuse any other target.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "handoff.hpp: the sc1 hand-off of tile-crossing segments is written for gfx950 only"
#endif

// row tiles [t0, t1] a dst segment [b, e) touches, and the partial-sum slot of row tile t in the
// per-tile pair (tile t * tiles_n + tn): the first tile holds the segment's head rows at its
// tail end (slot 1), every later tile at its head end (slot 0) -- a middle tile is all one
// segment, its slot 0
__device__ __forceinline__ int seg_tiles(int b, int e, int BM) { return (e - 1) / BM - b / BM + 1; }
__device__ __forceinline__ int slot_of(int t, int t0) { return t == t0 ? 1 : 0; }

// handed-off words (Guideline 16 R1): agent-scope relaxed atomic stores / loads are the sc1
// (write-through / L2-bypassing) forms, so the hand-off needs no release or acquire fence
__device__ __forceinline__ void sc1_store4(float* p, float4 v) {
  __hip_atomic_store(p, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 3, v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 sc1_load4(const float* p) {
  float* q = const_cast<float*>(p);
  return make_float4(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                     __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                     __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                     __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

}  // namespace cgr
