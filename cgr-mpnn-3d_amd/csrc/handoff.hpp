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

// Segment structure of a row tile (BM <= 128 dst-sorted rows): bit r of the 128-bit mask
// {lo, hi} is set when row r starts a dst segment in the tile (r == 0, dst(r) != dst(r - 1), or
// r >= the tile's row count: sentinels), built by one __ballot per wave before the epilogue's
// first barrier.  A row's segment [seg_first, seg_end) then costs a few scalar bit operations
// instead of a serial walk over LDS.
__device__ __forceinline__ bool seg_bit(uint64_t lo, uint64_t hi, int r) {
  return r < 64 ? (lo >> r) & 1 : (hi >> (r - 64)) & 1;
}
__device__ __forceinline__ int seg_first(uint64_t lo, uint64_t hi, int r) {
  if (r >= 64) {
    const uint64_t b = hi & (~0ull >> (127 - r));
    if (b) return 127 - __builtin_clzll(b);
    return 63 - __builtin_clzll(lo);
  }
  return 63 - __builtin_clzll(lo & (~0ull >> (63 - r)));  // bit 0 is always set
}
__device__ __forceinline__ int seg_end(uint64_t lo, uint64_t hi, int r) {
  if (r < 63) {
    const uint64_t b = lo & (~0ull << (r + 1));
    if (b) return __builtin_ctzll(b);
  }
  if (r < 127) {
    const uint64_t b = r < 63 ? hi : hi & (~0ull << (r - 63));
    if (b) return 64 + __builtin_ctzll(b);
  }
  return 128;
}

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
