// Deterministic split-K slab reduction, one output item per thread: shared by the flat reduce
// launch (kernels.hip) and the launch-boundary reduce in the split-bf16 TN's prologue
// (gemm_b3.hpp), which folds the previous weight gradient's slabs into the next TN launch.
#pragma once

#include "common.hpp"
#include "kernels.hpp"

namespace cgr {

// items of a job: Nout * round4(Kout) / 4 float4 outputs, then Nout bias sums (if bias_dst)
__host__ __device__ inline int64_t reduce_items(const RedJob& J) {
  return (int64_t)J.Nout * (((J.Kout + 3) & ~3) >> 2) + (J.bias_dst ? J.Nout : 0);
}

// item f: the loads of all splits are issued before they are summed, in split order p = 0..S-1
// (fixed order: deterministic, no LDS, no barrier)
__device__ __forceinline__ void reduce_slab_item(const RedJob& J, int64_t f) {
  const int ldk = (J.Kout + 3) & ~3;
  const int c4n = ldk >> 2;
  const int64_t nf = (int64_t)J.Nout * c4n;
  if (f < nf) {
    const float4* s4 = reinterpret_cast<const float4*>(J.slab) + f;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = 0;
    for (; p + 8 <= J.splits; p += 8) {
      float4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = s4[(int64_t)(p + q) * nf];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s.x += v[q].x;
        s.y += v[q].y;
        s.z += v[q].z;
        s.w += v[q].w;
      }
    }
    for (; p < J.splits; ++p) {
      const float4 v = s4[(int64_t)p * nf];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    const int64_t n = f / c4n;
    const int k = (int)(f - n * c4n) * 4;
    float* o = J.dst + n * J.ld_dst + J.col_off;
    const float tv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int kk = k + q;
      if (kk >= J.Kout || (kk >= J.gap_at && kk < J.gap_at + J.gap_len)) continue;
      o[kk >= J.gap_at + J.gap_len ? kk - J.gap_len : kk] = tv[q];
    }
  } else if (J.bias_dst && f - nf < J.Nout) {
    const int n = (int)(f - nf);
    float s = 0.f;
    for (int p = 0; p < J.splits; ++p) s += J.bslab[(int64_t)p * J.Nout + n];
    J.bias_dst[n] = s;
  }
}

}  // namespace cgr
