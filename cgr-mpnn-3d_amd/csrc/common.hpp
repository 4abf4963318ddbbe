// Shared device helpers for the CGR-MPNN-3D HIP kernels (gfx950 / CDNA4 only).
//
// Conventions (DESIGN.md "Data layout in HBM"):
//   * every per-edge activation is an [E, Hp] fp32 row-major matrix in *dst-sorted* edge order
//     (position i, see graph_prep.hip); every per-node activation is [N, Hp]; Hp = round_up(H, 4)
//     so rows are 16-byte aligned and all internal loads are float4;
//   * external tensors (x, edge_attr, weights) keep the caller's layout; loaders read them with a
//     vector width VEC in {4, 2, 1} chosen on the host from the leading dimension and alignment.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

namespace cgr {

typedef float floatx4 __attribute__((ext_vector_type(4)));
// a float4 store marked non-temporal (global_store_dwordx4 ... nt): the forward layer GEMM's h and
// a rows, streamed out by every workgroup's epilogue at once (same-box A/B +0.8 % on the step,
// profiles/r05_nt_store_ab.txt; the backward's dpre rows stored this way ran 0.4 % slower)
__device__ __forceinline__ void st4_nt(float* p, const float4& v) {
  __builtin_nontemporal_store(floatx4{v.x, v.y, v.z, v.w}, reinterpret_cast<floatx4*>(p));
}

// activation_fn of GNN.__init__ (reference GNN.py:21,127: any callable).  ReLU and SiLU have
// kernels specialised at compile time; GELU and the rest share one runtime-selected slot (the
// kernels' third instantiation, `A = -1`), with torch's default parameters: ELU alpha 1,
// leaky_relu slope 0.01, softplus beta 1 / threshold 20, SELU's fixed constants.
enum Act : int {
  ACT_RELU = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_TANH = 3, ACT_SIGMOID = 4, ACT_ELU = 5,
  ACT_LEAKY_RELU = 6, ACT_SOFTPLUS = 7, ACT_MISH = 8, ACT_SELU = 9, ACT_COUNT = 10
};
constexpr float kSeluAlpha = 1.6732632423543772848f, kSeluScale = 1.0507009873554804934f;

__device__ __forceinline__ float softplus1(float z) { return z > 20.f ? z : log1pf(expf(z)); }

// codes 3-9: out of line, so the fused kernels that carry the runtime slot keep GELU's register
// budget and code size (inlined, the switch grew the fused layer backward by 13 us per launch)
__device__ __attribute__((noinline)) static float act_fwd_ext(float z, int act) {
  switch (act) {
    case ACT_TANH: return tanhf(z);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-z));
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    case ACT_LEAKY_RELU: return z > 0.f ? z : 0.01f * z;
    case ACT_SOFTPLUS: return softplus1(z);
    case ACT_MISH: return z * tanhf(softplus1(z));
    default: return kSeluScale * (z > 0.f ? z : kSeluAlpha * expm1f(z));  // ACT_SELU
  }
}

// leaky_relu / ELU / SELU take the negative branch at z == 0 as ATen's backward does
__device__ __attribute__((noinline)) static float act_grad_ext(float z, int act) {
  switch (act) {
    case ACT_TANH: {
      const float t = tanhf(z);
      return 1.f - t * t;
    }
    case ACT_SIGMOID: {
      const float s = 1.f / (1.f + expf(-z));
      return s * (1.f - s);
    }
    case ACT_ELU: return z > 0.f ? 1.f : expf(z);
    case ACT_LEAKY_RELU: return z > 0.f ? 1.f : 0.01f;
    case ACT_SOFTPLUS: return z > 20.f ? 1.f : 1.f / (1.f + expf(-z));
    case ACT_MISH: {
      const float t = tanhf(softplus1(z));
      const float s = 1.f / (1.f + expf(-z));
      return t + z * s * (1.f - t * t);
    }
    default: return z > 0.f ? kSeluScale : kSeluScale * kSeluAlpha * expf(z);  // ACT_SELU
  }
}

__device__ __forceinline__ float act_fwd(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? z : 0.f;
  if (act == ACT_SILU) return z / (1.f + __expf(-z));
  // GELU, exact erf form (F.gelu default approximate='none')
  if (act == ACT_GELU) return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
  return act_fwd_ext(z, act);
}

// d act / dz.  ReLU: 0 at z == 0 (ATen threshold_backward).
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SILU) {
    const float s = 1.f / (1.f + __expf(-z));
    return s * (1.f + z * (1.f - s));
  }
  if (act == ACT_GELU) {
    const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
    return cdf + z * pdf;
  }
  return act_grad_ext(z, act);
}

// Counter-based dropout RNG: keep(seed, layer, element) is a pure function, so the backward
// regenerates the mask instead of storing it.  32-bit integer hash (Wellons' lowbias32
// finaliser) of a Weyl sequence over the element index, keyed per (seed, layer): ~10 VALU per
// element where a splitmix64 finaliser (64-bit multiplies) took ~30 -- the mask is evaluated for
// all E*H elements in both the layer epilogue and layer_act_bwd.  Bijective in the low 32 index
// bits for a fixed key; keep fractions and neighbour / cross-layer / cross-seed correlations
// measured at the 1/sqrt(n) noise floor over 6.1M elements.
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, uint32_t layer, uint64_t idx) {
  const uint32_t k = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + layer * 0x9E3779B9u));
  uint32_t x = (uint32_t)idx * 0x9E3779B1u + k;
  x ^= (uint32_t)(idx >> 32) * 0x85EBCA77u;
  return mix32(x);
}

// keep with probability 1-p: hash >= p * 2^32
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint32_t layer, uint64_t idx,
                                          uint32_t thresh) {
  return drop_hash(seed, layer, idx) >= thresh;
}

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// float4 t of x rows padded to ldp (c4n = ldp / 4 per row): xp[r, 4k .. 4k + 3] = x[r, 4k ..] or 0
// past F; vec2: F even and x 8-byte aligned (two 8-byte loads, the float2 past F is zeros)
__device__ __forceinline__ void pad_row4(const float* __restrict__ x, int F, float* __restrict__ xp,
                                         int ldp, int c4n, int64_t t, bool vec2) {
  const int64_t r = t / c4n;
  const int k = 4 * (int)(t - r * c4n);
  const float* src = x + r * F;
  float4 v;
  if (vec2) {
    const float2 u = k < F ? *reinterpret_cast<const float2*>(src + k) : make_float2(0.f, 0.f);
    const float2 w = k + 2 < F ? *reinterpret_cast<const float2*>(src + k + 2) : make_float2(0.f, 0.f);
    v = make_float4(u.x, u.y, w.x, w.y);
  } else {
    v.x = k < F ? src[k] : 0.f;
    v.y = k + 1 < F ? src[k + 1] : 0.f;
    v.z = k + 2 < F ? src[k + 2] : 0.f;
    v.w = k + 3 < F ? src[k + 3] : 0.f;
  }
  *reinterpret_cast<float4*>(xp + r * ldp + k) = v;
}
__device__ __forceinline__ float4 f4sub(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}
__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 f4scale(float4 a, float s) {
  return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}

// Load 4 consecutive floats p[0..3] of a row whose valid length from p is `valid` (elements at
// index >= valid read as 0).  VEC = guaranteed alignment/divisibility of the row and of the
// logical length: sub-chunks of VEC are either fully valid or fully invalid.
template <int VEC>
__device__ __forceinline__ float4 load4(const float* __restrict__ p, int valid) {
  if constexpr (VEC == 4) {
    if (valid <= 0) return f4zero();
    float4 v = *reinterpret_cast<const float4*>(p);
    if (valid < 4) {  // only internal [*, Hp] rows (Hp = round_up(H, 4)) reach this
      if (valid < 2) v.y = 0.f;
      if (valid < 3) v.z = 0.f;
      v.w = 0.f;
    }
    return v;
  } else if constexpr (VEC == 2) {
    float4 r = f4zero();
    if (valid > 0) {
      const float2 u = *reinterpret_cast<const float2*>(p);
      r.x = u.x;
      r.y = valid > 1 ? u.y : 0.f;
    }
    if (valid > 2) {
      const float2 u = *reinterpret_cast<const float2*>(p + 2);
      r.z = u.x;
      r.w = valid > 3 ? u.y : 0.f;
    }
    return r;
  } else {
    float4 r;
    r.x = valid > 0 ? p[0] : 0.f;
    r.y = valid > 1 ? p[1] : 0.f;
    r.z = valid > 2 ? p[2] : 0.f;
    r.w = valid > 3 ? p[3] : 0.f;
    return r;
  }
}

// internal [*, Hp] buffers: chunk is always in-bounds of the padded row; zero beyond `valid`
__device__ __forceinline__ float4 load4_masked_internal(const float* __restrict__ p, int valid) {
  if (valid <= 0) return f4zero();
  float4 v = *reinterpret_cast<const float4*>(p);
  if (valid < 4) {
    if (valid < 2) v.y = 0.f;
    if (valid < 3) v.z = 0.f;
    v.w = 0.f;
  }
  return v;
}

__device__ __forceinline__ float f4get(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

__host__ __device__ inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int64_t cdiv(int64_t x, int64_t m) { return (x + m - 1) / m; }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): one static per
// launch-template instantiation, a bit per device ordinal, safe from several host threads
struct LdsLimit {
  std::atomic<uint64_t> done{0};
  hipError_t ensure(const void* kern, int bytes) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
    e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.fetch_or(bit, std::memory_order_acq_rel);
    return e;
  }
};

// Wave-level sum (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// the unpaired form of the fused layer backward (ep_bwd.hpp): its completers' wait bound in polls
// (~0.3 s of s_sleep polling), after which they report a timeout
constexpr int kUnpairedSpinLimit = 1 << 22;
// words of the host-visible error block (pinned host memory mapped into the device, one block per
// device: streams.hip); plain system-scope stores of 1, never read-modify-write across the bus
enum : int { kDevErrUnpairedTimeout = 0, kDevErrUnpairedSeen = 1, kDevErrWords = 16 };

// an A/B toggle read per call: VAR=1 in the environment
inline bool getenv_flag(const char* var) {
  const char* v = getenv(var);
  return v && v[0] == '1';
}

}  // namespace cgr
