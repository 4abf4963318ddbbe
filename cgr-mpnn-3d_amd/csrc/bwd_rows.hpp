// Per-row pieces of the layer / edge-init backward (GNN.py:85-102 reversed), shared by the
// segmented-sum backward kernels (kernels.hip) and the fused layer-backward GEMM epilogue
// (ep_bwd.hpp).  One call handles one float4 of one edge row i (sorted position), columns n..n+3,
// given dh = dL/dh_{l+1}[i, n..n+3]:
//   layer:      dpre = dh * keep/(1-p) * act'(pre) ; dsig += dpre . h0
//   edge init:  dpre0 = (dh0 + dh) * act'(pre0), dh0 = sum_l sigma_l dpre_l (GNN.py:97: every
//               layer adds sigma_l h0) summed from the layers' dpre buffers, top layer first.
// The operand loads (*_loads) are separate from the arithmetic (*_apply) so callers can issue
// every load of a row group before the first dh is known.
#pragma once

#include "common.hpp"
#include "kernels.hpp"

namespace cgr {

struct RowOps {
  float4 m;    // h_{l+1} (ReLU mask) or pre (other activations); edge init: h_0 or pre_0
  float4 acc;  // edge init: dh0 = sum_l sigma_l dpre_l
  float4 h0;   // h_0 (learnable-skip partials)
};

__device__ __forceinline__ RowOps layer_row_loads(const LayerBwdArgs& a, int64_t i, int n) {
  const int64_t o = i * a.Hp + n;
  RowOps r;
  r.m = *reinterpret_cast<const float4*>((a.act == ACT_RELU ? a.hnext : a.pre) + o);
  r.acc = f4zero();
  r.h0 = a.dsig_part ? *reinterpret_cast<const float4*>(a.h0 + o) : f4zero();
  return r;
}

// A >= 0: the activation as a compile-time constant (one straight-line path per activation, no
// per-element branch tree); A < 0: a.act at run time
template <int A = -1>
__device__ __forceinline__ float4 layer_row_apply(const LayerBwdArgs& a, int64_t i, int n,
                                                  float4 dh, uint64_t key, float& dsig,
                                                  const RowOps& r) {
  const int act = A < 0 ? a.act : A;
  const int64_t o = i * a.Hp + n;
  float d[4] = {dh.x, dh.y, dh.z, dh.w};
  if (act == ACT_RELU) {  // h_{l+1} > 0 <=> relu active and kept by dropout
    const float hh[4] = {r.m.x, r.m.y, r.m.z, r.m.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = hh[k] > 0.f ? d[k] * a.scale : 0.f;
  } else {
    const float zz[4] = {r.m.x, r.m.y, r.m.z, r.m.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float m = a.scale;
      if (a.thresh && n + k < a.H)
        m = drop_keep(key, (uint32_t)a.layer, (uint64_t)i * a.H + n + k, a.thresh) ? a.scale
                                                                                      : 0.f;
      d[k] = d[k] * m * act_grad(zz[k], act);
    }
  }
  const float4 dp = make_float4(d[0], d[1], d[2], d[3]);
  *reinterpret_cast<float4*>(a.dpre + o) = dp;
  if (a.dsig_part) {
    const float hz[4] = {r.h0.x, r.h0.y, r.h0.z, r.h0.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (n + k < a.H) dsig += d[k] * hz[k];
  }
  return dp;
}

__device__ __forceinline__ RowOps edge_row_loads(const LayerBwdArgs& a, int64_t i, int n) {
  const int64_t o = i * a.Hp + n;
  RowOps r;
  r.m = *reinterpret_cast<const float4*>((a.act == ACT_RELU ? a.h0 : a.pre) + o);
  float4 acc = f4zero();
  for (int l = a.nlayers - 1; l >= 0; --l) {
    const float sg = a.sig[l] ? a.sig[l][0] : 1.f;
    const float4 dp = *reinterpret_cast<const float4*>(a.dpre_all + l * a.dpre_stride + o);
    acc.x += sg * dp.x;
    acc.y += sg * dp.y;
    acc.z += sg * dp.z;
    acc.w += sg * dp.w;
  }
  r.acc = acc;
  r.h0 = f4zero();
  return r;
}

template <int A = -1>
__device__ __forceinline__ void edge_row_apply(const LayerBwdArgs& a, int64_t i, int n, float4 dh,
                                               const RowOps& r) {
  const int act = A < 0 ? a.act : A;
  const int64_t o = i * a.Hp + n;
  float4 d = f4add(r.acc, dh);
  if (act == ACT_RELU) {
    d.x = r.m.x > 0.f ? d.x : 0.f;
    d.y = r.m.y > 0.f ? d.y : 0.f;
    d.z = r.m.z > 0.f ? d.z : 0.f;
    d.w = r.m.w > 0.f ? d.w : 0.f;
  } else {
    d.x *= act_grad(r.m.x, act);
    d.y *= act_grad(r.m.y, act);
    d.z *= act_grad(r.m.z, act);
    d.w *= act_grad(r.m.w, act);
  }
  *reinterpret_cast<float4*>(a.dpre + o) = d;
}

// either form, by EDGE_INIT
template <bool EDGE_INIT>
__device__ __forceinline__ RowOps bwd_row_loads(const LayerBwdArgs& a, int64_t i, int n) {
  if constexpr (EDGE_INIT) return edge_row_loads(a, i, n);
  else return layer_row_loads(a, i, n);
}
template <bool EDGE_INIT, int A = -1>
__device__ __forceinline__ void bwd_row_apply(const LayerBwdArgs& a, int64_t i, int n, float4 dh,
                                              uint64_t key, float& dsig, const RowOps& r) {
  if constexpr (EDGE_INIT) edge_row_apply<A>(a, i, n, dh, r);
  else (void)layer_row_apply<A>(a, i, n, dh, key, dsig, r);
}

}  // namespace cgr
