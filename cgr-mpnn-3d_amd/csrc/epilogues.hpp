// GEMM epilogue functors: called once per output element (row, col, accumulator).
#pragma once

#include "common.hpp"

namespace cgr {

// C[r, c] = acc (+ bias[c])
struct EpStore {
  float* C;
  int64_t ld;
  int M, N;
  const float* bias;
  __device__ __forceinline__ void operator()(int r, int c, float v) const {
    if (r < M && c < N) C[(int64_t)r * ld + c] = bias ? v + bias[c] : v;
  }
  // c % 4 == 0; columns >= N are dropped (ld >= round_up(N, 4) for internal buffers)
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    if (r >= M || c >= N) return;
    if (bias) {
      v.x += bias[c];
      if (c + 1 < N) v.y += bias[c + 1];
      if (c + 2 < N) v.z += bias[c + 2];
      if (c + 3 < N) v.w += bias[c + 3];
    }
    float* o = C + (int64_t)r * ld + c;
    if (c + 4 <= N && ((ld & 3) == 0)) {
      *reinterpret_cast<float4*>(o) = v;
    } else {
      o[0] = v.x;
      if (c + 1 < N) o[1] = v.y;
      if (c + 2 < N) o[2] = v.z;
      if (c + 3 < N) o[3] = v.w;
    }
  }
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&) const {
    apply4(r, c, v);
  }
};

// D-MPNN layer (GNN.py:91-102):
//   pre = (m W^T + b) + sigma * h0 ; h = dropout(act(pre))
struct EpLayer {
  const float* bias;
  const float* sigma;  // learnable skip weight (device scalar) or nullptr (= 1, GNN.py:97)
  const float* h0;
  float* hout;
  float* pre;  // nullptr for ReLU (backward uses h > 0)
  int64_t ld;
  int M, N;
  int act;
  uint32_t thresh;  // dropout: keep iff hash >= thresh (0 = no dropout)
  float scale;      // 1 / (1 - p)
  const uint64_t* seed;  // device: the forward's dropout key (arena "rng"); read iff thresh
  int layer;
  __device__ __forceinline__ void operator()(int r, int c, float v) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float sg = sigma ? sigma[0] : 1.f;
    const float z = (v + bias[c]) + sg * h0[o];
    if (pre) pre[o] = z;
    float h = act_fwd(z, act);
    if (thresh) h = drop_keep(*seed, (uint32_t)layer, (uint64_t)r * N + c, thresh) ? h * scale : 0.f;

    else h *= scale;
    hout[o] = h;
  }
  // internal [M, ld] buffers, ld % 4 == 0: whole float4 in bounds of the padded row; columns >= N
  // hold don't-care values (never read as data)
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    if (r >= M || c >= N) return;
    apply4p(r, c, v, *reinterpret_cast<const float4*>(h0 + (int64_t)r * ld + c));
  }
  // h0 prefetch: unconditional load from a clamped in-bounds address (no branch around the load)
  typedef float4 Pre;
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return *reinterpret_cast<const float4*>(h0 + (ok ? (int64_t)r * ld + c : 0));
  }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& hz) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float sg = sigma ? sigma[0] : 1.f;
    float z[4] = {v.x, v.y, v.z, v.w};
    const float h0v[4] = {hz.x, hz.y, hz.z, hz.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (z[k] + bias[min(c + k, N - 1)]) + sg * h0v[k];
    if (pre) *reinterpret_cast<float4*>(pre + o) = make_float4(z[0], z[1], z[2], z[3]);
    float h[4];
    const uint64_t key = thresh ? *seed : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[k] = act_fwd(z[k], act);
      if (thresh)
        h[k] = drop_keep(key, (uint32_t)layer, (uint64_t)r * N + c + k, thresh) ? h[k] * scale
                                                                                 : 0.f;
      else
        h[k] *= scale;
    }
    *reinterpret_cast<float4*>(hout + o) = make_float4(h[0], h[1], h[2], h[3]);
  }
};

// merged x-GEMM output [N, 2H]: columns [0, H) -> P (edge-init half), [H, 2H) -> Q (readout's
// x-part); both internal [N, ld] buffers.
struct EpSplit2 {
  float* P;
  float* Q;
  int64_t ld;
  int M, H;
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    if (r >= M || c >= 2 * H) return;
    if (c + 4 <= H) {
      *reinterpret_cast<float4*>(P + (int64_t)r * ld + c) = v;
    } else if (c >= H) {
      *reinterpret_cast<float4*>(Q + (int64_t)r * ld + (c - H)) = v;  // padding cols don't-care
    } else {  // straddles H (H % 4 != 0)
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cc = c + k;
        if (cc < H) P[(int64_t)r * ld + cc] = e[k];
        else if (cc < 2 * H) Q[(int64_t)r * ld + (cc - H)] = e[k];
      }
    }
  }
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&) const {
    apply4(r, c, v);
  }
};

// readout with the x-part precomputed: hn = act((s W_n[:, F:]^T + Q) + b_n)   (GNN.py:106-107)
struct EpReadoutQ {
  const float* bias;
  const float* Q;
  float* hn;
  float* zn;  // nullptr for ReLU
  int64_t ld;
  int M, N;
  int act;
  typedef float4 Pre;
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return *reinterpret_cast<const float4*>(Q + (ok ? (int64_t)r * ld + c : 0));
  }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& q) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    float z[4] = {v.x + q.x, v.y + q.y, v.z + q.z, v.w + q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] += bias[min(c + k, N - 1)];
    if (zn) *reinterpret_cast<float4*>(zn + o) = make_float4(z[0], z[1], z[2], z[3]);
    *reinterpret_cast<float4*>(hn + o) =
        make_float4(act_fwd(z[0], act), act_fwd(z[1], act), act_fwd(z[2], act), act_fwd(z[3], act));
  }
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    if (r >= M || c >= N) return;
    apply4p(r, c, v, *reinterpret_cast<const float4*>(Q + (int64_t)r * ld + c));
  }
};

// edge_to_node readout (GNN.py:106-107): hn = act([x | s] W_n^T + b_n)
struct EpReadout {
  const float* bias;
  float* hn;
  float* zn;  // nullptr for ReLU
  int64_t ld;
  int M, N;
  int act;
  __device__ __forceinline__ void operator()(int r, int c, float v) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float z = v + bias[c];
    if (zn) zn[o] = z;
    hn[o] = act_fwd(z, act);
  }
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    float z[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] += bias[min(c + k, N - 1)];
    if (zn) *reinterpret_cast<float4*>(zn + o) = make_float4(z[0], z[1], z[2], z[3]);
    *reinterpret_cast<float4*>(hn + o) =
        make_float4(act_fwd(z[0], act), act_fwd(z[1], act), act_fwd(z[2], act), act_fwd(z[3], act));
  }
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&) const {
    apply4(r, c, v);
  }
};

}  // namespace cgr
