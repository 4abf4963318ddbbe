// GEMM epilogue functors: called once per output element (row, col, accumulator).
#pragma once

#include "common.hpp"

namespace cgr {

// C[r, c] = acc (+ bias[c])
struct EpStore {
  static constexpr bool kSeg = false;
  float* C;
  int64_t ld;
  int M, N;
  const float* bias;
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
  // prefetched epilogue operands (gemm_nt_kernel issues every pre4 load of a tile before the
  // accumulators go through LDS, so the loads overlap instead of one round trip per float4)
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  typedef float4 Pre;
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    if (!bias) return f4zero();
    return make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                       bias[min(c + 3, N - 1)]);
  }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& b, const Ctx&) const {
    if (r >= M || c >= N) return;
    v = f4add(v, b);
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
};

// C[r, :] = s_r * acc with s_r = dy[node_graph[r]] (readout backward ds = dzn W_n[:, F:], the
// row factor of dzn; LdActGrad).  Internal [M, ld] buffers, ld % 4 == 0.
struct EpStoreRowScale {
  static constexpr bool kSeg = false;
  float* C;
  int64_t ld;
  int M, N;
  const float* dy;
  const int* node_graph;
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  typedef float Pre;
  __device__ __forceinline__ Pre pre4(int r, int) const { return dy[node_graph[min(r, M - 1)]]; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, Pre s, const Ctx&) const {
    if (r >= M || c >= N) return;
    *reinterpret_cast<float4*>(C + (int64_t)r * ld + c) =
        make_float4(s * v.x, s * v.y, s * v.z, s * v.w);
  }
};

// D-MPNN layer (GNN.py:91-102):
//   pre = (m W^T + b) + sigma * h0 ; h = dropout(act(pre))
struct EpLayer {
  static constexpr bool kSeg = false;
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
  // internal [M, ld] buffers, ld % 4 == 0: whole float4 in bounds of the padded row; columns >= N
  // hold don't-care values (never read as data)
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    apply4p(r, c, v, pre4(r, c), ctx());
  }
  // prefetch: h0 and bias of a float4 piece, unconditional loads from clamped in-bounds addresses
  // (no branch around the loads); the scalars (sigma, dropout key) once per workgroup
  struct Ctx {
    float sg;
    uint64_t key;
  };
  __device__ __forceinline__ Ctx ctx() const {
    return Ctx{sigma ? sigma[0] : 1.f, thresh ? *seed : 0ull};
  }
  struct Pre {
    float4 h0, b;
  };
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return Pre{*reinterpret_cast<const float4*>(h0 + (ok ? (int64_t)r * ld + c : 0)),
               make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                           bias[min(c + 3, N - 1)])};
  }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& p,
                                          const Ctx& cx) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    float z[4] = {v.x, v.y, v.z, v.w};
    const float h0v[4] = {p.h0.x, p.h0.y, p.h0.z, p.h0.w};
    const float bv[4] = {p.b.x, p.b.y, p.b.z, p.b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (z[k] + bv[k]) + cx.sg * h0v[k];
    if (pre) *reinterpret_cast<float4*>(pre + o) = make_float4(z[0], z[1], z[2], z[3]);
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[k] = act_fwd(z[k], act);
      if (thresh)
        h[k] = drop_keep(cx.key, (uint32_t)layer, (uint64_t)r * N + c + k, thresh) ? h[k] * scale
                                                                                    : 0.f;
      else
        h[k] *= scale;
    }
    *reinterpret_cast<float4*>(hout + o) = make_float4(h[0], h[1], h[2], h[3]);
  }
};

// EpLayer whose GEMM also produces the layer's scatter-add a[v] = sum_{dst(e) = v} h'[e]
// (GNN.py:134) from its row tile (rows are dst-sorted; gemm_b3nt_kernel's SEG epilogue): the
// "gather -> MLP -> segmented reduce" pass in one launch
struct EpLayerSeg : EpLayer {
  static constexpr bool kSeg = true;
  const int* dst_s;  // [M] node of each (dst-sorted) row
  float* aout;       // [nodes, lda]; crossing / empty segments zeroed beforehand
  int64_t lda;
  float* znext;      // or null: [nodes, lda] whose crossing segments this GEMM zeroes (eval ring)
  // hub segments (over >= 3 row tiles: in-degree > rows per tile + 1), completed in fixed order
  // by their last contributor (gemm_b3nt_kernel, handoff.hpp)
  const int* dst_ptr;  // [nodes + 1] dst CSR of the sorted rows
  float* part;         // [tiles, 2, BN] their partial sums (slot_of)
  int* cnt;            // [nodes * tiles_n] tickets (zero on entry, left zero)
  int tiles_n;
  // apply4p that also returns the stored h (rows / columns outside: v unchanged)
  __device__ __forceinline__ float4 apply4p_h(int r, int c, float4 v, const Pre& p,
                                              const Ctx& cx) const {
    if (r >= M || c >= N) return v;
    const int64_t o = (int64_t)r * ld + c;
    float z[4] = {v.x, v.y, v.z, v.w};
    const float h0v[4] = {p.h0.x, p.h0.y, p.h0.z, p.h0.w};
    const float bv[4] = {p.b.x, p.b.y, p.b.z, p.b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (z[k] + bv[k]) + cx.sg * h0v[k];
    if (pre) *reinterpret_cast<float4*>(pre + o) = make_float4(z[0], z[1], z[2], z[3]);
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[k] = act_fwd(z[k], act);
      if (thresh)
        h[k] = drop_keep(cx.key, (uint32_t)layer, (uint64_t)r * N + c + k, thresh) ? h[k] * scale
                                                                                    : 0.f;
      else
        h[k] *= scale;
    }
    const float4 hv = make_float4(h[0], h[1], h[2], h[3]);
    *reinterpret_cast<float4*>(hout + o) = hv;
    return hv;
  }
};

// merged x-GEMM output [N, 2H]: columns [0, H) -> P (edge-init half), [H, 2H) -> Q (readout's
// x-part); both internal [N, ld] buffers.
struct EpSplit2 {
  static constexpr bool kSeg = false;
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
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&, const Ctx&) const {
    apply4(r, c, v);
  }
};

// readout with the x-part precomputed: hn = act((s W_n[:, F:]^T + Q) + b_n)   (GNN.py:106-107)
struct EpReadoutQ {
  static constexpr bool kSeg = false;
  const float* bias;
  const float* Q;
  float* hn;
  float* zn;  // nullptr for ReLU
  int64_t ld;
  int M, N;
  int act;
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  struct Pre {
    float4 q, b;
  };
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return Pre{*reinterpret_cast<const float4*>(Q + (ok ? (int64_t)r * ld + c : 0)),
               make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                           bias[min(c + 3, N - 1)])};
  }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& p,
                                          const Ctx&) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float4 z4 = f4add(f4add(v, p.q), p.b);
    const float z[4] = {z4.x, z4.y, z4.z, z4.w};
    if (zn) *reinterpret_cast<float4*>(zn + o) = make_float4(z[0], z[1], z[2], z[3]);
    *reinterpret_cast<float4*>(hn + o) =
        make_float4(act_fwd(z[0], act), act_fwd(z[1], act), act_fwd(z[2], act), act_fwd(z[3], act));
  }
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    apply4p(r, c, v, pre4(r, c), ctx());
  }
};

// edge_to_node readout (GNN.py:106-107): hn = act([x | s] W_n^T + b_n)
struct EpReadout {
  static constexpr bool kSeg = false;
  const float* bias;
  float* hn;
  float* zn;  // nullptr for ReLU
  int64_t ld;
  int M, N;
  int act;
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
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx() const { return Ctx{}; }
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&, const Ctx&) const {
    apply4(r, c, v);
  }
};

}  // namespace cgr
