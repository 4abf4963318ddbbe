// GEMM epilogue functors: called once per output element (row, col, accumulator).
#pragma once

#include "common.hpp"
#include "prep_one.hpp"

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
  // Epilogue protocol of the GEMM kernels: ctx(c) = the constants of the float4 column group at
  // c (loaded once per thread: the split-bf16 NT keeps one column group per thread), pre4(r, c) =
  // the row operands of one float4 piece (issued for a whole tile before the accumulators go
  // through LDS), apply4p = the arithmetic and the stores.
  struct Ctx {
    float4 b;
  };
  __device__ __forceinline__ Ctx ctx(int c) const {
    if (!bias) return Ctx{f4zero()};
    return Ctx{make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                           bias[min(c + 3, N - 1)])};
  }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&, const Ctx& cx) const {
    if (r >= M || c >= N) return;
    v = f4add(v, cx.b);
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

// C[rows[r], :] = acc: output rows scattered through a permutation (the edge-feature input
// gradient: sorted edge position r -> the caller's edge id perm[r]).  C is the caller's [M, N]
// tensor (any N: scalar stores unless the row is float4-aligned).
struct EpStorePermRows {
  static constexpr bool kSeg = false;
  float* C;
  int64_t ld;
  int M, N;
  const int* rows;
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx(int) const { return Ctx{}; }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  typedef int Pre;
  __device__ __forceinline__ Pre pre4(int r, int) const { return rows[min(r, M - 1)]; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, Pre pr, const Ctx&) const {
    if (r >= M || c >= N) return;
    float* o = C + (int64_t)pr * ld + c;
    if (c + 4 <= N && (ld & 3) == 0 && ((uintptr_t)C & 15) == 0) {
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
// gscale / nscale (nullable): mean pooling's per-graph 1 / count, mean aggregation's per-node
// 1 / in-degree (ds feeds dh_D = ds[dst] / deg(dst) only)
struct EpStoreRowScale {
  static constexpr bool kSeg = false;
  float* C;
  int64_t ld;
  int M, N;
  const float* dy;
  const int* node_graph;
  const float* gscale = nullptr;
  const float* nscale = nullptr;
  struct Ctx {};
  __device__ __forceinline__ Ctx ctx(int) const { return Ctx{}; }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  typedef float Pre;
  __device__ __forceinline__ Pre pre4(int r, int) const {
    const int rr = min(r, M - 1);
    const int g = node_graph[rr];
    float s = dy ? dy[g] : 1.f;  // (dy null: the A operand already holds it, max pooling)
    if (gscale) s *= gscale[g];
    if (nscale) s *= nscale[rr];
    return s;
  }
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
    Ctx cx = ctx(c);
    finish_ctx(cx);
    apply4p<-1>(r, c, v, pre4(r, c), cx);
  }
  // per column group: bias and the scalars (sigma, dropout key); per piece: h0, an unconditional
  // load from a clamped in-bounds address (no branch around the loads)
  struct Ctx {
    float sg;
    uint64_t key;
    float4 b;
  };
  // ctx(c): the per-column vector loads (issued early); finish_ctx: the workgroup scalars (scalar
  // loads count against lgkmcnt, which every LDS barrier drains: loaded at the epilogue)
  __device__ __forceinline__ Ctx ctx(int c) const {
    return Ctx{1.f, 0ull,
               make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                           bias[min(c + 3, N - 1)])};
  }
  __device__ __forceinline__ void finish_ctx(Ctx& cx) const {
    cx.sg = sigma ? sigma[0] : 1.f;
    cx.key = thresh ? *seed : 0ull;
  }
  struct Pre {
    float4 h0;
  };
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return Pre{*reinterpret_cast<const float4*>(h0 + (ok ? (int64_t)r * ld + c : 0))};
  }
  // A >= 0: the activation as a compile-time constant (the GEMM kernel switches on `act` once,
  // outside its epilogue loop: kAct); A < 0: `act` at run time
  static constexpr bool kAct = true;
  template <int A = -1>
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& p,
                                          const Ctx& cx) const {
    if (r >= M || c >= N) return;
    float z[4] = {v.x, v.y, v.z, v.w};
    const float h0v[4] = {p.h0.x, p.h0.y, p.h0.z, p.h0.w};
    const float bv[4] = {cx.b.x, cx.b.y, cx.b.z, cx.b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (z[k] + bv[k]) + cx.sg * h0v[k];
    finish4<A>(r, c, make_float4(z[0], z[1], z[2], z[3]), cx);
  }
  // pre = z -> act -> dropout -> h stored (and returned); the caller checked r < M, c < N
  template <int A = -1>
  __device__ __forceinline__ float4 finish4(int r, int c, float4 z4, const Ctx& cx) const {
    const int64_t o = (int64_t)r * ld + c;
    const float z[4] = {z4.x, z4.y, z4.z, z4.w};
    if (pre) *reinterpret_cast<float4*>(pre + o) = z4;
    float h[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      h[k] = act_fwd(z[k], A < 0 ? act : A);
      if (thresh)
        h[k] = drop_keep(cx.key, (uint32_t)layer, (uint64_t)r * N + c + k, thresh) ? h[k] * scale
                                                                                    : 0.f;
      else
        h[k] *= scale;
    }
    const float4 hv = make_float4(h[0], h[1], h[2], h[3]);
    st4_nt(hout + o, hv);
    return hv;
  }
  // the addend (b + sigma h0) taken into the accumulators in the GEMM's MFMA layout
  // (gemm_b3nt_kernel kAddend): loads of element (r, c) from clamped in-bounds addresses, then
  // z = (acc + b) + sigma h0 -- the operation order of apply4p, so both forms agree bit for bit
  static constexpr bool kAddend = true;
  __device__ __forceinline__ Ctx ctx_add() const { return Ctx{1.f, 0ull, f4zero()}; }
  __device__ __forceinline__ float add_row(int r, int c) const {
    return h0[(int64_t)(r < M ? r : M - 1) * ld + (c < N ? c : N - 1)];
  }
  __device__ __forceinline__ float add_col(int c) const { return bias[c < N ? c : N - 1]; }
  __device__ __forceinline__ float add_apply(float acc, float h0v, float b, const Ctx& cx) const {
    return (acc + b) + cx.sg * h0v;
  }
  template <int A = -1>
  __device__ __forceinline__ void apply4z(int r, int c, float4 z, const Ctx& cx) const {
    if (r >= M || c >= N) return;
    finish4<A>(r, c, z, cx);
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
  // apply4p / apply4z that also return the stored h (rows / columns outside: v unchanged)
  template <int A = -1>
  __device__ __forceinline__ float4 apply4p_h(int r, int c, float4 v, const Pre& p,
                                              const Ctx& cx) const {
    if (r >= M || c >= N) return v;
    float z[4] = {v.x, v.y, v.z, v.w};
    const float h0v[4] = {p.h0.x, p.h0.y, p.h0.z, p.h0.w};
    const float bv[4] = {cx.b.x, cx.b.y, cx.b.z, cx.b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) z[k] = (z[k] + bv[k]) + cx.sg * h0v[k];
    return this->template finish4<A>(r, c, make_float4(z[0], z[1], z[2], z[3]), cx);
  }
  template <int A = -1>
  __device__ __forceinline__ float4 apply4z_h(int r, int c, float4 z, const Ctx& cx) const {
    if (r >= M || c >= N) return z;
    return this->template finish4<A>(r, c, z, cx);
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
  // the graph bookkeeping as the launch's extra workgroup when side_on (gemm_b3.hpp kSideBlock,
  // prep_one.hpp; gnn_fwd.hip decides)
  static constexpr bool kSideBlock = true;
  int side_on;
  PrepOne prep;
  __device__ __forceinline__ void side(void* lds) const {
    graph_prep_one(prep, static_cast<int*>(lds));
  }
  __host__ __device__ size_t side_lds_bytes() const {
    return (size_t)prep_one_lds_ints(prep.N, prep.E, prep.B) * 4;
  }
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
  __device__ __forceinline__ Ctx ctx(int) const { return Ctx{}; }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
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
  struct Ctx {
    float4 b;
  };
  __device__ __forceinline__ Ctx ctx(int c) const {
    return Ctx{make_float4(bias[min(c, N - 1)], bias[min(c + 1, N - 1)], bias[min(c + 2, N - 1)],
                           bias[min(c + 3, N - 1)])};
  }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  struct Pre {
    float4 q;
  };
  __device__ __forceinline__ Pre pre4(int r, int c) const {
    const bool ok = r < M && c < N;
    return Pre{*reinterpret_cast<const float4*>(Q + (ok ? (int64_t)r * ld + c : 0))};
  }
  static constexpr bool kAct = true;  // see EpLayer
  template <int A = -1>
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre& p,
                                          const Ctx& cx) const {
    if (r >= M || c >= N) return;
    apply4z<A>(r, c, f4add(f4add(v, p.q), cx.b), cx);
  }
  // the addend (Q + b) taken into the accumulators in MFMA layout (gemm_b3nt_kernel kAddend),
  // z = (acc + Q) + b in apply4p's order
  static constexpr bool kAddend = true;
  __device__ __forceinline__ Ctx ctx_add() const { return Ctx{f4zero()}; }
  __device__ __forceinline__ float add_row(int r, int c) const {
    return Q[(int64_t)(r < M ? r : M - 1) * ld + (c < N ? c : N - 1)];
  }
  __device__ __forceinline__ float add_col(int c) const { return bias[c < N ? c : N - 1]; }
  __device__ __forceinline__ float add_apply(float acc, float q, float b, const Ctx&) const {
    return (acc + q) + b;
  }
  template <int A = -1>
  __device__ __forceinline__ void apply4z(int r, int c, float4 z4, const Ctx&) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float z[4] = {z4.x, z4.y, z4.z, z4.w};
    const int ac = A < 0 ? act : A;
    if (zn) *reinterpret_cast<float4*>(zn + o) = make_float4(z[0], z[1], z[2], z[3]);
    *reinterpret_cast<float4*>(hn + o) =
        make_float4(act_fwd(z[0], ac), act_fwd(z[1], ac), act_fwd(z[2], ac), act_fwd(z[3], ac));
  }
  __device__ __forceinline__ void apply4(int r, int c, float4 v) const {
    apply4p<-1>(r, c, v, pre4(r, c), ctx(c));
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
  __device__ __forceinline__ Ctx ctx(int) const { return Ctx{}; }
  __device__ __forceinline__ void finish_ctx(Ctx&) const {}
  struct Pre {};
  __device__ __forceinline__ Pre pre4(int, int) const { return Pre{}; }
  __device__ __forceinline__ void apply4p(int r, int c, float4 v, const Pre&, const Ctx&) const {
    apply4(r, c, v);
  }
};

}  // namespace cgr
