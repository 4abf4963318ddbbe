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
  uint64_t seed;
  int layer;
  __device__ __forceinline__ void operator()(int r, int c, float v) const {
    if (r >= M || c >= N) return;
    const int64_t o = (int64_t)r * ld + c;
    const float sg = sigma ? sigma[0] : 1.f;
    const float z = (v + bias[c]) + sg * h0[o];
    if (pre) pre[o] = z;
    float h = act_fwd(z, act);
    if (thresh) h = drop_keep(seed, (uint32_t)layer, (uint64_t)r * N + c, thresh) ? h * scale : 0.f;
    else h *= scale;
    hout[o] = h;
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
};

}  // namespace cgr
