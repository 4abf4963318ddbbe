// Host-side tile / vector-width selection shared by forward, backward and workspace sizing.
//
// GEMM families (one per shape class, picked per call site by same-box A/B of the whole step,
// DESIGN.md §4):
//   gemm_b3.hpp   split-bf16 NT (every NT GEMM of the model) and TN (layer / node / readout
//                 weight gradients whose output rows fit one workgroup)
//   gemm_tnr.hpp  register-direct fp32 TN (weight gradients of shapes the split TN does not cover)
//   gemm.hpp      LDS-staged fp32 NT / TN (standalone DMPNNConv, the edge-feature weight gradient
//                 with K = Fe = 14, and any remaining shape)
#pragma once

#include <stdint.h>

#include <type_traits>

#include "gemm.hpp"
#include "gemm_b3.hpp"
#include "gemm_tnr.hpp"

namespace cgr {

template <int V>
using IC = std::integral_constant<int, V>;

// widest of {4, 2, 1} such that every row starts VEC-aligned (ld, pointer) and the VEC-wide
// chunk holding the last logical element stays inside the row (round_up(K, VEC) <= ld): the
// loaders read whole chunks and mask elements >= K
inline int vec_for(const void* p, int64_t ld, int64_t K) {
  const uintptr_t a = (uintptr_t)p;
  if (ld % 4 == 0 && (K + 3) / 4 * 4 <= ld && a % 16 == 0) return 4;
  if (ld % 2 == 0 && K % 2 == 0 && a % 8 == 0) return 2;
  return 1;
}

template <class F>
inline auto with_vec(int v, F&& f) {
  if (v == 4) return f(IC<4>{});
  if (v == 2) return f(IC<2>{});
  return f(IC<1>{});
}

// fp32 NT GEMM: 4 waves (BM = 64 rows), RN column fragments: 5 when the output width tiles by 80
// (H = 400 -> 5 tiles, no waste), else 4 (BN = 64).
template <class F>
inline auto with_nt_rn(int N, F&& f) {
  if (N % 80 == 0) return f(IC<5>{});
  return f(IC<4>{});
}

// fp32 TN GEMM: WAVES from the output-row count (= H), RN from the output-column count.
template <class F>
inline auto with_tn_shape(int Nout, int Kout, F&& f) {
  if (Nout % 80 == 0) {
    if (Kout <= 16) return f(IC<5>{}, IC<1>{});
    if (Kout % 80 == 0) return f(IC<5>{}, IC<5>{});
    return f(IC<5>{}, IC<4>{});
  }
  if (Kout <= 16) return f(IC<4>{}, IC<1>{});
  if (Kout % 80 == 0) return f(IC<4>{}, IC<5>{});
  return f(IC<4>{}, IC<4>{});
}

// LDS-staged fp32 TN: floor(target / tiles) splits, 4 workgroups per CU (A/B: step-neutral vs
// 768, isolated weight gradient -20 %)
constexpr int kTnTargetWorkgroups = 1024;
// edge-feature weight gradient (K = 14) beside the node TN: fewer splits, fewer CUs taken from
// it (A/B 1024 -> 256 -0.3 %, 128 +0.4 %, 64 +2 %)
constexpr int kEdgeTnTargetWorkgroups = 256;

template <int W, int RM, int RN, int KT, class AL, class BL, class EP>
inline hipError_t launch_nt(const AL& al, const BL& bl, const EP& ep, int M, int N, int K,
                            hipStream_t st) {
  return launch_gemm_nt<W, RM, RN, KT>(al, bl, ep, M, N, K, st);
}

inline TnPlan tn_plan(int Nout, int Kout, int R, int target = kTnTargetWorkgroups) {
  return with_tn_shape(Nout, Kout, [&](auto W, auto RN) {
    return plan_tn<decltype(W)::value, 1, decltype(RN)::value, 1>(Nout, Kout, R, target);
  });
}

template <int W, int RN, class AL, class BL>
inline hipError_t launch_tn(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                            float* bslab, int Nout, int Kout, int R, bool want_bias,
                            hipStream_t st) {
  return launch_gemm_tn<W, 1, RN, 1>(al, bl, p, slab, bslab, Nout, Kout, R, want_bias, st);
}

// Register-direct fp32 TN (gemm_tnr.hpp): fragments per lane 5 (H % 5 == 0: 80 x 80 tiles) or 4.
// Split targets: layer 512 (2 workgroups per CU: floor(512 / 25 tiles) = 20 splits), node 512,
// readout 256 (1 workgroup per CU beside the main-stream tail; A/B +0.5 %).
constexpr int kTnrLayerTarget = 512;
constexpr int kTnrNodeTarget = 512;
constexpr int kTnrReadoutTarget = 256;
inline int tnr_layer_frags(int H) {
  if (tnr_ok<5, 5>(H, H)) return 5;
  if (tnr_ok<4, 4>(H, H)) return 4;
  return 0;
}
// x-side weight gradients (node: Gs^T x, readout: dzn^T [x | s]), 80 x 64 tiles: H % 5 == 0, the
// x columns padded to 16-byte rows (Fx % 4 == 0)
inline bool tnr_x_ok(int H, int Kx, int64_t ldx, const void* x) {
  return tnr_ok<5, 4>(H, Kx) && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
}

// Split-bf16 TN (gemm_b3.hpp) workgroup targets: readout beside the critical readout NT 112
// (A/B +0.7 % vs 176, 64 -6 %), node (the backward's tail) 256 (+0.7 % vs 176, 352 -0.8 %)
constexpr int kB3TnReadoutTarget = 112;
constexpr int kB3TnNodeTarget = 256;
inline TnPlan b3tn_tnplan(int Nout, int Kout, int R, int target = kB3TnTarget) {
  const B3TnPlan q = b3tn_plan(Nout, Kout, R, target);
  return TnPlan{1, q.tiles_k, q.splits, q.rows_per_split};
}

}  // namespace cgr
