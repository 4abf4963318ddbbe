// Host-side tile / vector-width selection shared by forward, backward and workspace sizing.
#pragma once

#include <stdint.h>

#include <type_traits>

#include "gemm.hpp"
#include "gemm_tn.hpp"
#include "gemm_x3.hpp"
#include "gemm_rs.hpp"
#include "gemm_tnr.hpp"
#include "gemm_b3.hpp"
#include "gemm_b3tp.hpp"

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

// NT GEMM: 4 waves (BM = 64 rows), RN column fragments: 5 when the output width tiles by 80
// (H = 400 -> 5 tiles, no waste), else 4 (BN = 64).
template <class F>
inline auto with_nt_rn(int N, F&& f) {
  if (N % 80 == 0) return f(IC<5>{});
  return f(IC<4>{});
}

// x-GEMM k-tile depth (BK = 16 * KT) and the waves of the node-row (N-row) NT GEMMs
#ifndef CGR_XGEMM_KT
#define CGR_XGEMM_KT 1  // with interleaved loads (CGR_NT_IL) 16-deep tiles win: x-GEMM 119 -> 113 us
#endif
#ifndef CGR_NODE_NT_WAVES
#define CGR_NODE_NT_WAVES 4
#endif

// Edge-row (layer) NT GEMMs: (WAVES, RN).  Default 4 waves x 5 fragments (64 x 80 tiles) when
// H tiles by 80; CGR_NT_WIDE selects 8 waves x 13 fragments (128 x 208 tiles) for A/B runs.
#ifndef CGR_NT_WIDE
#define CGR_NT_WIDE 0
#endif
template <class F>
inline auto with_nt_layer(int N, F&& f) {
#if CGR_NT_WIDE
  if (N > 160) return f(IC<8>{}, IC<13>{});
#endif
  if (N % 80 == 0) return f(IC<4>{}, IC<5>{});
  return f(IC<4>{}, IC<4>{});
}

// TN GEMM: WAVES from the output-row count (= H), RN from the output-column count.
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

#ifndef CGR_TN_KT
#define CGR_TN_KT 1  // TN k-tile depth: BE = 16 * CGR_TN_KT rows per barrier
#endif
#ifndef CGR_TN_TARGET_WGS
#define CGR_TN_TARGET_WGS 1024  // floor(target / tiles) splits: 4 workgroups per CU; step-neutral vs 768 (A/B), isolated wgrad -20%
#endif
constexpr int kTnTargetWorkgroups = CGR_TN_TARGET_WGS;

// TN kernel version: 1 = transposed staging + b128 fragment reads (gemm_tn.hpp; same-box A/B:
// layer wgrad -6% isolated but the step -4% with it, so off), 0 = e-major
// image with b32 reads (gemm.hpp)
#ifndef CGR_TN_V2
#define CGR_TN_V2 0
#endif

// GEMM arithmetic: 1 = fp32 operands split into bf16 hi + lo, three bf16 MFMAs per product
// (gemm_x3.hpp); 0 = exact fp32 MFMA (gemm.hpp / gemm_tn.hpp)
#ifndef CGR_GEMM_X3
#define CGR_GEMM_X3 0
#endif

template <int W, int RM, int RN, int KT, class AL, class BL, class EP>
inline hipError_t launch_nt(const AL& al, const BL& bl, const EP& ep, int M, int N, int K,
                            hipStream_t st) {
#if CGR_GEMM_X3
  return launch_gemm_nt_x3<W, RM, RN>(al, bl, ep, M, N, K, st);
#else
  return launch_gemm_nt<W, RM, RN, KT>(al, bl, ep, M, N, K, st);
#endif
}

// Edge-row layer GEMMs (E x H x H) on the row-block-stationary kernel (gemm_rs.hpp) when the
// shape allows it: lab A/B at cfg2 59 us vs 66-68 us for the 64x80-tile kernel, bitwise-equal
// output (same k order per output).  CGR_RS_LAYER=0 builds the tiled kernel only.
#ifndef CGR_RS_LAYER
#define CGR_RS_LAYER 1
#endif
#ifndef CGR_RS_BWD
#define CGR_RS_BWD 0  // 1: also the layer backward NT (dm = dpre W_l); A/B: no gain beside the side-stream TN kernels (one 1024-thread WG per CU co-schedules poorly)
#endif
#ifndef CGR_RS_RM
#define CGR_RS_RM 2
#endif
inline bool use_rs(int N, int K, int64_t ldb, const void* B) {
  if (!CGR_RS_LAYER || CGR_GEMM_X3 || !rs_ok(N, K, ldb, B)) return false;
  // every column group needs >= 1 fragment: all 16 waves produce A chunks and meet the barriers
  if ((N + 15) / 16 < 4 * CGR_RS_RM) return false;
  const int f = rs_fmax(N, CGR_RS_RM);
  return CGR_RS_RM == 2 ? (f == 1 || f == 4) : (f == 2 || f == 7 || f == 8);
}
template <class F>
inline hipError_t with_rs_fmax(int N, F&& f) {
#if CGR_RS_RM == 2
  switch (rs_fmax(N, 2)) {
    case 1: return f(IC<1>{});
    case 4: return f(IC<4>{});
  }
#else
  switch (rs_fmax(N, 1)) {
    case 2: return f(IC<2>{});
    case 7: return f(IC<7>{});
    case 8: return f(IC<8>{});
  }
#endif
  return hipErrorInvalidValue;
}

// Layer weight gradients (H x H over E rows) on the register-direct TN kernel (gemm_tnr.hpp):
// fragments per lane 5 (H % 5 == 0: H = 400 -> 80 x 80 tiles) or 4; 0 = LDS-staged gemm_tn.
// Lab at cfg2: 61.6 us at 20 splits vs 70 us at 40 splits for gemm_tn (and half the slab bytes).
#ifndef CGR_TNR
#define CGR_TNR 1
#endif
#ifndef CGR_TNR_TARGET_WGS
#define CGR_TNR_TARGET_WGS 512  // 2 workgroups (8 waves) per CU: floor(512 / 25 tiles) = 20 splits
#endif
#ifndef CGR_TNR_NODE_TARGET
#define CGR_TNR_NODE_TARGET CGR_TNR_TARGET_WGS  // node TN (Gs^T x, the backward's tail)
#endif
#ifndef CGR_TNR_RO_TARGET
#define CGR_TNR_RO_TARGET 256  // readout TN (dzn^T [x | s]): 1 WG/CU, runs beside the main-stream tail; A/B +0.5 %
#endif
inline int tnr_layer_frags(int H) {
  if (!CGR_TNR || CGR_GEMM_X3) return 0;
  if (tnr_ok<5, 5>(H, H)) return 5;
  if (tnr_ok<4, 4>(H, H)) return 4;
  return 0;
}

// x-side weight gradients (node: Gs^T x, readout: dzn^T [x | s]) on the register-direct kernel,
// 80 x 64 tiles: H % 5 == 0, the x columns padded to 16-byte rows (Fx % 4 == 0)
#ifndef CGR_TNR_X
#define CGR_TNR_X 1
#endif
#ifndef CGR_TNR_NODE
#define CGR_TNR_NODE 1
#endif
#ifndef CGR_TNR_RO
#define CGR_TNR_RO 1  // isolated 105 -> 80 us; with the main-first stream order (gnn_bwd.hip) the
                      // step is 1.0 % faster (same-box A/B; before that order it was 2-3 % slower)
#endif
inline bool tnr_x_ok(int H, int Kx, int64_t ldx, const void* x) {
  return CGR_TNR_X && CGR_TNR && !CGR_GEMM_X3 && tnr_ok<5, 4>(H, Kx) && ldx % 4 == 0 &&
         ((uintptr_t)x & 15) == 0;
}

// Weight gradients on the split-bf16 TN kernel (gemm_b3.hpp): layer (dpre^T (a[src] - h[rev])),
// node (Gs^T x) and readout (dzn^T [x | s]) when the n side fits one workgroup (b3tn_ok).
// Lab at cfg2 (tools/b3tn_lab): layer 50.6 us vs 60.4 us fp32 register-direct, node 42 vs 62.
#ifndef CGR_B3TN
#define CGR_B3TN 1
#endif
#ifndef CGR_B3TN_RO_TARGET
#define CGR_B3TN_RO_TARGET 112  // readout weight gradient beside the critical readout NT: A/B
                                // 112 +0.7 % vs 176, 64 -6 %
#endif
#ifndef CGR_B3TN_NODE_TARGET
#define CGR_B3TN_NODE_TARGET 256  // node weight gradient, the backward's tail: A/B 256 +0.7 %
                                  // vs 176, 352 -0.8 %
#endif
inline TnPlan b3tn_tnplan(int Nout, int Kout, int R, int target = CGR_B3TN_TARGET) {
  const B3TnPlan q = b3tn_plan(Nout, Kout, R, target);
  return TnPlan{1, q.tiles_k, q.splits, q.rows_per_split};
}

inline TnPlan tn_plan(int Nout, int Kout, int R, int target = kTnTargetWorkgroups) {
  return with_tn_shape(Nout, Kout, [&](auto W, auto RN) {
#if CGR_GEMM_X3
    return plan_tn_x3<decltype(W)::value, 1, decltype(RN)::value>(Nout, Kout, R,
                                                                   target);
#elif CGR_TN_V2
    return plan_tn2<decltype(W)::value, 1, decltype(RN)::value>(Nout, Kout, R,
                                                                 target);
#else
    return plan_tn<decltype(W)::value, 1, decltype(RN)::value, CGR_TN_KT>(Nout, Kout, R,
                                                                           target);
#endif
  });
}

template <int W, int RN, class AL, class BL>
inline hipError_t launch_tn(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                            float* bslab, int Nout, int Kout, int R, bool want_bias,
                            hipStream_t st) {
#if CGR_GEMM_X3
  return launch_gemm_tn_x3<W, 1, RN>(al, bl, p, slab, bslab, Nout, Kout, R, want_bias, st);
#elif CGR_TN_V2
  return launch_gemm_tn2<W, 1, RN>(al, bl, p, slab, bslab, Nout, Kout, R, want_bias, st);
#else
  return launch_gemm_tn<W, 1, RN, CGR_TN_KT>(al, bl, p, slab, bslab, Nout, Kout, R, want_bias, st);
#endif
}

}  // namespace cgr
