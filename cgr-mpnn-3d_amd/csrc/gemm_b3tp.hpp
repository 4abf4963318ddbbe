// Weight-gradient TN GEMM from pre-split operands ("planes"): C[n, k] = sum_e A(e, n) B(e, k)
// with A and B each given as two row-major bf16 planes (hi = bf16(x), lo = bf16(x - hi), written
// by the producers of dpre and of the layer messages) and three products per fp32 product
// (lo.hi, hi.lo, hi.hi: the split of gemm_b3.hpp's TN, the same values).  Compared with
// gemm_b3tn_kernel nothing is split or transposed here:
//   * staging is LDS-DMA only (global_load_lds_dwordx4, lane-linear 1 KB per wave instruction,
//     the tile's layout chosen through the per-lane SOURCE addresses), double-buffered: the DMA of
//     step t + 1 is in flight across the MFMAs of step t, retired by the step's barrier;
//   * fragments come out of LDS already transposed (ds_read_b64_tr_b16: lane i of a 16-lane group
//     receives column i of a 4-row block), two reads per 8-row half-fragment.
// LDS image of one 32-row step, per piece and operand, C columns = NB 16-column blocks:
// sub-blocks (G = row / 8, b) in G-major order, 256 B each: row r8 = row % 8 at slot
// r8 ^ 4 (G & 1) (the two row groups a 32-lane half reads land in opposite bank halves), 32 B
// per row (16 bf16).  A DMA instruction fills 4 consecutive sub-blocks: 8 rows x 128 contiguous
// bytes of the plane.
// Rows: the planes hold round_up(R, 32) rows, rows >= R zero (both operands, so padded products
// are 0 x 0).  The bias gradient (column sums of A) comes from the fp32 A rows: workgroup
// (split, k tile t) sums columns [t SW, (t + 1) SW) of its split, loads issued ahead of the DMA
// so the step's one wait retires both.
#pragma once

#include "gemm_b3.hpp"

namespace cgr {

typedef short b3_s4 __attribute__((ext_vector_type(4)));

struct B3Planes {  // a row-major operand as two bf16 planes [rows][ld]
  const uint16_t* hi;
  const uint16_t* lo;
  int64_t ld;  // elements; a multiple of 8 (16-byte rows pieces)
};

template <int TNN, int TNK>
struct B3TpShape {
  static constexpr int WAVES = 8, NT = 512;
  static constexpr int NBA = TNN, NBB = TNK;  // 16-column blocks per operand
  static constexpr int RN = TNN / WAVES;
  static constexpr int REM = (TNN % WAVES) * TNK;
  static constexpr int RX = (REM + WAVES - 1) / WAVES;
  static constexpr int PIECE_B = (NBA + NBB) * 1024;  // bytes of one piece of one step
  static constexpr int STAGE_B = 2 * PIECE_B;
  static constexpr int NINS = STAGE_B / 1024;  // DMA wave instructions per step
  static constexpr int INS_PER_WAVE = (NINS + WAVES - 1) / WAVES;
  static constexpr size_t LDS_BYTES = (size_t)2 * STAGE_B + 8192;  // + bias partials [<=512] float4
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

__device__ __forceinline__ void b3tp_dma16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds(
      const_cast<void*>(g), reinterpret_cast<__attribute__((address_space(3))) void*>(
                                reinterpret_cast<uintptr_t>(lds)),
      16, 0, 0);
}

__device__ __forceinline__ b3_s4 b3tp_tr(const unsigned char* lds_byte) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      reinterpret_cast<__attribute__((address_space(3))) b3_s4*>(
          reinterpret_cast<uintptr_t>(lds_byte)));
}

// byte offset, inside one operand-piece image, of (row, 16-column block b), for lane group
// reads: row = 8 G + r8
__device__ __forceinline__ int b3tp_off(int NB, int G, int r8, int b) {
  return ((G * NB + b) * 8 + (r8 ^ ((G & 1) << 2))) * 32;
}

// one 16x32 operand fragment (hi or lo piece) of 16-column block b: two transposed reads
__device__ __forceinline__ b3_u4 b3tp_frag(const unsigned char* img, int NB, int b, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const b3_s4 r0 = b3tp_tr(img + b3tp_off(NB, g, q, b) + 8 * p);
  const b3_s4 r1 = b3tp_tr(img + b3tp_off(NB, g, 4 + q, b) + 8 * p);
  const uint32_t w0 = (uint16_t)r0.x | ((uint32_t)(uint16_t)r0.y << 16);
  const uint32_t w1 = (uint16_t)r0.z | ((uint32_t)(uint16_t)r0.w << 16);
  const uint32_t w2 = (uint16_t)r1.x | ((uint32_t)(uint16_t)r1.y << 16);
  const uint32_t w3 = (uint16_t)r1.z | ((uint32_t)(uint16_t)r1.w << 16);
  return b3_u4{w0, w1, w2, w3};
}

#ifndef CGR_B3TP_LAB
#define CGR_B3TP_LAB 0  // lab ablations (tools/b3tp_lab): 1 no MFMA / fragment reads, 2 no DMA
#endif
template <int TNN, int TNK>
__global__ __launch_bounds__(512) void gemm_b3tp_kernel(B3Planes A, B3Planes B,
                                                        const float* __restrict__ a32,
                                                        int64_t lda32, float* __restrict__ slab,
                                                        float* __restrict__ bslab, int Nout,
                                                        int Kout, int R, int rows_per_split,
                                                        int tiles_n, int tiles_k, int want_bias) {
  using S = B3TpShape<TNN, TNK>;
  constexpr int WAVES = S::WAVES, NT = S::NT, RN = S::RN, RX = S::RX, NBA = S::NBA,
                NBB = S::NBB;
  extern __shared__ __attribute__((aligned(16))) unsigned char b3tp_lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / (tiles_n * tiles_k);
  const int tnk = lin - split * tiles_n * tiles_k;
  const int tn = tnk / tiles_k, tkk = tnk - tn * tiles_k;
  const int n0 = tn * TNN * 16, k0 = tkk * TNK * 16;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + 31) / 32 : 0;

  // ---- DMA: wave w issues instructions w, w + WAVES, ... of the step (1 KB each, lane-linear):
  // per lane the element offset of its 16-byte chunk at step 0 (rows advance 32 per step) ----
  const uint16_t* ibase[S::INS_PER_WAVE];
  int64_t ioff[S::INS_PER_WAVE];
  int iins[S::INS_PER_WAVE];
#pragma unroll
  for (int x = 0; x < S::INS_PER_WAVE; ++x) {
    const int ins = w + x * WAVES;
    iins[x] = ins;
    const int ci = (ins < S::NINS ? ins : 0) * 64 + lane;  // chunk index in the stage image
    const int pb = S::PIECE_B / 16;                        // chunks per piece
    const int piece = ci / pb, cp = ci - piece * pb;
    const bool isA = cp < NBA * 64;
    const int NB = isA ? NBA : NBB;
    const int cc = isA ? cp : cp - NBA * 64;
    const int G = cc / (NB * 16), rem = cc - G * NB * 16;
    const int b = rem >> 4, s = (rem >> 1) & 7, half = rem & 1;
    const int row = e_begin + 8 * G + (s ^ ((G & 1) << 2));
    const int col = (isA ? n0 : k0) + 16 * b + 8 * half;
    const B3Planes& P = isA ? A : B;
    ibase[x] = piece ? P.lo : P.hi;
    ioff[x] = (int64_t)row * P.ld + col;
  }
  const int64_t astep = 32 * A.ld, bstep = 32 * B.ld;
  auto dma = [&](int t, int buf) {
    if constexpr ((CGR_B3TP_LAB & 2) != 0) return;
    unsigned char* dst = b3tp_lds + buf * S::STAGE_B;
#pragma unroll
    for (int x = 0; x < S::INS_PER_WAVE; ++x) {
      if (iins[x] < S::NINS) {  // wave-uniform
        const int ci = iins[x] * 64;
        const int pb = S::PIECE_B / 16;
        const int cp = ci % pb;
        const int64_t stp = cp < NBA * 64 ? astep : bstep;
        b3tp_dma16(ibase[x] + ioff[x] + (int64_t)t * stp, dst + iins[x] * 1024);
      }
    }
  };

  // ---- bias: column sums of the fp32 A rows over this split; the tiles_k workgroups of an
  // n tile take SW-column slices of its columns [n0, n0 + 16 TNN) ----
  const int SW = ((16 * TNN + tiles_k - 1) / tiles_k + 3) & ~3;
  const int C4B = SW >> 2;
  const int RSL = C4B > 0 ? NT / C4B : 0;  // row slots
  const int bc4 = C4B > 0 ? tid % C4B : 0, brs = C4B > 0 ? tid / C4B : NT;
  const int bcol = n0 + tkk * SW + 4 * bc4;
  const bool bias_on = want_bias && brs < RSL && bcol < Nout;
  float4 bacc = f4zero();
  float4 braw[2] = {f4zero(), f4zero()};  // rows brs, brs + RSL of a step (RSL >= 16)
  auto bias_load = [&](int t) {
    if (!bias_on) return;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = brs + u * RSL;
      const int e = e_begin + t * 32 + r;
      if (r < 32 && e < e_end) braw[u] = *reinterpret_cast<const float4*>(a32 + (int64_t)e * lda32 + bcol);
      else braw[u] = f4zero();
    }
  };
  auto bias_add = [&]() {
    if (!bias_on) return;
    bacc = f4add(bacc, braw[0]);
    bacc = f4add(bacc, braw[1]);
  };

  floatx4 acc[RN > 0 ? RN : 1][TNK], accx[RX > 0 ? RX : 1];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < TNK; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int x = 0; x < RX; ++x) accx[x] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    if constexpr ((CGR_B3TP_LAB & 1) != 0) return;
    const unsigned char* st = b3tp_lds + buf * S::STAGE_B;
    const unsigned char* aH = st;
    const unsigned char* bH = st + NBA * 1024;
    const unsigned char* aL = st + S::PIECE_B;
    const unsigned char* bL = st + S::PIECE_B + NBA * 1024;
#pragma unroll
    for (int x = 0; x < RX; ++x) {
      const int q = w + x * WAVES;
      const int qq = q < S::REM ? q : 0;
      const int nb = RN * WAVES + qq / TNK, kb = qq % TNK;
      const b3_u4 xah = b3tp_frag(aH, NBA, nb, lane), xal = b3tp_frag(aL, NBA, nb, lane);
      const b3_u4 xbh = b3tp_frag(bH, NBB, kb, lane), xbl = b3tp_frag(bL, NBB, kb, lane);
      floatx4 c = accx[x];
      c = b3_mfma(xal, xbh, c);
      c = b3_mfma(xah, xbl, c);
      accx[x] = b3_mfma(xah, xbh, c);
    }
    if constexpr (RN > 0) {
      b3_u4 ah[RN], al2[RN];
#pragma unroll
      for (int i = 0; i < RN; ++i) {
        ah[i] = b3tp_frag(aH, NBA, w + i * WAVES, lane);
        al2[i] = b3tp_frag(aL, NBA, w + i * WAVES, lane);
      }
#pragma unroll
      for (int j = 0; j < TNK; ++j) {
        const b3_u4 bh = b3tp_frag(bH, NBB, j, lane), bl_ = b3tp_frag(bL, NBB, j, lane);
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          floatx4 c = acc[i][j];
          c = b3_mfma(al2[i], bh, c);
          c = b3_mfma(ah[i], bl_, c);
          acc[i][j] = b3_mfma(ah[i], bh, c);
        }
      }
    }
  };

  if (nt > 0) {
    bias_load(0);
    dma(0, 0);
    __syncthreads();  // (vmcnt(0): the DMA and the bias loads of step 0)
    for (int t = 0; t < nt; ++t) {
      bias_add();
      if (t + 1 < nt) {
        bias_load(t + 1);
        dma(t + 1, (t + 1) & 1);
      }
      compute(t & 1);
      __syncthreads();  // retires step t + 1's DMA; every wave is done with buffer t & 1
    }
  }

  // ---- epilogue: accumulators straight to the slab (rows n = 16 nf + 4 fg + r) ----
  const int ldk = (Kout + 3) & ~3;
  float* out = slab + (int64_t)split * Nout * ldk;
  auto store = [&](int nf, int kf, const floatx4& c) {
    const int col = k0 + kf * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = n0 + nf * 16 + fg * 4 + r;
      if (row < Nout && col < Kout) out[(int64_t)row * ldk + col] = c[r];
    }
  };
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < TNK; ++j) store(w + i * WAVES, j, acc[i][j]);
#pragma unroll
  for (int x = 0; x < RX; ++x) {
    const int q = w + x * WAVES;
    if (q < S::REM) store(RN * WAVES + q / TNK, q % TNK, accx[x]);
  }
  if (want_bias) {  // row slots of a column reduced in slot order (deterministic)
    float4* bp = reinterpret_cast<float4*>(b3tp_lds + 2 * S::STAGE_B);  // [RSL][C4B] <= 512
    // (the stage buffers are dead after the last barrier; bp sits past them)
    if (bias_on) bp[brs * C4B + bc4] = bacc;
    __syncthreads();
    if (tid < C4B) {
      const int col = n0 + tkk * SW + 4 * tid;
      float4 s = f4zero();
      for (int r = 0; r < RSL; ++r) s = f4add(s, bp[r * C4B + tid]);
      const float v[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (col + u < Nout && col + u < n0 + (tkk + 1) * SW && col + u < n0 + 16 * TNN)
          bslab[(int64_t)split * Nout + col + u] = v[u];
    }
  }
}

struct B3TpPlan {
  int tnn, tnk, tiles_n, tiles_k, splits, rows_per_split;
};
inline B3TpPlan plan_b3tp(int Nout, int Kout, int R, int tnn, int tnk, int target_wgs) {
  B3TpPlan p;
  p.tnn = tnn;
  p.tnk = tnk;
  p.tiles_n = (Nout + 16 * tnn - 1) / (16 * tnn);
  p.tiles_k = (Kout + 16 * tnk - 1) / (16 * tnk);
  const int tiles = p.tiles_n * p.tiles_k;
  int splits = target_wgs / tiles;
  const int max_splits = (R + 63) / 64;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + 31) / 32 * 32;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

template <int TNN, int TNK>
inline hipError_t launch_b3tp_t(const B3Planes& A, const B3Planes& B, const float* a32,
                                int64_t lda32, const B3TpPlan& p, float* slab, float* bslab,
                                int Nout, int Kout, int R, bool want_bias, hipStream_t st) {
  using S = B3TpShape<TNN, TNK>;
  auto kern = gemm_b3tp_kernel<TNN, TNK>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.tiles_n * p.tiles_k * p.splits), dim3(S::NT), S::LDS_BYTES, st,
                     A, B, a32, lda32, slab, bslab, Nout, Kout, R, p.rows_per_split, p.tiles_n,
                     p.tiles_k, want_bias ? 1 : 0);
  return hipGetLastError();
}

// plane row pitch (elements) for a width: 16-byte pieces, rows 128-byte aligned
inline int64_t b3tp_ld(int width) { return ((int64_t)width + 63) / 64 * 64; }
inline int64_t b3tp_rows(int64_t R) { return (R + 31) / 32 * 32; }

#ifndef CGR_B3TP_TNN
#define CGR_B3TP_TNN 25  // n fragments per workgroup (25 x 5: A whole, B in 80-column slices)
#endif
#ifndef CGR_B3TP_TNK
#define CGR_B3TP_TNK 5
#endif
#ifndef CGR_B3TP_TARGET
#define CGR_B3TP_TARGET 176
#endif
inline B3TpPlan b3tp_plan(int Nout, int Kout, int R, int target = CGR_B3TP_TARGET) {
  return plan_b3tp(Nout, Kout, R, CGR_B3TP_TNN, CGR_B3TP_TNK, target);
}
// plane row pitch of an H-wide layer operand: covers the TN's n and k tiles and the producing NT
// GEMM's k steps
inline int64_t b3tp_layer_ld(int H) {
  const int64_t a = (int64_t)((H + 16 * CGR_B3TP_TNN - 1) / (16 * CGR_B3TP_TNN)) * 16 * CGR_B3TP_TNN;
  const int64_t b = (int64_t)((H + 16 * CGR_B3TP_TNK - 1) / (16 * CGR_B3TP_TNK)) * 16 * CGR_B3TP_TNK;
  const int64_t c = (int64_t)b3_nk(H) * B3_BK;
  const int64_t m = a > b ? (a > c ? a : c) : (b > c ? b : c);
  return b3tp_ld((int)m);
}

// requirements: the planes cover the tiles' columns (ld >= tiles x 16 x fragments), a32 with
// 16-byte rows, bias row slots >= 16 (a step's 32 rows in two passes)
inline bool b3tp_ok(const B3Planes& A, const B3Planes& B, int64_t lda32, const B3TpPlan& p) {
  const int c4b = ((((16 * p.tnn + p.tiles_k - 1) / p.tiles_k) + 3) & ~3) / 4;
  return A.ld >= (int64_t)p.tiles_n * p.tnn * 16 && B.ld >= (int64_t)p.tiles_k * p.tnk * 16 &&
         A.ld % 8 == 0 && B.ld % 8 == 0 && lda32 % 4 == 0 && c4b > 0 && 512 / c4b >= 16;
}

inline hipError_t launch_b3tp(const B3Planes& A, const B3Planes& B, const float* a32,
                              int64_t lda32, const B3TpPlan& p, float* slab, float* bslab,
                              int Nout, int Kout, int R, bool want_bias, hipStream_t st) {
  if (!b3tp_ok(A, B, lda32, p)) return hipErrorInvalidValue;
  if (p.tnn == 25 && p.tnk == 5)
    return launch_b3tp_t<25, 5>(A, B, a32, lda32, p, slab, bslab, Nout, Kout, R, want_bias, st);
  if (p.tnn == 13 && p.tnk == 13)
    return launch_b3tp_t<13, 13>(A, B, a32, lda32, p, slab, bslab, Nout, Kout, R, want_bias, st);
  if (p.tnn == 8 && p.tnk == 5)
    return launch_b3tp_t<8, 5>(A, B, a32, lda32, p, slab, bslab, Nout, Kout, R, want_bias, st);
  return hipErrorInvalidValue;
}

}  // namespace cgr
