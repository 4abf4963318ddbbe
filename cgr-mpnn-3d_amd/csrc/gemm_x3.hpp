// fp32 GEMMs on the bf16 matrix cores: split-bf16 NT and TN kernels (gfx950,
// v_mfma_f32_16x16x32_bf16).
//
// Every fp32 operand element is split at LDS-staging time into three bf16 pieces
// x = hi + mid + lo + r: hi = bf16(x) (round to nearest even), mid = bf16(x - hi),
// lo = bf16(x - hi - mid), each remainder exact in fp32, |r| <= 2^-27 |x|.  A product is the sum
// of the six piece products that can reach 2^-16 |ab| (hi.hi, hi.mid, mid.hi, hi.lo, lo.hi,
// mid.mid; the dropped ones are <= 2^-26 |ab|), each bf16 product exact, all of them accumulated
// in fp32 by the MFMA -- an error at the level of fp32 rounding itself.  Storage, epilogues,
// reductions and every other step stay fp32; the results go through the same fp64-oracle parity
// tests as the exact fp32 MFMA path (v_mfma_f32_16x16x4_f32, gemm.hpp; -DCGR_GEMM_X3=0).
// The bf16 MFMA has 16x the fp32 MFMA rate (MI355X_MICROARCH.md § Matrix cores): six of them
// cost 3/8 of the exact path's matrix-core time.  (A two-piece split, three terms, errs ~2^-16
// relative: measured 2.4e-4 relative on a small GELU output and ~2e-2 on a ReLU-masked weight
// gradient -- outside the 1e-4 bar; -DCGR_X3_PIECES=2 keeps it for A/B only.)
//
// LDS images: per 32-deep k slice, operand and piece, [row][4 chunks of 8 bf16], chunk c of row r
// at slot c ^ lds_swz(r) -- the fp32 kernel's 64-byte-row geometry, so each fragment is one
// conflict-free ds_read_b128 (lane l: row l & 15, k = 8 (l >> 4) .. +7).
//   NT: a thread stages 8-element k chunks of rows (two float4 loader fetches, split, one b128
//       store per piece); prefetch distance 2 through registers as in gemm_nt_kernel.
//   TN: the reduction runs over rows e, so a thread stages an 8 (e) x 1 (column) block: eight
//       scalar loader fetches (lanes along the columns: 256-byte coalesced rows), split, one b128
//       store per piece into the column's chunk.  Bias column sums of A are accumulated from the
//       fp32 values in registers and reduced across the 4 e-blocks at the end.
#pragma once

#include "gemm.hpp"

namespace cgr {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx2_t __attribute__((ext_vector_type(2)));

// Number of bf16 pieces per fp32 operand: 3 (x = hi + mid + lo, six MFMA terms, ~fp32 accuracy)
// or 2 (x = hi + lo, three terms, ~2^-16 relative: too coarse for the 1e-4 parity bar on small
// outputs and ReLU-masked gradients -- kept for A/B only).
#ifndef CGR_X3_PIECES
#define CGR_X3_PIECES 3
#endif
constexpr int kPieces = CGR_X3_PIECES;
static_assert(kPieces == 2 || kPieces == 3, "CGR_X3_PIECES must be 2 or 3");

// 2 fp32 -> packed bf16x2 (RNE) and the two values it represents
__device__ __forceinline__ uint32_t bf16_pair(float a, float b, float& fa, float& fb) {
  const uint32_t u =
      __builtin_bit_cast(uint32_t, __builtin_convertvector(floatx2_t{a, b}, bf16x2_t));
  fa = __uint_as_float(u << 16);
  fb = __uint_as_float(u & 0xffff0000u);
  return u;
}

// 8 fp32 -> kPieces packed bf16x8 pieces (element 0 in the low half): piece i = bf16 of the
// remainder after pieces 0..i-1 (every remainder is exact in fp32)
__device__ __forceinline__ void split_bf16x8(const float (&v)[8], uint4 (&out)[kPieces]) {
  uint32_t w[kPieces][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float a = v[2 * p], b = v[2 * p + 1];
#pragma unroll
    for (int i = 0; i < kPieces; ++i) {
      float fa, fb;
      w[i][p] = bf16_pair(a, b, fa, fb);
      a -= fa;
      b -= fb;
    }
  }
#pragma unroll
  for (int i = 0; i < kPieces; ++i) out[i] = make_uint4(w[i][0], w[i][1], w[i][2], w[i][3]);
}

__device__ __forceinline__ floatx4 mfma_bf16(const uint4& a, const uint4& b, const floatx4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

// (piece of A, piece of B) of term t: every pair whose product can reach 2^-16 |a b|, smallest
// first -- 3 pieces: (1,1) (0,2) (2,0) (0,1) (1,0) (0,0); 2 pieces: (1,0) (0,1) (0,0)
constexpr int kTerms = kPieces == 3 ? 6 : 3;
__host__ __device__ constexpr int term_piece_a(int t) {
  return kPieces == 3 ? (t == 0 ? 1 : t == 2 ? 2 : t == 4 ? 1 : 0) : (t == 0 ? 1 : 0);
}
__host__ __device__ constexpr int term_piece_b(int t) {
  return kPieces == 3 ? (t == 0 ? 1 : t == 1 ? 2 : t == 3 ? 1 : 0) : (t == 1 ? 1 : 0);
}

// acc[i][j] += A_i B_j^T over one 32-deep slice.  A / B: kPieces images each (piece stride
// astr / bstr uint4); fragment rows fr, chunk slot sw.  Terms smallest first; the RM * RN
// independent accumulators interleave within each term.
template <int RM, int RN>
__device__ __forceinline__ void x3_slice(floatx4 (&acc)[RM][RN], const uint4* A, int astr,
                                         const uint4* B, int bstr, int arow0, int fr, int sw) {
  uint4 a[kPieces][RM], b[kPieces][RN];
#pragma unroll
  for (int q = 0; q < kPieces; ++q) {
#pragma unroll
    for (int i = 0; i < RM; ++i) a[q][i] = A[q * astr + (arow0 + i * 16 + fr) * 4 + sw];
#pragma unroll
    for (int j = 0; j < RN; ++j) b[q][j] = B[q * bstr + (j * 16 + fr) * 4 + sw];
  }
#pragma unroll
  for (int t = 0; t < kTerms; ++t)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = mfma_bf16(a[term_piece_a(t)][i], b[term_piece_b(t)][j], acc[i][j]);
}

// ------------------------------------------------------------------------------------------
// NT: C[m, n] = sum_k A(m, k) B(n, k), epilogue functor as gemm_nt_kernel
// ------------------------------------------------------------------------------------------
template <int WAVES, int RM, int RN>
struct NTX3Shape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RM, BN = RN * 16, BK = 32;
  static constexpr int ACH = BM * 4, BCH = BN * 4;  // 8-element chunks per stage
  static constexpr int APT = (ACH + NT - 1) / NT, BPT = (BCH + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr int BUF = kPieces * (ACH + BCH);  // one buffer: A pieces, then B pieces
  static constexpr int STAGE_U4 = 2 * BUF;
  static constexpr int EPI_U4 = (BM * LDC + 3) / 4;
  static constexpr int LDS_U4 = STAGE_U4 > EPI_U4 ? STAGE_U4 : EPI_U4;
};

template <int WAVES, int RM, int RN, class AL, class BL, class EP>
__global__ __launch_bounds__(WAVES * 64) void gemm_nt_x3_kernel(AL al, BL bl, EP ep, int M, int N,
                                                                int K, int tiles_n) {
  using S = NTX3Shape<WAVES, RM, RN>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BK = S::BK;
  constexpr int ACH = S::ACH, BCH = S::BCH, APT = S::APT, BPT = S::BPT;
  __shared__ uint4 lds[S::LDS_U4];
  // buffer b at b * BUF: piece q of A at q * ACH, piece q of B at kPieces * ACH + q * BCH
  constexpr int BUF = S::BUF;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  typename AL::Row arow[APT];
  int adst[APT], akof[APT];
  bool ain[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT;
    ain[p] = q < ACH;
    const int r = ain[p] ? q >> 2 : 0, kc = q & 3;
    arow[p] = al.row(m0 + r, M);
    akof[p] = kc * 8;
    adst[p] = r * 4 + (kc ^ lds_swz(r));
  }
  typename BL::Row brow[BPT];
  int bdst[BPT], bkof[BPT];
  bool bin[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    bin[p] = q < BCH;
    const int r = bin[p] ? q >> 2 : 0, kc = q & 3;
    brow[p] = bl.row(n0 + r, N);
    bkof[p] = kc * 8;
    bdst[p] = r * 4 + (kc ^ lds_swz(r));
  }

  struct RawA {
    typename AL::Raw v[2];
  };
  struct RawB {
    typename BL::Raw v[2];
  };
  floatx4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fg ^ lds_swz(fr);

  // chunk guards (ain / bin) are wave-uniform: ACH and BCH are multiples of 64
  auto fetch = [&](RawA(&xa)[APT], RawB(&xb)[BPT], int kb) {
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p]) {
        xa[p].v[0] = al.fetch(arow[p], kb + akof[p], K);
        xa[p].v[1] = al.fetch(arow[p], kb + akof[p] + 4, K);
      }
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p]) {
        xb[p].v[0] = bl.fetch(brow[p], kb + bkof[p], K);
        xb[p].v[1] = bl.fetch(brow[p], kb + bkof[p] + 4, K);
      }
  };
  auto put = [](uint4* img, int stride, int dst, const float4& u, const float4& v) {
    const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
    uint4 pc[kPieces];
    split_bf16x8(f, pc);
#pragma unroll
    for (int q = 0; q < kPieces; ++q) img[q * stride + dst] = pc[q];
  };
  auto sstore = [&](const RawA(&xa)[APT], const RawB(&xb)[BPT], int buf, int kb) {
    uint4* base = lds + buf * BUF;
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p])
        put(base, ACH, adst[p], al.combine(xa[p].v[0], arow[p], kb + akof[p], K),
            al.combine(xa[p].v[1], arow[p], kb + akof[p] + 4, K));
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p])
        put(base + kPieces * ACH, BCH, bdst[p],
            bl.combine(xb[p].v[0], brow[p], kb + bkof[p], K),
            bl.combine(xb[p].v[1], brow[p], kb + bkof[p] + 4, K));
  };
  auto compute = [&](int buf) {
    const uint4* base = lds + buf * BUF;
    x3_slice<RM, RN>(acc, base, ACH, base + kPieces * ACH, BCH, w * 16 * RM, fr, sw);
  };

  // prefetch distance 2 (see gemm_nt_kernel): register sets alternate by tile parity
  RawA ra[APT], ra2[APT];
  RawB rb[BPT], rb2[BPT];
  fetch(ra, rb, 0);
  fetch(ra2, rb2, BK);
  sstore(ra, rb, 0, 0);
  __syncthreads();
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    fetch(ra, rb, (kt + 2) * BK);
    __builtin_amdgcn_sched_barrier(0);
    compute(0);
    __builtin_amdgcn_sched_barrier(0);
    sstore(ra2, rb2, 1, (kt + 1) * BK);
    __syncthreads();
    fetch(ra2, rb2, (kt + 3) * BK);
    __builtin_amdgcn_sched_barrier(0);
    compute(1);
    __builtin_amdgcn_sched_barrier(0);
    sstore(ra, rb, 0, (kt + 2) * BK);
    __syncthreads();
  }
  if (kt < nk) {
    compute(0);
    __syncthreads();
  }

  float* C = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(w * 16 * RM + i * 16 + fg * 4 + r) * S::LDC + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int C4 = BN / 4;
  for (int q = tid; q < BM * C4; q += NT) {
    const int r = q / C4, c4 = q - r * C4;
    const float4 v = *reinterpret_cast<const float4*>(&C[r * S::LDC + 4 * c4]);
    ep.apply4(m0 + r, n0 + 4 * c4, v);
  }
}

template <int WAVES, int RM, int RN, class AL, class BL, class EP>
inline hipError_t launch_gemm_nt_x3(const AL& al, const BL& bl, const EP& ep, int M, int N, int K,
                                    hipStream_t st) {
  using S = NTX3Shape<WAVES, RM, RN>;
  static_assert(S::ACH % 64 == 0 && S::BCH % 64 == 0, "chunk guards must be wave-uniform");
  if (M <= 0 || N <= 0) return hipSuccess;
  const int tm = (M + S::BM - 1) / S::BM, tn = (N + S::BN - 1) / S::BN;
  hipLaunchKernelGGL((gemm_nt_x3_kernel<WAVES, RM, RN, AL, BL, EP>), dim3(tm * tn),
                     dim3(WAVES * 64), 0, st, al, bl, ep, M, N, K, tn);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// TN split-K: C[n, k] = sum_e A(e, n) B(e, k) into fp32 slabs (same plan / slab / bias contract
// as gemm_tn_kernel, so reduce_slabs is shared)
// ------------------------------------------------------------------------------------------
template <int WAVES, int RM, int RN>
struct TNX3Shape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RM, BN = RN * 16, BE = 32;
  static constexpr int NBA = 4 * BM, NBB = 4 * BN;  // 8 x 1 blocks per stage
  static constexpr int APT = (NBA + NT - 1) / NT, BPT = (NBB + NT - 1) / NT;
  static constexpr int ACH = BM * 4, BCH = BN * 4;  // uint4 per image
  static constexpr int LDC = BN + 4;
  static constexpr int BUF = kPieces * (ACH + BCH);
  static constexpr int STAGE_U4 = 2 * BUF;
  static constexpr int EPI_U4 = (BM * LDC + 3) / 4 + BM;  // + bias partials [4][BM] floats
  static constexpr int LDS_U4 = STAGE_U4 > EPI_U4 ? STAGE_U4 : EPI_U4;
};

template <int WAVES, int RM, int RN, class AL, class BL>
__global__ __launch_bounds__(WAVES * 64) void gemm_tn_x3_kernel(
    AL al, BL bl, float* __restrict__ slab, float* __restrict__ bslab, int Nout, int Kout, int R,
    int rows_per_split, int tiles_k, int want_bias) {
  using S = TNX3Shape<WAVES, RM, RN>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BE = S::BE;
  constexpr int APT = S::APT, BPT = S::BPT, ACH = S::ACH, BCH = S::BCH, BUF = S::BUF;
  __shared__ uint4 lds[S::LDS_U4];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntiles = ((Nout + BM - 1) / BM) * tiles_k;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles, tile = lin - split * ntiles;
  const int tnn = tile / tiles_k, tkk = tile - tnn * tiles_k;
  const int n0 = tnn * BM, k0 = tkk * BN;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + BE - 1) / BE : 0;

  // block q -> (e block eb = q / cols, column c = q % cols); guards are wave-uniform
  int aeb[APT], ac[APT], adst[APT];
  bool ain[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT;
    ain[p] = q < S::NBA;
    const int qq = ain[p] ? q : 0;
    aeb[p] = qq / BM;
    ac[p] = qq % BM;
    adst[p] = ac[p] * 4 + (aeb[p] ^ lds_swz(ac[p]));
  }
  int beb[BPT], bc[BPT], bdst[BPT];
  bool bin[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    bin[p] = q < S::NBB;
    const int qq = bin[p] ? q : 0;
    beb[p] = qq / BN;
    bc[p] = qq % BN;
    bdst[p] = bc[p] * 4 + (beb[p] ^ lds_swz(bc[p]));
  }

  typename AL::Row arow[APT][8], arow_f[APT][8];
  typename BL::Row brow[BPT][8], brow_f[BPT][8];
  typename AL::Raw1 ra[APT][8];
  typename BL::Raw1 rb[BPT][8];
  auto mkrows = [&](int t) {
    const int e0 = e_begin + t * BE;
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p])
#pragma unroll
        for (int j = 0; j < 8; ++j) arow[p][j] = al.row(e0 + 8 * aeb[p] + j, e_end);
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p])
#pragma unroll
        for (int j = 0; j < 8; ++j) brow[p][j] = bl.row(e0 + 8 * beb[p] + j, e_end);
  };
  auto fetch = [&]() {
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p])
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          arow_f[p][j] = arow[p][j];
          ra[p][j] = al.fetch1(arow[p][j], n0 + ac[p], Nout);
        }
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p])
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          brow_f[p][j] = brow[p][j];
          rb[p][j] = bl.fetch1(brow[p][j], k0 + bc[p], Kout);
        }
  };
  float bsum[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) bsum[p] = 0.f;
  const bool do_bias = want_bias && tkk == 0;
  auto sstore = [&](int buf) {
    uint4* base = lds + buf * BUF;
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p]) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = al.combine1(ra[p][j], arow_f[p][j], n0 + ac[p], Nout);
        if (do_bias) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) s += f[j];
          bsum[p] += s;
        }
        uint4 pc[kPieces];
        split_bf16x8(f, pc);
#pragma unroll
        for (int q = 0; q < kPieces; ++q) base[q * ACH + adst[p]] = pc[q];
      }
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p]) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = bl.combine1(rb[p][j], brow_f[p][j], k0 + bc[p], Kout);
        uint4 pc[kPieces];
        split_bf16x8(f, pc);
#pragma unroll
        for (int q = 0; q < kPieces; ++q) base[kPieces * ACH + q * BCH + bdst[p]] = pc[q];
      }
  };

  floatx4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fg ^ lds_swz(fr);

  if (nt > 0) {
    mkrows(0);
    fetch();
    mkrows(1);
    sstore(0);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) {
      fetch();        // tile t+1
      mkrows(t + 2);  // index loads for tile t+2
    }
    const uint4* base = lds + cur * BUF;
    x3_slice<RM, RN>(acc, base, ACH, base + kPieces * ACH, BCH, w * 16 * RM, fr, sw);
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }

  float* C = reinterpret_cast<float*>(lds);
  float* bpart = C + (BM * S::LDC + 3) / 4 * 4;  // [4][BM]
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(w * 16 * RM + i * 16 + fg * 4 + r) * S::LDC + j * 16 + fr] = acc[i][j][r];
  if (do_bias) {
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p]) bpart[aeb[p] * BM + ac[p]] = bsum[p];
  }
  __syncthreads();
  const int ldk = (Kout + 3) & ~3;
  float* out = slab + (int64_t)split * Nout * ldk;
  constexpr int C4 = BN / 4;
  for (int q = tid; q < BM * C4; q += NT) {
    const int r = q / C4, c4 = q - r * C4;
    const int row = n0 + r, col = k0 + 4 * c4;
    if (row >= Nout || col >= Kout) continue;
    *reinterpret_cast<float4*>(out + (int64_t)row * ldk + col) =
        *reinterpret_cast<const float4*>(&C[r * S::LDC + 4 * c4]);
  }
  if (do_bias && tid < BM && n0 + tid < Nout)
    bslab[(int64_t)split * Nout + n0 + tid] =
        (bpart[tid] + bpart[BM + tid]) + (bpart[2 * BM + tid] + bpart[3 * BM + tid]);
}

template <int WAVES, int RM, int RN>
inline TnPlan plan_tn_x3(int Nout, int Kout, int R, int target_wgs) {
  using S = TNX3Shape<WAVES, RM, RN>;
  TnPlan p;
  p.tiles_n = (Nout + S::BM - 1) / S::BM;
  p.tiles_k = (Kout + S::BN - 1) / S::BN;
  const int tiles = p.tiles_n * p.tiles_k;
  // floor, not ceil: the grid must not exceed the target (a whole number of workgroups per CU);
  // one workgroup past it puts an extra one on a few CUs, and those CUs set the kernel's time
  int splits = target_wgs / tiles;
  const int max_splits = (R + 4 * S::BE - 1) / (4 * S::BE);  // >= 4 stages per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + S::BE - 1) / S::BE * S::BE;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

template <int WAVES, int RM, int RN, class AL, class BL>
inline hipError_t launch_gemm_tn_x3(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                                    float* bslab, int Nout, int Kout, int R, bool want_bias,
                                    hipStream_t st) {
  using S = TNX3Shape<WAVES, RM, RN>;
  static_assert(S::NBA % 64 == 0 && S::NBB % 64 == 0, "block guards must be wave-uniform");
  hipLaunchKernelGGL((gemm_tn_x3_kernel<WAVES, RM, RN, AL, BL>),
                     dim3(p.tiles_n * p.tiles_k * p.splits), dim3(WAVES * 64), 0, st, al, bl,
                     slab, bslab, Nout, Kout, R, p.rows_per_split, p.tiles_k,
                     want_bias ? 1 : 0);
  return hipGetLastError();
}

}  // namespace cgr
