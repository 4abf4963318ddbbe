// Row-block-stationary NT GEMM for the edge-row GEMMs of the D-MPNN layers (gfx950, fp32 MFMA).
//
//   C[m, n] = sum_k A(m, k) * B(n, k),  n < N <= 16 * 4 * FMAX,  K <= RS_KMAX
//
// One workgroup = 16 waves (1024 threads) owns a block of 64 A rows and ALL N output columns:
//   * the 64 x K A block is produced once by the row loader (plain rows, or the gathered
//     a[src] - h[rev] message rows) into LDS ([k16][row][4 float4] with the chunk XOR swizzle of
//     gemm.hpp: conflict-free ds_read_b128);
//   * main loop: no per-k-tile barrier.  Wave w computes row fragment rf = w & 3 (16 rows) against column
//     group cg = w >> 2 (6-7 fragments of 16 columns, 25 fragments for N = 400); its B fragments
//     are loaded straight from global/L2 into registers (B rows are weight rows [out, in]: one float4
//     per lane per fragment per 16-deep k-tile), software-pipelined PF k-tiles ahead.  The four
//     waves of a column group (one per SIMD) read the same B lines, which the CU's L1 serves;
//     each SIMD holds one wave of every column group, so every SIMD does the same MFMA work;
//   * the A block streams into LDS in chunks of 4 k-tiles, one chunk ahead of the MFMAs (one
//     barrier per chunk, no LDS slot is reused);
//   * epilogue: accumulators -> LDS -> float4 rows -> ep.apply4p; a thread keeps one float4
//     column, all its operand loads issued before the accumulators go through LDS.
// Compared with the 64x80-tile register-staged kernel (gemm.hpp) this reads every A row once (not
// once per 80-column tile), drops the per-k-tile LDS stores and barriers, and balances work per
// CU exactly (one 64-row block per workgroup, one workgroup per CU).
#pragma once

#include "gemm.hpp"

namespace cgr {

constexpr int RS_BM = 64;
constexpr int RS_WAVES = 16;
constexpr int RS_NT = RS_WAVES * 64;
constexpr int RS_KMAX = 512;  // LDS: 64 rows x 512 floats = 128 KB
constexpr int RS_NMAX = 512;  // epilogue image 64 x (N + 4) floats <= 160 KB
constexpr int RS_EPASS = 8;   // epilogue row passes: ceil(64 / floor(1024 / (N / 4))) <= 8 for N <= 512

// column-fragment group of wave group cg: fragments [f0, f0 + nf) of NF total, split 4 ways with
// the larger groups first
__device__ __forceinline__ void rs_group(int NF, int G, int cg, int& f0, int& nf) {
  const int q = NF / G, r = NF % G;
  nf = q + (cg < r ? 1 : 0);
  f0 = cg * q + (cg < r ? cg : r);
}

// One wave's share of a 64-row block: A chunks (4 k-tiles = 64 k of the 64 rows, one float4 per
// thread) are produced by all 1024 threads into LDS one chunk ahead of the MFMAs that read them
// (one barrier per chunk); B fragments are loaded per wave straight into registers one k-tile
// ahead; the epilogue runs from the accumulators (no LDS round trip), all its operand loads issued
// together.
#ifndef CGR_RS_MODE
#define CGR_RS_MODE 0  // lab only: 1 = no B loads after the first tiles, 3 = one B row set for all waves
#endif
#ifdef CGR_RS_STAMPS
__device__ unsigned long long* rs_stamps;  // lab: [block][wave][4] s_memrealtime stamps
#define RS_STAMP(i)                                                                             \
  if ((tid & 63) == 0)                                                                          \
    rs_stamps[((size_t)blockIdx.x * 16 + (tid >> 6)) * 4 + (i)] = __builtin_amdgcn_s_memrealtime();
#else
#define RS_STAMP(i)
#endif

template <int RM, int NFW, class AL, class EP>
__device__ __forceinline__ void rs_body(const AL& al, float4* __restrict__ As,
                                        const float* __restrict__ B, int64_t ldb, const EP& ep,
                                        int M, int N, int K, int m0, int f0, int row0, int tid) {
  const int lane = tid & 63, fr = lane & 15, fg = lane >> 4;
  const int sw = fg ^ lds_swz(fr);
  const int nk = (K + 15) >> 4, nch = (nk + 3) >> 2;

  // ---- A chunk producer: thread -> (row ar, float4 column akc of the 16 in a chunk) ----
  const int ar = tid >> 4, akc = tid & 15;
  const typename AL::Row arow = al.row(m0 + ar, M);
  const int adst = ((akc >> 2) * RS_BM + ar) * 4 + ((akc & 3) ^ lds_swz(ar));
  typename AL::Raw ra;
  auto fetchA = [&](int c) { ra = al.fetch(arow, c * 64 + akc * 4, K); };
  auto storeA = [&](int c) {
    if (4 * c + (akc >> 2) < nk) As[c * 4 * RS_BM * 4 + adst] = al.combine(ra, arow, c * 64 + akc * 4, K);
  };

  // ---- B fragments: row n = (f0 + j) * 16 + fr (N % 16 == 0: always a real row), one 32-bit
  // lane offset plus a uniform per-fragment stride ----
#if CGR_RS_MODE == 3
  const int boff = ((0 * 16 + fr) * (int)ldb) + 4 * fg;  // lab: every wave reads group 0's rows
#else
  const int boff = ((f0 * 16 + fr) * (int)ldb) + 4 * fg;
#endif
  const int bstride = 16 * (int)ldb;
  // unconditional loads: k-tiles past the end read k = 0 (in bounds, never consumed); k chunks
  // past K inside the last tile read k = 0 too and meet zeros in the A image
  auto fetchB = [&](float4(&x)[NFW], int kt) {
    if (CGR_RS_MODE == 1 && kt > 1) return;
    const int kb = kt < nk ? kt * 16 : 0;
    const int o = boff + ((kb + 4 * fg < K) ? kb : 0);
#pragma unroll
    for (int j = 0; j < NFW; ++j) x[j] = *reinterpret_cast<const float4*>(B + o + j * bstride);
  };
  floatx4 acc[RM][NFW];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < NFW; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const float4(&x)[NFW], int kt) {
    float4 a[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) a[i] = As[(kt * RS_BM + row0 + i * 16 + fr) * 4 + sw];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < NFW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a[i], s), f4get(x[j], s),
                                                           acc[i][j], 0, 0, 0);
  };

  // Branch-free steady state (a runtime-conditional load makes hipcc wait vmcnt(0) at the merge,
  // which serialises the prefetch): every fetch is unconditional from a clamped address, the A
  // store is a per-lane predicate; only the last partial chunk (nk % 4 k-tiles) branches.
#ifndef CGR_RS_INTERLEAVE
#define CGR_RS_INTERLEAVE 3  // MFMAs per interleaved B load: A/B 3 -0.2 % vs 4 (twice), 2 +0.7 %, 5 ±0
#endif
  auto step = [&](float4(&xn)[NFW], int ktn, const float4(&xc)[NFW], int ktc) {
    fetchB(xn, ktn);
    compute(xc, ktc);
    if constexpr (CGR_RS_INTERLEAVE > 0) {
      __builtin_amdgcn_sched_group_barrier(0x100, RM, 0);  // the A fragment ds_reads
#pragma unroll
      for (int i = 0; i < NFW; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, CGR_RS_INTERLEAVE * RM, 0);  // MFMAs
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);                       // one B load
      }
      __builtin_amdgcn_sched_group_barrier(0x008, (4 - CGR_RS_INTERLEAVE) * RM * NFW, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
#ifndef CGR_RS_PFD
#define CGR_RS_PFD 1  // B prefetch distance in k-tiles: 1 (two register sets) or 3 (four sets)
#endif
  RS_STAMP(0)
  const int nfull = nk >> 2;
  if constexpr (CGR_RS_PFD == 3) {
    float4 x0[NFW], x1[NFW], x2[NFW], x3[NFW];
    fetchA(0);
    fetchB(x0, 0);
    fetchB(x1, 1);
    fetchB(x2, 2);
    storeA(0);
    fetchA(nch > 1 ? 1 : 0);
    __syncthreads();
    RS_STAMP(1)
    for (int c = 0; c < nfull; ++c) {
      const int kt = 4 * c;
      step(x3, kt + 3, x0, kt);
      step(x0, kt + 4, x1, kt + 1);
      step(x1, kt + 5, x2, kt + 2);
      step(x2, kt + 6, x3, kt + 3);
      storeA(c + 1);
      fetchA(min(c + 2, nch - 1));
      __syncthreads();
    }
    const int kt = 4 * nfull, rem = nk - kt;
    if (rem > 0) compute(x0, kt);
    if (rem > 1) compute(x1, kt + 1);
    if (rem > 2) compute(x2, kt + 2);
  } else {
    float4 x0[NFW], x1[NFW];
    fetchA(0);
    fetchB(x0, 0);
    storeA(0);
    fetchA(nch > 1 ? 1 : 0);
    __syncthreads();
    RS_STAMP(1)
    for (int c = 0; c < nfull; ++c) {
      const int kt = 4 * c;
      // each k-tile step: the next tile's B loads are interleaved one per 4 MFMAs of the current
      // tile (sched_group_barrier), so the vector-memory pipe is fed throughout the MFMA stream
      // instead of in one burst per tile that every wave of the SIMD issues at the same moment
      step(x1, kt + 1, x0, kt);
      step(x0, kt + 2, x1, kt + 1);
      step(x1, kt + 3, x0, kt + 2);
      step(x0, kt + 4, x1, kt + 3);
      storeA(c + 1);  // k-tiles >= nk are not written
      fetchA(min(c + 2, nch - 1));
      __syncthreads();
    }
    const int kt = 4 * nfull, rem = nk - kt;
    if (rem > 0) {
      fetchB(x1, kt + 1);
      compute(x0, kt);
    }
    if (rem > 1) {
      fetchB(x0, kt + 2);
      compute(x1, kt + 1);
    }
    if (rem > 2) compute(x0, kt + 2);
  }

  // ---- epilogue: accumulators -> LDS (the A block is dead after the barrier) -> float4 rows.
  // Thread t owns float4 column c4 = t % C4 of rows t / C4 + RPP * it, so its column operands
  // (bias) are loaded once; every operand load is issued before the barrier.
  RS_STAMP(2)
  const int C4 = N >> 2, RPP = RS_NT / C4, npass = (RS_BM + RPP - 1) / RPP;
  const int ec4 = tid % C4, er0 = tid / C4;
  const bool eact = er0 < RPP;
  const typename EP::Ctx cx = ep.ctx();
  typename EP::Pre pv[RS_EPASS];
#pragma unroll
  for (int it = 0; it < RS_EPASS; ++it) {
    const int r = min(er0 + RPP * it, RS_BM - 1);
    pv[it] = ep.pre4(m0 + r, 4 * ec4);
  }
  __syncthreads();
  float* C = reinterpret_cast<float*>(As);
  const int LDC = N + 4;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < NFW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(row0 + i * 16 + fg * 4 + r) * LDC + (f0 + j) * 16 + fr] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < RS_EPASS; ++it) {
    const int r = er0 + RPP * it;
    if (eact && it < npass && r < RS_BM) {
      const float4 v = *reinterpret_cast<const float4*>(&C[r * LDC + 4 * ec4]);
      ep.apply4p(m0 + r, 4 * ec4, v, pv[it], cx);
    }
  }
  RS_STAMP(3)
}

// RM = row fragments per wave: the 16 waves form 4 / RM row groups x 4 * RM column groups
// (RM = 2: every B fragment a wave loads feeds 8 MFMAs instead of 4, halving the B load traffic;
// N = 400 splits its 25 column fragments 4,3,...,3 over 8 groups, so SIMDs get 26/26/24/24)
template <int RM, int FMAX, class AL, class EP>
__global__ __launch_bounds__(RS_NT) void gemm_rs_kernel(AL al, const float* __restrict__ B,
                                                        int64_t ldb, EP ep, int M, int N, int K) {
  extern __shared__ float4 rs_lds[];
  const int tid = threadIdx.x, w = tid >> 6;
  constexpr int RG = 4 / RM;
  const int m0 = blockIdx.x * RS_BM;
  const int row0 = (w % RG) * 16 * RM, cg = w / RG;
  int f0, nf;
  rs_group((N + 15) >> 4, 4 * RM, cg, f0, nf);
  // wave-uniform split into the two register shapes (nf differs by at most 1 between groups);
  // both paths execute the same barriers (one per A chunk, two in the epilogue)
  if (nf == FMAX)
    rs_body<RM, FMAX>(al, rs_lds, B, ldb, ep, M, N, K, m0, f0, row0, tid);
  else if constexpr (FMAX > 1)
    rs_body<RM, FMAX - 1>(al, rs_lds, B, ldb, ep, M, N, K, m0, f0, row0, tid);
}

// FMAX: max column fragments per wave = ceil(ceil(N / 16) / (4 RM)); N = 400 -> 7 (RM 1), 4 (RM 2).
inline int rs_fmax(int N, int RM) { return (((N + 15) / 16) + 4 * RM - 1) / (4 * RM); }

inline size_t rs_lds_bytes(int N, int K) {
  const size_t a = (size_t)RS_BM * ((K + 15) / 16) * 16 * 4, c = (size_t)RS_BM * (N + 4) * 4;
  return a > c ? a : c;
}

// B: [N, ldb] row-major weight rows (n, k), 16-byte aligned rows (ldb % 4 == 0), K % 4 == 0,
// N % 16 == 0, N <= 64 * FMAX, K <= RS_KMAX, N * ldb < 2^31 (rs_ok checks these).
// (the dispatcher also requires ceil(N / 16) >= 4 * RM: a wave group without a column fragment
// would skip the A-chunk production and the barriers)
inline bool rs_ok(int N, int K, int64_t ldb, const void* B) {
  return N > 0 && N % 16 == 0 && N <= RS_NMAX && K % 4 == 0 && K <= RS_KMAX && ldb % 4 == 0 &&
         ((uintptr_t)B & 15) == 0 && (int64_t)N * ldb < (int64_t(1) << 31);
}
template <int RM, int FMAX, class AL, class EP>
inline hipError_t launch_gemm_rs(const AL& al, const float* B, int64_t ldb, const EP& ep, int M,
                                 int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const size_t lds = rs_lds_bytes(N, K);
  auto kern = gemm_rs_kernel<RM, FMAX, AL, EP>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((M + RS_BM - 1) / RS_BM), dim3(RS_NT), lds, st, al, B, ldb, ep, M,
                     N, K);
  return hipGetLastError();
}

}  // namespace cgr
