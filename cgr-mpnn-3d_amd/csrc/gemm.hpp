// fp32 MFMA GEMM templates for the D-MPNN path (gfx950, v_mfma_f32_16x16x4_f32).
//
// Two shapes cover every GEMM of the forward and backward (SURVEY.md §2a K3,K7,K10 and their
// backward):
//
//   gemm_nt:  C[m, n] = sum_k A(m, k) * B(n, k)      A rows produced by a *loader* (plain rows,
//             gathered a[src]-h[rev] rows, or the [x | s] concat), B = rows of a weight matrix
//             ([out, in] = nn.Linear layout); an *epilogue* functor consumes every C element
//             (bias / skip / activation / dropout / stores).
//   gemm_tn:  C[n, k] = sum_e A(e, n) * B(e, k)      weight gradients dW = dZ^T Q, reduction over
//             the (long) edge / node dimension, split over gridDim.z into fp32 partial slabs
//             (deterministic: a separate kernel sums the slabs in a fixed order).  The k-tile-0
//             workgroups also emit the column sums of A (= the bias gradient) per split.
//
// Tiling (one workgroup = WAVES waves of 64 lanes):
//   NT: BM = 16*WAVES rows (one 16-row MFMA fragment per wave), BN = 16*RN columns (RN column
//       fragments per wave, A fragment reused RN times), BK = 16.  H = 400 -> RN = 5 (BN = 80)
//       tiles the hidden dimension exactly.  LDS tile = [row][4 x float4], chunk c of row r
//       stored at slot c ^ swz(r): every ds_read_b128 of a fragment is bank-conflict free
//       (16-lane groups of ds_read_b128, MI355X_MICROARCH.md §LDS).  The MFMA's 4-deep k is
//       mapped so that lane group g = lane>>4 owns k = 4g..4g+3 of the 16-deep tile: one b128
//       read feeds four MFMAs.
//   TN: LDS tiles stay e-major ([16][BM + pad], stride = 16 mod 32 floats) and fragments are read
//       with conflict-free ds_read_b32 (global loads stay coalesced float4 along n / k).
//   Double-buffered LDS with register prefetch (global loads for tile k+1 issued before the
//   MFMAs of tile k, written to the other buffer after them); one barrier per k-tile.
//   Grid: 1-D, remapped so consecutive tiles of one row panel land on one XCD (shared L2).
#pragma once

#include "common.hpp"

namespace cgr {

__device__ __forceinline__ int lds_swz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md §5 "XCD swizzle"): blocks
// b, b+8, ... run on one XCD; give each XCD a contiguous range of logical tiles.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// ------------------------------------------------------------------------------------------
// Row loaders.  Interface: Row row(int r, int limit) ; float4 load(const Row&, int k, int K)
// returning elements k..k+3 of logical row r (0 beyond K or for r >= limit).
// ------------------------------------------------------------------------------------------
template <int VEC>
struct LdPlain {
  const float* base;
  int64_t ld;
  struct Row {
    const float* p;
  };
  __device__ __forceinline__ Row row(int r, int limit) const {
    return Row{r < limit ? base + (int64_t)r * ld : nullptr};
  }
  __device__ __forceinline__ float4 load(const Row& rw, int k, int K) const {
    if (rw.p == nullptr) return f4zero();
    return load4<VEC>(rw.p + k, K - k);
  }
};

// m[e, :] = a[src[e], :] - h[rev[e], :]   (GNN.py:136-141).  Internal buffers, ld = Hp.
// REV_XOR: rev[e] = e ^ 1 (caller's original edge order, no index array).
template <bool REV_XOR>
struct LdGatherDiff {
  const float* a;
  const float* h;
  const int* src;
  const int* rev;
  int64_t ld;
  struct Row {
    const float* pa;
    const float* ph;
  };
  __device__ __forceinline__ Row row(int r, int limit) const {
    if (r >= limit) return Row{nullptr, nullptr};
    const int rv = REV_XOR ? (r ^ 1) : rev[r];
    return Row{a + (int64_t)src[r] * ld, h + (int64_t)rv * ld};
  }
  __device__ __forceinline__ float4 load(const Row& rw, int k, int K) const {
    if (rw.pa == nullptr) return f4zero();
    return f4sub(load4_masked_internal(rw.pa + k, K - k), load4_masked_internal(rw.ph + k, K - k));
  }
};

// q[v, :] = [x[v, :F] | s[v, :H]]  (GNN.py:106).  VEC divides F and ld_x.
template <int VEC>
struct LdConcat {
  const float* x;
  int64_t ldx;
  const float* s;
  int64_t lds;
  int F;
  struct Row {
    const float* px;
    const float* ps;
  };
  __device__ __forceinline__ Row row(int r, int limit) const {
    if (r >= limit) return Row{nullptr, nullptr};
    return Row{x + (int64_t)r * ldx, s + (int64_t)r * lds};
  }
  __device__ __forceinline__ float4 load(const Row& rw, int k, int K) const {
    if (rw.px == nullptr) return f4zero();
    if (k + 4 <= F) return load4<VEC>(rw.px + k, F - k);
    if (k >= F) return load4<VEC>(rw.ps + (k - F), K - k);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = k + i;
      v[i] = kk < F ? rw.px[kk] : (kk < K ? rw.ps[kk - F] : 0.f);
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
};

// ------------------------------------------------------------------------------------------
// NT GEMM
// ------------------------------------------------------------------------------------------
template <int WAVES, int RN, class AL, class BL, class EP>
__global__ __launch_bounds__(WAVES * 64) void gemm_nt_kernel(AL al, BL bl, EP ep, int M, int N,
                                                             int K, int tiles_n) {
  constexpr int BM = WAVES * 16, BN = RN * 16, NT = WAVES * 64;
  constexpr int BCH = BN * 4;
  constexpr int BPT = (BCH + NT - 1) / NT;
  __shared__ float4 As[2][BM * 4];
  __shared__ float4 Bs[2][BN * 4];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging assignment: A one float4 chunk per thread, B up to BPT chunks
  const int ar = tid >> 2, ac = tid & 3;
  const typename AL::Row arow = al.row(m0 + ar, M);
  typename BL::Row brow[BPT];
  int bdst[BPT], bcol[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int c = tid + p * NT;
    const int br = c >> 2, bc = c & 3;
    bcol[p] = bc * 4;
    bdst[p] = c < BCH ? br * 4 + (bc ^ lds_swz(br)) : -1;
    brow[p] = bl.row(c < BCH ? n0 + br : N, N);
  }
  const int adst = ar * 4 + (ac ^ lds_swz(ar));

  float4 ra, rb[BPT];
  const int nk = (K + 15) >> 4;

  floatx4 acc[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // prologue
  ra = al.load(arow, ac * 4, K);
#pragma unroll
  for (int p = 0; p < BPT; ++p) rb[p] = bl.load(brow[p], bcol[p], K);
  As[0][adst] = ra;
#pragma unroll
  for (int p = 0; p < BPT; ++p)
    if (bdst[p] >= 0) Bs[0][bdst[p]] = rb[p];
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  const int aread = (w * 16 + fr) * 4 + (fg ^ lds_swz(fr));
  int bread[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) bread[j] = (j * 16 + fr) * 4 + (fg ^ lds_swz(fr));

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int kb = (kt + 1) * 16;
      ra = al.load(arow, kb + ac * 4, K);
#pragma unroll
      for (int p = 0; p < BPT; ++p) rb[p] = bl.load(brow[p], kb + bcol[p], K);
    }
    const float4 a = As[cur][aread];
    float4 b[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) b[j] = Bs[cur][bread[j]];
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b[j].x, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b[j].y, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b[j].z, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b[j].w, acc[j], 0, 0, 0);
    if (more) {
      As[cur ^ 1][adst] = ra;
#pragma unroll
      for (int p = 0; p < BPT; ++p)
        if (bdst[p] >= 0) Bs[cur ^ 1][bdst[p]] = rb[p];
    }
    __syncthreads();
  }

  // epilogue: C/D map of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg
  const int rbase = m0 + w * 16 + fg * 4;
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = n0 + j * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) ep(rbase + r, col, acc[j][r]);
  }
}

template <int WAVES, int RN, class AL, class BL, class EP>
inline hipError_t launch_gemm_nt(const AL& al, const BL& bl, const EP& ep, int M, int N, int K,
                                 hipStream_t st) {
  constexpr int BM = WAVES * 16, BN = RN * 16;
  if (M <= 0 || N <= 0) return hipSuccess;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_nt_kernel<WAVES, RN, AL, BL, EP>), dim3(tm * tn), dim3(WAVES * 64), 0,
                     st, al, bl, ep, M, N, K, tn);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// TN split-K GEMM (weight gradients)
// ------------------------------------------------------------------------------------------
template <int WAVES, int RN, class AL, class BL>
__global__ __launch_bounds__(WAVES * 64) void gemm_tn_kernel(AL al, BL bl, float* __restrict__ slab,
                                                             float* __restrict__ bslab, int Nout,
                                                             int Kout, int R, int rows_per_split,
                                                             int tiles_k, int want_bias) {
  constexpr int BM = WAVES * 16, BN = RN * 16, NT = WAVES * 64;
  constexpr int SA = BM + (((16 - BM % 32) % 32) + 32) % 32;  // stride == 16 (mod 32)
  constexpr int SB = BN + (((16 - BN % 32) % 32) + 32) % 32;
  constexpr int ACH = 16 * BM / 4;  // == NT
  constexpr int BCH = 16 * BN / 4;
  constexpr int BPT = (BCH + NT - 1) / NT;
  static_assert(ACH == NT, "one A chunk per thread");
  __shared__ float At[2][16 * SA];
  __shared__ float Bt[2][16 * SB];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tiles = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, tiles);
  const int tnn = tile / tiles_k, tkk = tile - tnn * tiles_k;
  const int n0 = tnn * BM, k0 = tkk * BN;
  const int split = blockIdx.y;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + 15) >> 4 : 0;

  const int ae = tid / (BM / 4), ac = tid % (BM / 4);
  int be[BPT], bc[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int c = tid + p * NT;
    be[p] = c < BCH ? c / (BN / 4) : -1;
    bc[p] = c < BCH ? c % (BN / 4) : 0;
  }

  float4 ra, rb[BPT];
  auto gload = [&](int t) {
    const int e = e_begin + t * 16 + ae;
    const typename AL::Row r = al.row(e, e_end);
    ra = al.load(r, n0 + ac * 4, Nout);
#pragma unroll
    for (int p = 0; p < BPT; ++p) {
      if (be[p] >= 0) {
        const typename BL::Row rr = bl.row(e_begin + t * 16 + be[p], e_end);
        rb[p] = bl.load(rr, k0 + bc[p] * 4, Kout);
      }
    }
  };
  auto sstore = [&](int buf) {
    *reinterpret_cast<float4*>(&At[buf][ae * SA + ac * 4]) = ra;
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (be[p] >= 0) *reinterpret_cast<float4*>(&Bt[buf][be[p] * SB + bc[p] * 4]) = rb[p];
  };

  floatx4 acc[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const bool do_bias = want_bias && tkk == 0 && tid < BM;

  if (nt > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) gload(t + 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int er = 4 * s + fg;
      const float av = At[cur][er * SA + w * 16 + fr];
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const float bv = Bt[cur][er * SB + j * 16 + fr];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    }
    if (do_bias) {
#pragma unroll
      for (int e = 0; e < 16; ++e) bsum += At[cur][e * SA + tid];
    }
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }

  float* out = slab + (int64_t)split * Nout * Kout;
  const int rbase = n0 + w * 16 + fg * 4;
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = k0 + j * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rbase + r;
      if (row < Nout && col < Kout) out[(int64_t)row * Kout + col] = acc[j][r];
    }
  }
  if (do_bias && n0 + tid < Nout) bslab[(int64_t)split * Nout + n0 + tid] = bsum;
}

struct TnPlan {
  int tiles_n, tiles_k, splits, rows_per_split;
};

template <int WAVES, int RN>
inline TnPlan plan_tn(int Nout, int Kout, int R, int target_wgs) {
  constexpr int BM = WAVES * 16, BN = RN * 16;
  TnPlan p;
  p.tiles_n = (Nout + BM - 1) / BM;
  p.tiles_k = (Kout + BN - 1) / BN;
  const int tiles = p.tiles_n * p.tiles_k;
  int splits = (target_wgs + tiles - 1) / tiles;
  const int max_splits = (R + 63) / 64;  // at least 64 rows (4 k-tiles) per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + 15) / 16 * 16;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

template <int WAVES, int RN, class AL, class BL>
inline hipError_t launch_gemm_tn(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                                 float* bslab, int Nout, int Kout, int R, bool want_bias,
                                 hipStream_t st) {
  hipLaunchKernelGGL((gemm_tn_kernel<WAVES, RN, AL, BL>), dim3(p.tiles_n * p.tiles_k, p.splits),
                     dim3(WAVES * 64), 0, st, al, bl, slab, bslab, Nout, Kout, R,
                     p.rows_per_split, p.tiles_k, want_bias ? 1 : 0);
  return hipGetLastError();
}

}  // namespace cgr
