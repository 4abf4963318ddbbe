// TN split-K GEMM, version 2: weight gradients C[n, k] = sum_e A(e, n) * B(e, k) with the NT
// kernel's fragment path (gemm.hpp): both tiles are staged TRANSPOSED into the n-major /
// k-major LDS image [c16][row][4 float4 over e] (XOR-swizzled chunks), so every MFMA operand
// comes from a conflict-free ds_read_b128 that feeds four MFMAs -- the v1 TN kernel read one
// ds_read_b32 per operand per MFMA (e-major image).
//
// Staging: a thread owns a 2 (e) x 4 (n or k) block of a tile: two row loads through the usual
// loaders (plain rows / gathered a[src] - h[rev] / [x | s] concat), a 2x4 register transpose, and
// four ds_write_b64 into the chunk slots of the four rows.  BE = 32 rows per stage (KT = 2), so a
// 5-wave workgroup with 80 x 80 tiles has exactly one A block and one B block per thread.
// Split-K over row ranges into fp32 slabs (rows padded to 4 floats), XCD-contiguous splits, bias
// column sums of A from the staged image by the workgroups of k-tile 0 -- as in v1.
#pragma once

#include "gemm.hpp"

namespace cgr {

#ifndef CGR_TN2_KT
#define CGR_TN2_KT 2
#endif

template <int WAVES, int RM, int RN>
struct TN2Shape {
  static constexpr int KT = CGR_TN2_KT;
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RM, BN = RN * 16, BE = 16 * KT;
  static constexpr int A_F4 = KT * BM * 4, B_F4 = KT * BN * 4;  // float4 per stage
  static constexpr int NBA = (BE / 2) * (BM / 4), NBB = (BE / 2) * (BN / 4);  // 2x4 blocks
  static constexpr int APT = (NBA + NT - 1) / NT, BPT = (NBB + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr int STAGE_F4 = 2 * (A_F4 + B_F4);
  static constexpr int EPI_F4 = (BM * LDC + 3) / 4;
  static constexpr int LDS_F4 = STAGE_F4 > EPI_F4 ? STAGE_F4 : EPI_F4;
};

// float offset of element (row r, e_local) of a [KT][rows][4 float4] image with `rows` rows
__device__ __forceinline__ int tn2_off(int rows, int r, int el) {
  const int c16 = el >> 4, q = (el >> 2) & 3;
  return (((c16 * rows + r) * 4) + (q ^ lds_swz(r))) * 4 + (el & 3);
}

template <int WAVES, int RM, int RN, class AL, class BL>
__global__ __launch_bounds__(WAVES * 64) void gemm_tn2_kernel(
    AL al, BL bl, float* __restrict__ slab, float* __restrict__ bslab, int Nout, int Kout, int R,
    int rows_per_split, int tiles_k, int want_bias) {
  using S = TN2Shape<WAVES, RM, RN>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BE = S::BE, KT = S::KT;
  constexpr int APT = S::APT, BPT = S::BPT;
  __shared__ float4 lds[S::LDS_F4];
  float4* As = lds;
  float4* Bs = lds + 2 * S::A_F4;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ntiles = ((Nout + BM - 1) / BM) * tiles_k;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles, tile = lin - split * ntiles;
  const int tnn = tile / tiles_k, tkk = tile - tnn * tiles_k;
  const int n0 = tnn * BM, k0 = tkk * BN;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + BE - 1) / BE : 0;

  // block -> (e pair, 4-column group); blocks past the tile are fetched clamped, never stored
  int ae[APT], ac[APT];
  bool ain[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT;
    ain[p] = q < S::NBA;
    const int qq = ain[p] ? q : 0;
    ae[p] = 2 * (qq / (BM / 4));
    ac[p] = (qq % (BM / 4)) * 4;
  }
  int be[BPT], bc[BPT];
  bool bin[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    bin[p] = q < S::NBB;
    const int qq = bin[p] ? q : 0;
    be[p] = 2 * (qq / (BN / 4));
    bc[p] = (qq % (BN / 4)) * 4;
  }

  typename AL::Row arow[APT][2], arow_f[APT][2];
  typename BL::Row brow[BPT][2], brow_f[BPT][2];
  typename AL::Raw ra[APT][2];
  typename BL::Raw rb[BPT][2];
  auto mkrows = [&](int t) {  // row state (index loads) one tile ahead
    const int e0 = e_begin + t * BE;
#pragma unroll
    for (int p = 0; p < APT; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) arow[p][h] = al.row(e0 + ae[p] + h, e_end);
#pragma unroll
    for (int p = 0; p < BPT; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) brow[p][h] = bl.row(e0 + be[p] + h, e_end);
  };
  auto fetch = [&]() {
#pragma unroll
    for (int p = 0; p < APT; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        arow_f[p][h] = arow[p][h];
        ra[p][h] = al.fetch(arow[p][h], n0 + ac[p], Nout);
      }
#pragma unroll
    for (int p = 0; p < BPT; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        brow_f[p][h] = brow[p][h];
        rb[p][h] = bl.fetch(brow[p][h], k0 + bc[p], Kout);
      }
  };
  // 2 x 4 block -> four (row, e-pair) float2 in the transposed image
  auto put = [&](float* img, int rows, int r0, int el, const float4& v0, const float4& v1) {
    const float a0[4] = {v0.x, v0.y, v0.z, v0.w}, a1[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<float2*>(img + tn2_off(rows, r0 + j, el)) = make_float2(a0[j], a1[j]);
  };
  auto sstore = [&](int buf) {
    float* Ab = reinterpret_cast<float*>(As + buf * S::A_F4);
    float* Bb = reinterpret_cast<float*>(Bs + buf * S::B_F4);
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (ain[p])
        put(Ab, BM, ac[p], ae[p], al.combine(ra[p][0], arow_f[p][0], n0 + ac[p], Nout),
            al.combine(ra[p][1], arow_f[p][1], n0 + ac[p], Nout));
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p])
        put(Bb, BN, bc[p], be[p], bl.combine(rb[p][0], brow_f[p][0], k0 + bc[p], Kout),
            bl.combine(rb[p][1], brow_f[p][1], k0 + bc[p], Kout));
  };

  floatx4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const bool do_bias = want_bias && tkk == 0 && tid < BM;
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
    const float4* Ac = As + cur * S::A_F4;
    const float4* Bc = Bs + cur * S::B_F4;
#pragma unroll
    for (int c16 = 0; c16 < KT; ++c16) {
      float4 a[RM], b[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) a[i] = Ac[(c16 * BM + w * 16 * RM + i * 16 + fr) * 4 + sw];
#pragma unroll
      for (int j = 0; j < RN; ++j) b[j] = Bc[(c16 * BN + j * 16 + fr) * 4 + sw];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a[i], s), f4get(b[j], s),
                                                             acc[i][j], 0, 0, 0);
    }
    if (do_bias) {  // column sums of A (= bias gradient) over this stage's rows
#pragma unroll
      for (int c = 0; c < 4 * KT; ++c) {
        const float4 v = Ac[((c >> 2) * BM + tid) * 4 + (c & 3)];
        bsum += (v.x + v.y) + (v.z + v.w);
      }
    }
    if (more) sstore(cur ^ 1);
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
  if (do_bias && n0 + tid < Nout) bslab[(int64_t)split * Nout + n0 + tid] = bsum;
}

template <int WAVES, int RM, int RN>
inline TnPlan plan_tn2(int Nout, int Kout, int R, int target_wgs) {
  using S = TN2Shape<WAVES, RM, RN>;
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
inline hipError_t launch_gemm_tn2(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                                  float* bslab, int Nout, int Kout, int R, bool want_bias,
                                  hipStream_t st) {
  hipLaunchKernelGGL((gemm_tn2_kernel<WAVES, RM, RN, AL, BL>),
                     dim3(p.tiles_n * p.tiles_k * p.splits), dim3(WAVES * 64), 0, st, al, bl,
                     slab, bslab, Nout, Kout, R, p.rows_per_split, p.tiles_k,
                     want_bias ? 1 : 0);
  return hipGetLastError();
}

}  // namespace cgr
