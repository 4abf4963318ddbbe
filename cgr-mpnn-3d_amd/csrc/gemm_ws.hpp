// Weight-stationary NT GEMM for the hidden x hidden products of the D-MPNN (K = H <= 512):
//   layer forward   h' = epi((a[src] - h[rev]) W_l^T)      (M = E, N = K = H)
//   backward        dm = dpre W_l,  ds = dzn W_n[:, F:]     (B = transposed weights)
//
// Why a second NT kernel: at E = 15,360 rows the staged kernel (gemm.hpp) only gets ~4.7 waves per
// SIMD and each wave serialises LDS-read -> MFMA -> LDS-write -> barrier every 16-deep k-tile;
// MFMA busy stayed ~45-49% whatever the tile shape (tools/gemm_bench.hip).  Here:
//   * one workgroup (4 waves) per CU keeps a BN-column slice of B (= W rows [n0, n0+BN), all of
//     K) resident in LDS for its whole lifetime: [k16][BN][4 x float4], swizzled like gemm.hpp so
//     every fragment ds_read_b128 is conflict-free; loaded once, then never written -> no
//     barrier in the main loop;
//   * A never touches LDS: in the 16x16x4 operand layout a lane needs row (lane & 15), k = 4g..4g+3
//     of a 16-deep chunk (g = lane >> 4) - exactly one float4 of its row, fetched straight from
//     global (gathered a[src] - h[rev] rows included) and fed to 4 MFMAs per B fragment;
//   * A chunks are prefetched P chunks ahead through a static register ring, B fragments one chunk
//     ahead; the ring keeps running across row tiles (the next tile's first chunks are fetched
//     during the current tile's last group), so a wave never drains its pipeline;
//   * each wave owns whole 16-row tiles (round-robin over the slice's tiles); the epilogue goes
//     through a per-wave LDS scratch so every epilogue access is a coalesced float4, and its
//     side input (h0 for the layer) is prefetched at the start of the tile.
// Grid: nslices * groups WGs, XCD-remapped so the slices of one row group share an XCD's L2.
#pragma once

#include "gemm.hpp"

namespace cgr {

template <int RN>
struct WSShape {
  static constexpr int BN = RN * 16;
  static constexpr int LDC = BN + 4;
  static constexpr int SCRATCH_F = 16 * LDC;  // per wave
  static constexpr int WAVES = 4;
};

inline size_t ws_lds_bytes(int RN, int Kc_padded) {
  const int BN = RN * 16;
  return (size_t)Kc_padded * BN * 64 + 4 * 16 * (BN + 4) * 4;
}

// B rows (n) with leading dimension ldb, K columns; VEC 4 (ldb % 4 == 0, 16-byte rows)
template <int RN, int P, class AL, class EP>
__global__ __launch_bounds__(256, 1) void gemm_ws_kernel(AL al, const float* __restrict__ B,
                                                         int64_t ldb, EP ep, int M, int N, int K,
                                                         int Kcp, int nslices, int groups) {
  using S = WSShape<RN>;
  constexpr int BN = S::BN;
  extern __shared__ float4 smem[];
  float4* Ws = smem;                                                      // [Kcp][BN][4]
  float* scratch = reinterpret_cast<float*>(smem + (size_t)Kcp * BN * 4);  // [4][16][LDC]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = g / nslices, slice = g - grp * nslices;
  const int n0 = slice * BN;
  const int Kc = (K + 15) >> 4;

  // ---- resident B slice (zero rows beyond N, zero k beyond K) ----
  {
    const int kc4 = Kcp * 4;  // float4 chunks per row
    for (int q = tid; q < BN * kc4; q += 256) {
      const int r = q / kc4, kc = q - r * kc4;
      const int n = n0 + r, k = kc * 4;
      float4 v = f4zero();
      if (n < N && k < K) {
        v = *reinterpret_cast<const float4*>(B + (int64_t)n * ldb + k);
        if (k + 4 > K) v = mask4(v, true, k, K);
      }
      Ws[((kc >> 2) * BN + r) * 4 + ((kc & 3) ^ lds_swz(r))] = v;
    }
  }
  __syncthreads();

  const int ntiles = (M + 15) >> 4;
  const int wpg = groups * 4;       // waves working on this slice
  int t = grp * 4 + w;              // first tile of this wave
  if (t >= ntiles) return;
  const int fr = lane & 15, fg = lane >> 4, sw = fg ^ lds_swz(fr);
  const int kl = 4 * fg;
  float* scr = scratch + w * S::SCRATCH_F;

  typename AL::Row row = al.row(t * 16 + fr, M);
  int tn = t + wpg;
  typename AL::Row row_next = al.row(tn * 16 + fr, M);  // masked when tn >= ntiles

  // prime the ring with chunks 0..P-1 of the first tile
  typename AL::Raw ring[P];
#pragma unroll
  for (int u = 0; u < P; ++u) ring[u] = al.fetch(row, 16 * u + kl, K);

  constexpr int C4 = BN / 4;
  constexpr int EPQ = (16 * C4 + 63) / 64;  // epilogue float4 pieces per lane

  while (true) {
    const int m0 = t * 16;
    typename EP::Pre pre[EPQ];
#pragma unroll
    for (int i = 0; i < EPQ; ++i) {
      const int q = lane + 64 * i;
      const int r = q / C4, c4 = q - r * C4;
      pre[i] = ep.pre4(q < 16 * C4 ? m0 + r : M, n0 + 4 * c4);
    }
    floatx4 acc[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float4 bcur[RN];
#pragma unroll
    for (int j = 0; j < RN; ++j) bcur[j] = Ws[(j * 16 + fr) * 4 + sw];

    for (int c = 0; c < Kcp; c += P) {
#pragma unroll
      for (int u = 0; u < P; ++u) {
        const int cc = c + u;
        const int cn = cc + 1 < Kc ? cc + 1 : Kc - 1;  // next B chunk (clamped; A is 0 there)
        float4 bnext[RN];
#pragma unroll
        for (int j = 0; j < RN; ++j) bnext[j] = Ws[(cn * BN + j * 16 + fr) * 4 + sw];
        const float4 a = al.combine(ring[u], row, 16 * cc + kl, K);
        // refill slot u with chunk cc + P of this tile, or of the next tile past the end
        const int q = cc + P;
        const bool same = q < Kcp;
        ring[u] = al.fetch(same ? row : row_next, 16 * (same ? q : q - Kcp) + kl, K);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, s), f4get(bcur[j], s), acc[j],
                                                         0, 0, 0);
#pragma unroll
        for (int j = 0; j < RN; ++j) bcur[j] = bnext[j];
      }
    }

    // epilogue through the wave's LDS scratch (C/D map: col = lane & 15, row = 4*(lane>>4) + r)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) scr[(fg * 4 + r) * S::LDC + j * 16 + fr] = acc[j][r];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int i = 0; i < EPQ; ++i) {
      const int q = lane + 64 * i;
      if (q < 16 * C4) {
        const int r = q / C4, c4 = q - r * C4;
        const float4 v = *reinterpret_cast<const float4*>(&scr[r * S::LDC + 4 * c4]);
        ep.apply4p(m0 + r, n0 + 4 * c4, v, pre[i]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

    if (tn >= ntiles) break;
    t = tn;
    row = row_next;
    tn = t + wpg;
    row_next = al.row(tn * 16 + fr, M);
  }
}

struct WsPlan {
  int Kcp, nslices, groups;
  size_t lds;
  bool ok;
};

template <int RN, int P>
inline WsPlan plan_ws(int M, int N, int K, int num_cus) {
  WsPlan p{};
  const int Kc = (K + 15) / 16;
  p.Kcp = (Kc + P - 1) / P * P;
  p.lds = ws_lds_bytes(RN, p.Kcp);
  p.ok = p.lds <= 160 * 1024;
  p.nslices = (N + RN * 16 - 1) / (RN * 16);
  const int ntiles = (M + 15) / 16;
  int groups = num_cus / p.nslices;
  if (groups < 1) groups = 1;
  const int max_groups = (ntiles + 3) / 4;
  if (groups > max_groups) groups = max_groups;
  p.groups = groups;
  return p;
}

template <int RN, int P, class AL, class EP>
inline hipError_t launch_gemm_ws(const AL& al, const float* B, int64_t ldb, const EP& ep, int M,
                                 int N, int K, const WsPlan& p, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&gemm_ws_kernel<RN, P, AL, EP>),
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL((gemm_ws_kernel<RN, P, AL, EP>), dim3(p.nslices * p.groups), dim3(256),
                     p.lds, st, al, B, ldb, ep, M, N, K, p.Kcp, p.nslices, p.groups);
  return hipGetLastError();
}

}  // namespace cgr
