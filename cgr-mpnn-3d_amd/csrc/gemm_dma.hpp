// NT GEMM with LDS-DMA staging (global_load_lds_dwordx4) and a 3-stage ring, for the layer-shaped
// products whose reduction length is a multiple of the k-tile (K = H = 400 here):
//
//   C[m, n] = sum_k A(m, k) * B(n, k),  A(m, :) = a[src[m], :] - h[rev[m], :]  (GATHER)
//                                       A(m, :) = a[m, :]                      (plain)
//
// Why (tools/gemm_probe.hip ladder at E x 400 x 400): with register staging the loop time was the
// SUM of its memory phase (loads + ds_write + barrier, 31 us) and its MFMA phase (40 us): every
// workgroup stalled on its own loads between the two.  Here the loads write LDS directly and two
// tiles stay in flight across each barrier, so the waves only issue, wait (counted vmcnt) and run
// MFMAs (cdna_hip_programming.md §5 "Async global->LDS copy", "Pipelining across barriers").
//
// Geometry: W waves, wave w owns output rows [16w, 16w + 16) x all BN = 16 RN columns (RN % W == 0),
// k-tile BK = 16 KT.  One DMA wave-instruction moves 1 KiB = 16 rows x one 16-float k-chunk; wave w
// moves its own A rows (and h rows when gathering) and B rows [16j, 16j + 16) for j = w, w + W, ...
// LDS image per stage: [KT][rows][4 float4] with slot s of row r holding k-chunk s ^ swz(r) -- the
// swizzle is applied on the per-lane SOURCE address (the DMA destination is lane-linear), and the
// fragment reads are the conflict-free ds_read_b128 of gemm.hpp.
// Rows >= M / >= N read a clamped valid row; their outputs are never stored.  K % BK == 0 (host).
#pragma once

#include "gemm.hpp"

namespace cgr {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes from g land at
// lds_dst + 16 l.  Issued from inline asm so hipcc's waitcnt pass does not track it (it would
// drain it with vmcnt(0) before LDS reads it cannot disambiguate); every wait for it is the
// kernel's own counted s_waitcnt vmcnt.  M0 is saved/restored (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const float* g, const float4* lds_dst) {
  const uint32_t la =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const lds_ptr_t)(lds_dst));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(la)
      : "memory");
}

template <int W, int RN, int KT, bool GATHER>
struct DmaShape {
  static constexpr int NT = W * 64, BM = 16 * W, BN = 16 * RN, BK = 16 * KT;
  static constexpr int A_F4 = KT * BM * 4;  // float4 per stage per A image
  static constexpr int B_F4 = KT * BN * 4;
  static constexpr int STAGE_F4 = A_F4 * (GATHER ? 2 : 1) + B_F4;
  static constexpr int NSTAGE = 3;
  static constexpr int EPI_W_F4 = 16 * BN / 4;  // one wave's 16 x BN accumulator image
  static constexpr int EPI_PER_STAGE = STAGE_F4 / EPI_W_F4;
  static constexpr int BPW = RN / W;                           // B row groups per wave
  static constexpr int DMA_PER_TILE = KT * ((GATHER ? 2 : 1) + BPW);  // per wave
  static_assert(RN % W == 0, "B row groups must divide evenly over the waves");
  static_assert(EPI_PER_STAGE * NSTAGE >= W, "epilogue images must fit in the ring");
};

struct DmaA {
  const float* a;    // [*, ld]
  const float* h;    // GATHER only
  const int* src;    // GATHER only: row m reads a[src[m]] - h[rev[m]]
  const int* rev;
  int64_t ld;
};

template <int W, int RN, int KT, bool GATHER, class EP>
__global__ __launch_bounds__(W * 64) void gemm_nt_dma_kernel(DmaA A, const float* __restrict__ B,
                                                             int64_t ldb, EP ep, int M, int N, int K,
                                                             int tiles_n) {
  using S = DmaShape<W, RN, KT, GATHER>;
  constexpr int BM = S::BM, BN = S::BN, BK = S::BK;
  // three distinct LDS objects (not one array): hipcc's waitcnt pass can then prove that the
  // fragment reads of one stage do not alias the DMA in flight into another and keeps the DMA in
  // flight instead of draining it with vmcnt(0) before every read (cdna_hip_programming.md §5,
  // "Projection GEMM" item 4(a)); the loop below is unrolled by 3 so every access is static.
  __shared__ float4 st0[S::STAGE_F4];
  __shared__ float4 st1[S::STAGE_F4];
  __shared__ float4 st2[S::STAGE_F4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // per-lane source rows: lane l of a DMA piece covers local row (l >> 2), slot (l & 3)
  const int lr = lane >> 2;
  const int chunk = (lane & 3) ^ lds_swz(lr);  // lds_swz depends on (row >> 2) & 3 only
  const float* pa;
  const float* ph = nullptr;
  {
    const int r = min(m0 + 16 * w + lr, M - 1);
    if constexpr (GATHER) {
      pa = A.a + (int64_t)A.src[r] * A.ld + 4 * chunk;
      ph = A.h + (int64_t)A.rev[r] * A.ld + 4 * chunk;
    } else {
      pa = A.a + (int64_t)r * A.ld + 4 * chunk;
    }
  }
  const float* pb[S::BPW];
#pragma unroll
  for (int j = 0; j < S::BPW; ++j) {
    const int r = min(n0 + 16 * (w + j * W) + lr, N - 1);
    pb[j] = B + (int64_t)r * ldb + 4 * chunk;
  }

  auto issue = [&](float4* st, int kb) {
#pragma unroll
    for (int c = 0; c < KT; ++c) {
      glds16(pa + kb + 16 * c, st + (c * BM + 16 * w) * 4);
      if constexpr (GATHER) glds16(ph + kb + 16 * c, st + S::A_F4 + (c * BM + 16 * w) * 4);
#pragma unroll
      for (int j = 0; j < S::BPW; ++j)
        glds16(pb[j] + kb + 16 * c,
               st + S::A_F4 * (GATHER ? 2 : 1) + (c * BN + 16 * (w + j * W)) * 4);
    }
  };

  floatx4 acc[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fg ^ lds_swz(fr);

  auto compute = [&](const float4* st) {
#pragma unroll
    for (int c = 0; c < KT; ++c) {
      float4 a = st[(c * BM + 16 * w + fr) * 4 + sw];
      if constexpr (GATHER) a = f4sub(a, st[S::A_F4 + (c * BM + 16 * w + fr) * 4 + sw]);
      float4 b[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j)
        b[j] = st[S::A_F4 * (GATHER ? 2 : 1) + (c * BN + 16 * j + fr) * 4 + sw];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, s), f4get(b[j], s), acc[j], 0, 0,
                                                        0);
    }
  };

  const int nk = K / BK;
  issue(st0, 0);
  if (nk > 1) issue(st1, BK);
  // Steady state: wait until this wave's DMAs for tile kt have landed (tile kt + 1 may stay in
  // flight), barrier (every wave's DMAs for kt landed; every wave finished computing kt - 1, so
  // the stage of tile kt + 2 is free), refill that stage, compute kt.
  auto step = [&](const float4* cur, float4* fill, int kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S::DMA_PER_TILE) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(fill, (kt + 2) * BK);
    compute(cur);
  };
  for (int kt = 0; kt < nk; kt += 3) {
    step(st0, st2, kt);
    if (kt + 1 < nk) step(st1, st0, kt + 1);
    if (kt + 2 < nk) step(st2, st1, kt + 2);
  }
  __syncthreads();  // every wave done reading the ring before the epilogue reuses it

  // epilogue, per wave (no block barrier): own 16 x BN accumulator image in the ring ->
  // float4 rows -> ep.apply4
  float4* img = w < S::EPI_PER_STAGE       ? st0 + w * S::EPI_W_F4
                : w < 2 * S::EPI_PER_STAGE ? st1 + (w - S::EPI_PER_STAGE) * S::EPI_W_F4
                                           : st2 + (w - 2 * S::EPI_PER_STAGE) * S::EPI_W_F4;
  float* C = reinterpret_cast<float*>(img);
  constexpr int LDC = BN;  // row stride of the per-wave image (floats)
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) C[(fg * 4 + r) * LDC + j * 16 + fr] = acc[j][r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  constexpr int C4 = BN / 4;
#pragma unroll
  for (int q = lane; q < 16 * C4; q += 64) {
    const int r = q / C4, c4 = q - r * C4;
    const float4 v = *reinterpret_cast<const float4*>(&C[r * LDC + 4 * c4]);
    ep.apply4(m0 + 16 * w + r, n0 + 4 * c4, v);
  }
}

template <int W, int RN, int KT, bool GATHER, class EP>
inline hipError_t launch_gemm_nt_dma(const DmaA& A, const float* B, int64_t ldb, const EP& ep,
                                     int M, int N, int K, hipStream_t st) {
  using S = DmaShape<W, RN, KT, GATHER>;
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K % S::BK != 0) return hipErrorInvalidValue;
  const int tm = (M + S::BM - 1) / S::BM, tn = (N + S::BN - 1) / S::BN;
  hipLaunchKernelGGL((gemm_nt_dma_kernel<W, RN, KT, GATHER, EP>), dim3(tm * tn), dim3(W * 64), 0,
                     st, A, B, ldb, ep, M, N, K, tn);
  return hipGetLastError();
}

}  // namespace cgr
