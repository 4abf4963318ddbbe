// Bottleneck ladder for the NT GEMM main loop at the layer shape (E 15360 x 400 x 400, plain rows).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/gemm_probe.hip -o gemm_probe
// MODE 0 full loop | 1 no global loads in the loop (LDS tile rewritten from the prologue regs)
//      2 no MFMAs | 3 MFMA + LDS reads only (no loads, no stores, no barriers in the loop)
//      4 full loop, no epilogue stores
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"

using namespace cgr;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

template <int MODE, int WAVES, int RN, int KT = 1>
__global__ __launch_bounds__(WAVES * 64) void probe(const float* __restrict__ A,
                                                    const float* __restrict__ B,
                                                    float* __restrict__ C, int M, int N, int K,
                                                    int tiles_n) {
  constexpr int NT = WAVES * 64, BM = WAVES * 16, BN = RN * 16, CPR = 4 * KT;
  constexpr int ACH = BM * CPR, BCH = BN * CPR;
  constexpr int APT = ACH / NT, BPT = (BCH + NT - 1) / NT;
  __shared__ float4 lds[2 * (ACH + BCH)];
  float4* As = lds;
  float4* Bs = lds + 2 * ACH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* ap[APT];
  int adst[APT], akof[APT];
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT, r = q / CPR, kc = q % CPR;
    ap[p] = A + (int64_t)min(m0 + r, M - 1) * K;
    akof[p] = kc * 4;
    adst[p] = ((kc >> 2) * BM + r) * 4 + ((kc & 3) ^ lds_swz(r));
  }
  const float* bp[BPT];
  int bdst[BPT], bkof[BPT];
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT, r = q / CPR, kc = q % CPR;
    const bool in = q < BCH;
    bp[p] = B + (int64_t)min(n0 + (in ? r : 0), N - 1) * K;
    bkof[p] = kc * 4;
    bdst[p] = in ? ((kc >> 2) * BN + r) * 4 + ((kc & 3) ^ lds_swz(r)) : -1;
  }
  float4 ra[APT], rb[BPT];
  floatx4 acc[RN];
  for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / (16 * KT);
  for (int p = 0; p < APT; ++p) ra[p] = *reinterpret_cast<const float4*>(ap[p] + akof[p]);
  for (int p = 0; p < BPT; ++p) rb[p] = *reinterpret_cast<const float4*>(bp[p] + bkof[p]);
  for (int p = 0; p < APT; ++p) As[adst[p]] = ra[p];
  for (int p = 0; p < BPT; ++p)
    if (bdst[p] >= 0) Bs[bdst[p]] = rb[p];
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4, sw = fg ^ lds_swz(fr);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = (MODE == 3 || MODE == 5) ? 0 : (kt & 1);
    const bool more = kt + 1 < nk;
    const int kb = (kt + 1) * 16 * KT;
    if (MODE != 1 && MODE != 3 && MODE != 5 && more) {  // MODE 6/7: loads + register MFMAs
      for (int p = 0; p < APT; ++p) ra[p] = *reinterpret_cast<const float4*>(ap[p] + kb + akof[p]);
      for (int p = 0; p < BPT; ++p) rb[p] = *reinterpret_cast<const float4*>(bp[p] + kb + bkof[p]);
    }
    if (MODE == 5 || MODE == 6 || MODE == 7) {  // MFMA from registers (6/7: beside the loads)
      float4 a = ra[0], b0 = rb[0];
#pragma unroll
      for (int c = 0; c < KT; ++c)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, s), f4get(b0, s), acc[j], 0, 0,
                                                          0);
    } else if (MODE != 2) {
#pragma unroll
      for (int c = 0; c < KT; ++c) {
        const float4* Ac = As + cur * ACH + c * BM * 4;
        const float4* Bc = Bs + cur * BCH + c * BN * 4;
        float4 a = Ac[(w * 16 + fr) * 4 + sw], b[RN];
        for (int j = 0; j < RN; ++j) b[j] = Bc[(j * 16 + fr) * 4 + sw];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, s), f4get(b[j], s), acc[j], 0,
                                                          0, 0);
      }
    }
    if (MODE == 6) {  // consume the loads (no LDS, no barrier)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (MODE == 7) {  // loads -> LDS, barrier, but MFMA operands from registers
      if (more) {
        float4* An = As + (cur ^ 1) * ACH;
        float4* Bn = Bs + (cur ^ 1) * BCH;
        for (int p = 0; p < APT; ++p) An[adst[p]] = ra[p];
        for (int p = 0; p < BPT; ++p)
          if (bdst[p] >= 0) Bn[bdst[p]] = rb[p];
      }
      __syncthreads();
    }
    if (MODE != 3 && MODE != 5 && MODE != 6 && MODE != 7) {
      if (more) {
        float4* An = As + (cur ^ 1) * ACH;
        float4* Bn = Bs + (cur ^ 1) * BCH;
        for (int p = 0; p < APT; ++p) An[adst[p]] = ra[p];
        for (int p = 0; p < BPT; ++p)
          if (bdst[p] >= 0) Bn[bdst[p]] = rb[p];
      }
      __syncthreads();
    }
  }
  if (MODE == 2 || MODE == 6) {  // keep the loads alive
    float s = 0.f;
    for (int p = 0; p < APT; ++p) s += ra[p].x;
    for (int p = 0; p < BPT; ++p) s += rb[p].y;
    acc[0][0] += s * 1e-30f;
  }
  if (MODE == 4) {
    if (acc[0][0] == 12345.678f) C[tid] = acc[1][1];
    return;
  }
  for (int j = 0; j < RN; ++j)
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + w * 16 + fg * 4 + r, col = n0 + j * 16 + fr;
      if (row < M && col < N) C[(int64_t)row * N + col] = acc[j][r];
    }
}

// warp-specialised variant: CW consumer waves (16 rows x BN cols each: LDS reads + MFMA only)
// and PW producer waves (global loads -> ds_write of the next stage), one barrier per k-step.
template <int CW, int PW, int RN, int S>
__global__ __launch_bounds__((CW + PW) * 64) void wsprobe(const float* __restrict__ A,
                                                          const float* __restrict__ B,
                                                          float* __restrict__ C, int M, int N,
                                                          int K, int tiles_n) {
  constexpr int BM = CW * 16, BN = RN * 16, ACH = BM * 4, BCH = BN * 4, PT = PW * 64;
  constexpr int APT = (ACH + PT - 1) / PT, BPT = (BCH + PT - 1) / PT;
  __shared__ float4 lds[S * (ACH + BCH)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / 16;
  const bool producer = w >= CW;
  const int pt = tid - CW * 64;
  const float* ap[APT];
  int adst[APT];
  const float* bp[BPT];
  int bdst[BPT];
  if (producer) {
#pragma unroll
    for (int p = 0; p < APT; ++p) {
      const int q = pt + p * PT, r = q >> 2, kc = q & 3;
      const bool in = q < ACH;
      ap[p] = A + (int64_t)min(m0 + (in ? r : 0), M - 1) * K + kc * 4;
      adst[p] = in ? r * 4 + (kc ^ lds_swz(r)) : -1;
    }
#pragma unroll
    for (int p = 0; p < BPT; ++p) {
      const int q = pt + p * PT, r = q >> 2, kc = q & 3;
      const bool in = q < BCH;
      bp[p] = B + (int64_t)min(n0 + (in ? r : 0), N - 1) * K + kc * 4;
      bdst[p] = in ? r * 4 + (kc ^ lds_swz(r)) : -1;
    }
  }
  auto produce = [&](int t) {
    float4* As = lds + (t % S) * (ACH + BCH);
    float4* Bs = As + ACH;
    float4 ra[APT], rb[BPT];
#pragma unroll
    for (int p = 0; p < APT; ++p) ra[p] = *reinterpret_cast<const float4*>(ap[p] + t * 16);
#pragma unroll
    for (int p = 0; p < BPT; ++p) rb[p] = *reinterpret_cast<const float4*>(bp[p] + t * 16);
#pragma unroll
    for (int p = 0; p < APT; ++p)
      if (adst[p] >= 0) As[adst[p]] = ra[p];
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bdst[p] >= 0) Bs[bdst[p]] = rb[p];
  };
  floatx4 acc[RN];
#pragma unroll
  for (int j = 0; j < RN; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4, sw = fg ^ lds_swz(fr);
  if (producer) {
    for (int t = 0; t < S - 1 && t < nk; ++t) produce(t);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    if (producer) {
      if (t + S - 1 < nk) produce(t + S - 1);
    } else {
      const float4* As = lds + (t % S) * (ACH + BCH);
      const float4* Bs = As + ACH;
      const float4 a = As[(w * 16 + fr) * 4 + sw];
      float4 b[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) b[j] = Bs[(j * 16 + fr) * 4 + sw];
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, s), f4get(b[j], s), acc[j], 0, 0,
                                                        0);
    }
    __syncthreads();
  }
  if (!producer) {
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + w * 16 + fg * 4 + r, col = n0 + j * 16 + fr;
        if (row < M && col < N) C[(int64_t)row * N + col] = acc[j][r];
      }
  }
}

template <int CW, int PW, int RN, int S>
static float runws(const float* A, const float* B, float* C, int M, int N, int K, hipStream_t st,
                   int reps) {
  const int tm = (M + CW * 16 - 1) / (CW * 16), tn = (N + RN * 16 - 1) / (RN * 16);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((wsprobe<CW, PW, RN, S>), dim3(tm * tn), dim3((CW + PW) * 64), 0, st, A, B, C,
                     M, N, K, tn);
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((wsprobe<CW, PW, RN, S>), dim3(tm * tn), dim3((CW + PW) * 64), 0, st, A, B,
                       C, M, N, K, tn);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

// weight-stationary in REGISTERS: wave w of column group cg owns output columns
// [cg*80 + 16w, +16) and keeps W[those 16 columns][0..K) in 25 float4 = 100 VGPRs; the workgroup
// streams 16-row A tiles through LDS (double buffered) over a persistent row range.
template <int KC>  // KC = K / 16 chunks
__global__ __launch_bounds__(320) void wregprobe(const float* __restrict__ A,
                                                 const float* __restrict__ B,
                                                 float* __restrict__ C, int M, int N, int K,
                                                 int groups) {
  constexpr int K4 = KC * 4;  // float4 per row
  __shared__ float4 As[2][16 * K4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cg = blockIdx.x % 5, rg = blockIdx.x / 5;
  const int fr = lane & 15, fg = lane >> 4, sw = fg ^ lds_swz(fr);
  const int n = cg * 80 + w * 16 + fr;
  float4 breg[KC];
#pragma unroll
  for (int c = 0; c < KC; ++c)
    breg[c] = *reinterpret_cast<const float4*>(B + (int64_t)min(n, N - 1) * K + 16 * c + 4 * fg);
  const int ntiles = M / 16;
  auto load = [&](int t, int buf) {
    for (int q = tid; q < 16 * K4; q += 320) {
      const int r = q / K4, kc = q - r * K4;  // kc = float4 index along k
      const float4 v = *reinterpret_cast<const float4*>(A + (int64_t)(t * 16 + r) * K + 4 * kc);
      As[buf][((kc >> 2) * 16 + r) * 4 + ((kc & 3) ^ lds_swz(r))] = v;
    }
  };
  int t = rg, buf = 0;
  if (t < ntiles) load(t, 0);
  __syncthreads();
  for (; t < ntiles; t += groups) {
    const int tn = t + groups;
    if (tn < ntiles) load(tn, buf ^ 1);
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
    const float4* Ab = As[buf];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const float4 a = Ab[(c * 16 + fr) * 4 + sw];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f4get(a, j), f4get(breg[c], j), acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = t * 16 + fg * 4 + r;
      if (n < N) C[(int64_t)row * N + n] = acc[r];
    }
    __syncthreads();
    buf ^= 1;
  }
}

template <int KC>
static float runwreg(const float* A, const float* B, float* C, int M, int N, int K, hipStream_t st,
                     int reps, int groups) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((wregprobe<KC>), dim3(5 * groups), dim3(320), 0, st, A, B, C, M, N, K, groups);
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((wregprobe<KC>), dim3(5 * groups), dim3(320), 0, st, A, B, C, M, N, K,
                       groups);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

template <int MODE, int WAVES, int RN, int KT = 1>
static float run(const float* A, const float* B, float* C, int M, int N, int K, hipStream_t st,
                 int reps) {
  const int tm = (M + WAVES * 16 - 1) / (WAVES * 16), tn = (N + RN * 16 - 1) / (RN * 16);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((probe<MODE, WAVES, RN, KT>), dim3(tm * tn), dim3(WAVES * 64), 0, st, A, B, C, M,
                     N, K, tn);
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((probe<MODE, WAVES, RN, KT>), dim3(tm * tn), dim3(WAVES * 64), 0, st, A, B, C,
                       M, N, K, tn);
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / reps;
}

int main() {
  const int M = 15360, N = 400, K = 416;
  float *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 4));
  CK(hipMalloc(&B, (size_t)N * K * 4));
  CK(hipMalloc(&C, (size_t)M * N * 4));
  CK(hipMemset(A, 0, (size_t)M * K * 4));
  CK(hipMemset(B, 0, (size_t)N * K * 4));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const double fl = 2.0 * M * N * K;
  for (int round = 0; round < 3; ++round) {
    printf("K=416 regular w4 full %7.2f | wreg groups 51 %7.2f 102 %7.2f 153 %7.2f 204 %7.2f\n",
           run<0, 4, 5, 1>(A, B, C, M, N, K, st, 20), runwreg<26>(A, B, C, M, N, K, st, 20, 51),
           runwreg<26>(A, B, C, M, N, K, st, 20, 102), runwreg<26>(A, B, C, M, N, K, st, 20, 153),
           runwreg<26>(A, B, C, M, N, K, st, 20, 204));
  }
  (void)fl;
  return 0;
}
