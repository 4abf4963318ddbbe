// fp32 GEMMs on the bf16 matrix cores (gfx950 v_mfma_f32_16x16x32_bf16): three-piece split.
//
// An fp32 operand x is split x = p0 + p1 + p2 (+ r): p0 = bf16(x) (round to nearest even),
// p1 = bf16(x - p0), p2 = bf16(x - p0 - p1), every remainder exact in fp32, |r| <= 2^-24 |x|.
// A product a.b is the sum of the six piece products that can reach 2^-16 |ab| (p1p1, p0p2, p2p0,
// p0p1, p1p0, p0p0; dropped terms <= 2^-23 |ab|), each bf16 x bf16 product exact, all accumulated
// in fp32 by the MFMA.  The error is at the level of an fp32 GEMM's own rounding
// (tools/experiments/fp16_split_precision_sim.py, profiles/r02_split_precision_experiment.txt:
// gradients 2-4e-7 vs 4-14e-7 for a plain fp32 GEMM against the fp64 oracle).  The bf16 MFMA
// runs 16x the fp32 MFMA rate (MI355X_MICROARCH.md § Matrix cores), so six of them cost 3/8 of
// the matrix-core time of v_mfma_f32_16x16x4_f32; what bounds these kernels is operand delivery.
//
// NT: C[m, n] = sum_k A(m, k) B(n, k) (epilogue functors of epilogues.hpp).
//   * B (a weight matrix, small, read by every workgroup) is split ONCE per training step by
//     b3_pack (kernels: b3_pack.hip) into an *image*: per 32-deep k step ks and piece p a plane of
//     Nimg rows x 64 bytes; row n's 16-byte slot s holds the lane-group-c chunk c = s ^ lds_swz(n)
//     (8 bf16 of k = 32 ks + b3_kperm(c, j)).  A workgroup copies its column block of the plane
//     verbatim into LDS: the swizzle is baked into the image, so every B fragment read is one
//     conflict-free ds_read_b128 (the 64-byte-row geometry of gemm.hpp).
//   * A (the streamed, large operand: gathered messages, dpre, x, s, dzn) goes straight from
//     global memory into the lane's registers in MFMA fragment shape -- each A element belongs to
//     exactly one wave, so it is loaded once and split once (VALU), never staged through LDS.
//     The k permutation b3_kperm (lane group g holds k = 4g..4g+3 and 16+4g..16+4g+3) makes each
//     fragment load two float4s whose four lane groups cover 64 contiguous bytes of the row.
//   * workgroup = WAVES waves, wave w owns RF 16-row fragments and all NF 16-column fragments of
//     the tile (BM = 16 WAVES RF rows x BN = 16 NF columns); B is double-buffered in LDS, A and B
//     register-prefetched one k step ahead (unconditional in-bounds loads: no vmcnt(0) merges).
//   * epilogue: accumulators -> LDS [BM][BN+4] -> float4 row pieces -> ep.apply4p, operand loads
//     issued first (gemm_nt_kernel's pattern).
#pragma once

#include <type_traits>

#include "gemm.hpp"

namespace cgr {

typedef __bf16 b3_bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b3_bf16x8 __attribute__((ext_vector_type(8)));
typedef float b3_floatx2 __attribute__((ext_vector_type(2)));
// 16-byte fragments / image chunks as a native vector (a HIP_vector_type uint4 copy lowers to a
// memcpy through a private alloca: scratch traffic and a vmcnt(0) right behind every load)
typedef uint32_t b3_u4 __attribute__((ext_vector_type(4)));

constexpr int B3_BK = 32;  // k per MFMA step

// element j (0..7) of lane group g holds k = b3_kperm(g, j) of a 32-deep step
__host__ __device__ constexpr int b3_kperm(int g, int j) {
  return j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4);
}

// 2 fp32 -> packed bf16x2 (RNE, v_cvt_pk_bf16_f32) and the two values it represents
__device__ __forceinline__ uint32_t b3_cvt2(float a, float b, float& fa, float& fb) {
  const uint32_t u =
      __builtin_bit_cast(uint32_t, __builtin_convertvector(b3_floatx2{a, b}, b3_bf16x2));
  fa = __uint_as_float(u << 16);
  fb = __uint_as_float(u & 0xffff0000u);
  return u;
}

// 8 fp32 -> P packed bf16x8 pieces (element 0 in the low half of word 0)
template <int P>
__device__ __forceinline__ void b3_split8(const float (&v)[8], b3_u4 (&out)[P]) {
  uint32_t w[P][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float a = v[2 * q], b = v[2 * q + 1];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      float fa, fb;
      w[i][q] = b3_cvt2(a, b, fa, fb);
      a -= fa;
      b -= fb;
    }
  }
#pragma unroll
  for (int i = 0; i < P; ++i) out[i] = b3_u4{w[i][0], w[i][1], w[i][2], w[i][3]};
}

// sched_group_barrier with a count known only after unrolling (the builtin needs literals)
template <int MASK>
__device__ __forceinline__ void b3_sgb(int n) {
  switch (n) {
    case 1: __builtin_amdgcn_sched_group_barrier(MASK, 1, 0); break;
    case 2: __builtin_amdgcn_sched_group_barrier(MASK, 2, 0); break;
    case 3: __builtin_amdgcn_sched_group_barrier(MASK, 3, 0); break;
    case 4: __builtin_amdgcn_sched_group_barrier(MASK, 4, 0); break;
    case 5: __builtin_amdgcn_sched_group_barrier(MASK, 5, 0); break;
    case 6: __builtin_amdgcn_sched_group_barrier(MASK, 6, 0); break;
    case 7: __builtin_amdgcn_sched_group_barrier(MASK, 7, 0); break;
    case 8: __builtin_amdgcn_sched_group_barrier(MASK, 8, 0); break;
    default: break;
  }
}

__device__ __forceinline__ floatx4 b3_mfma(const b3_u4& a, const b3_u4& b, const floatx4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b3_bf16x8, a),
                                                 __builtin_bit_cast(b3_bf16x8, b), c, 0, 0, 0);
}

// acc += a.b over one 32-deep step from three-piece fragments, smallest terms first
__device__ __forceinline__ floatx4 b3_mfma6(const b3_u4 (&a)[3], const b3_u4& b0, const b3_u4& b1,
                                            const b3_u4& b2, floatx4 c) {
  c = b3_mfma(a[1], b1, c);
  c = b3_mfma(a[0], b2, c);
  c = b3_mfma(a[2], b0, c);
  c = b3_mfma(a[0], b1, c);
  c = b3_mfma(a[1], b0, c);
  return b3_mfma(a[0], b0, c);
}

// ------------------------------------------------------------------------------------------
// B images
// ------------------------------------------------------------------------------------------
// column tiling of an NT GEMM with N output columns: tiles of nf 16-column fragments (nf from
// the instantiated set), image rows nimg = tiles * nf * 16 (rows >= N are zero)
struct B3Cols {
  int tiles, nf, nimg;
};
inline B3Cols b3_cols(int N) {
  const int nft = (N + 15) / 16;
  const int tiles = (nft + 12) / 13;
  int nf = (nft + tiles - 1) / tiles;
  static const int sizes[] = {1, 2, 3, 4, 6, 8, 11, 13};
  for (int s : sizes)
    if (s >= nf) {
      nf = s;
      break;
    }
  return B3Cols{tiles, nf, tiles * nf * 16};
}
inline int b3_nk(int K) { return (K + B3_BK - 1) / B3_BK; }
// b3_u4 elements of an image (3 pieces)
inline size_t b3_img_u4(int N, int K) { return (size_t)b3_nk(K) * 3 * b3_cols(N).nimg * 4; }

// one pack job: image rows [n_begin, n_begin + rows) from B(n, k) = src[n * ldn + k * ldk]
// (n < N real rows of this job, zero beyond; k < K real, zero beyond)
struct B3PackJob {
  const float* src;
  int64_t ldn, ldk;
  b3_u4* img;
  int n_begin, rows, N, K, nimg, nk;
};
constexpr int kMaxB3PackJobs = 24;  // per launch (kernel-argument size); b3_pack_all splits
struct B3PackJobs {
  B3PackJob job[kMaxB3PackJobs];
  int n;
};
hipError_t b3_pack(const B3PackJobs& jobs, hipStream_t st);
// append a job, launching the batch when it is full
inline hipError_t b3_pack_add(B3PackJobs& jobs, const B3PackJob& j, hipStream_t st) {
  if (jobs.n == kMaxB3PackJobs) {
    const hipError_t e = b3_pack(jobs, st);
    if (e != hipSuccess) return e;
    jobs.n = 0;
  }
  jobs.job[jobs.n++] = j;
  return hipSuccess;
}
// image job for B(n, k) = src[n * ldn + k * ldk], n < N, k < K, into an image of its own
inline B3PackJob b3_job(const float* src, int64_t ldn, int64_t ldk, int N, int K, void* img) {
  const B3Cols c = b3_cols(N);
  return B3PackJob{src, ldn, ldk, static_cast<b3_u4*>(img), 0, c.nimg, N, K, c.nimg, b3_nk(K)};
}

// ------------------------------------------------------------------------------------------
// NT kernel
// ------------------------------------------------------------------------------------------
template <int WAVES, int RF, int NF>
struct B3NtShape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RF, BN = NF * 16;
  static constexpr int BU4 = 3 * BN * 4;  // b3_u4 per B stage buffer (3 pieces x BN rows x 64 B)
  static constexpr int BPT = (BU4 + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr size_t STAGE_BYTES = 3 * BU4 * 16;
  static constexpr size_t EPI_BYTES = (size_t)BM * LDC * 4;
  static constexpr size_t LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
};

#ifdef CGR_B3_STAMPS
__device__ unsigned long long* b3_stamps;  // lab: [block][wave][4] s_memrealtime
#define B3_STAMP(i)                                                                          \
  if ((threadIdx.x & 63) == 0)                                                               \
  {                                                                                          \
    b3_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (i)] =     \
        __builtin_amdgcn_s_memrealtime();                                                    \
    b3_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + 4 + (i)] = \
        __builtin_amdgcn_s_memtime();                                                        \
  }
#else
#define B3_STAMP(i)
#endif
#ifndef CGR_B3_LDA
#define CGR_B3_LDA 4  // B fragment groups read from LDS ahead of the MFMAs that use them
#endif
#ifndef CGR_B3_LAB
#define CGR_B3_LAB 0  // lab ablations (bit mask): 1 no loop loads, 2 no loop barrier, 4 no LDS B reads, 8 no staging
#endif

// Pipeline (one barrier per k step, 3 LDS buffers for B):
//   iteration ks computes step ks from LDS buffer ks % 3 and A fragments afr[ks & 1], and stages
//   step ks+2's B block (registers -> buffer (ks+2) % 3, which step ks-1 read before the previous
//   barrier) and step ks+1's A fragments (split into afr[(ks+1) & 1]); the global loads of A(ks+2)
//   and B(ks+3) are issued at its start, so every load has a full step to land.
//   Staggered halves (CGR_B3_STAGGER): waves 0 .. W/2-1 compute then stage, waves W/2 .. W-1
//   stage then compute, so the two waves sharing a SIMD (w, w + W/2) keep the matrix pipe busy
//   while the other one waits on its loads, writes LDS and splits.
//   Column groups are processed in pairs (CGR_B3_JPAIR): the six-term chains of two groups
//   alternate, two independent accumulators in flight.
//   Staging past the end writes a buffer nobody reads any more (unconditional, branch-free).
template <int WAVES, int RF, int NF, bool NOMASK, class AL, class EP>
__global__ __launch_bounds__(WAVES * 64) void gemm_b3nt_kernel(AL al, const b3_u4* __restrict__ Bimg,
                                                               int nimg, EP ep, int M, int N,
                                                               int K, int tiles_n) {
  using S = B3NtShape<WAVES, RF, NF>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BU4 = S::BU4, BPT = S::BPT;
  extern __shared__ b3_u4 b3_lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + B3_BK - 1) / B3_BK;
  const int sw = fg ^ lds_swz(fr);  // lds_swz(16 j + fr) == lds_swz(fr)
  B3_STAMP(0)

  // ---- A: RF row fragments per lane, two float4 fetches per fragment per k step ----
  typename AL::Row arow[RF];
#pragma unroll
  for (int i = 0; i < RF; ++i) arow[i] = al.row(m0 + (w * RF + i) * 16 + fr, M);
  typedef typename AL::Raw ARaw[RF][2];
  // unconditional loads: k >= K reads in-bounds element 0 (the loaders clamp), never used
  auto fetchA = [&](ARaw& a, int ks) {
    if ((CGR_B3_LAB & 1) && ks > 2) return;
    const int kb = ks * B3_BK + 4 * fg;
#pragma unroll
    for (int i = 0; i < RF; ++i) {
      a[i][0] = al.fetch(arow[i], kb, K);
      a[i][1] = al.fetch(arow[i], kb + 16, K);
    }
  };
  auto splitA = [&](const ARaw& a, b3_u4 (&af)[RF][3], int ks) {
    const int kb = ks * B3_BK + 4 * fg;
#pragma unroll
    for (int i = 0; i < RF; ++i) {
      float4 u, v;
      if constexpr (NOMASK) {
        u = al.combine_nm(a[i][0]);
        v = al.combine_nm(a[i][1]);
      } else {
        u = al.combine(a[i][0], arow[i], kb, K);
        v = al.combine(a[i][1], arow[i], kb + 16, K);
      }
      const float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      b3_split8<3>(f, af[i]);
    }
  };
  // ---- B: the tile's column block of one (ks, piece) plane is BN * 4 contiguous b3_u4 ----
  int boff[BPT], loff[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    const int qq = q < BU4 ? q : BU4 - 1;
    const int piece = qq / (BN * 4), rem = qq - piece * (BN * 4);
    boff[p] = (piece * nimg + n0) * 4 + rem;
    loff[p] = q < BU4 ? q : -1;
  }
  typedef b3_u4 BRaw[BPT];
  auto fetchB = [&](BRaw& b, int ks) {  // steps past the end re-read the last plane (unused)
    if ((CGR_B3_LAB & 1) && ks > 2) return;
    const b3_u4* src = Bimg + (size_t)(ks < nk ? ks : nk - 1) * 3 * nimg * 4;
#pragma unroll
    for (int p = 0; p < BPT; ++p) b[p] = src[boff[p]];
  };
  auto storeB1 = [&](const BRaw& b, int p, int buf) {
    if (loff[p] >= 0) b3_lds[buf * BU4 + loff[p]] = b[p];
  };
  auto storeB = [&](const BRaw& b, int buf) {
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (loff[p] >= 0) b3_lds[buf * BU4 + loff[p]] = b[p];
  };

  floatx4 acc[RF][NF];
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  constexpr int LDA = CGR_B3_LDA < NF ? CGR_B3_LDA : NF - 1;
  // One step: the MFMAs of step ks (LDS buffer cb, fragments afc), column groups in pairs, with
  // the step's other work spread over them (the vector-memory path and the matrix pipe overlap
  // only when loads are interleaved with the MFMAs; issued as one burst per step they stall every
  // wave of the workgroup at once): the global loads of the next raw set (A(ksa) -> ya,
  // B(ksb) -> yb), the LDS stores of the current set's B block (xb -> buffer wb) and the split of
  // its A fragments (xa -> afn, step ksn).
  constexpr int AV = (int)(sizeof(typename AL::Raw) / 16);  // VMEM instructions per A fetch unit
  constexpr int NAS = RF * 2;                               // A fetch units per step
  constexpr int NLS = NAS + BPT;                            // load slots per step
  constexpr int NP = (NF + 1) / 2;                          // MFMA pairs per step
  auto step = [&](int cb, const b3_u4 (&afc)[RF][3], const BRaw& xb, int wb, const ARaw& xa,
                  b3_u4 (&afn)[RF][3], int ksn, ARaw& ya, int ksa, BRaw& yb, int ksb) {
    const b3_u4* Bs = b3_lds + cb * BU4;
    const int kba = ksa * B3_BK + 4 * fg;
    const b3_u4* bsrc = Bimg + (size_t)(ksb < nk ? ksb : nk - 1) * 3 * nimg * 4;
    auto load_slot = [&](int s) {
      if ((CGR_B3_LAB & 1) && ksa > 2) return;
      if (s < NAS) {
        ya[s >> 1][s & 1] = al.fetch(arow[s >> 1], kba + 16 * (s & 1), K);
      } else {
        yb[s - NAS] = bsrc[boff[s - NAS]];
      }
    };
    constexpr int RING = LDA + 2;
    b3_u4 bq[RING][3];
    auto rd = [&](int j) {
      const int o = (j * 16 + fr) * 4 + sw;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bq[j % RING][q] = (CGR_B3_LAB & 4) ? afc[0][q] + (b3_u4)(j) : Bs[q * BN * 4 + o];
    };
#pragma unroll
    for (int j = 0; j < LDA; ++j) rd(j);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int j = 2 * p;
      const bool two = j + 1 < NF;
      int nrd = 0;
      if (j + LDA < NF) {
        rd(j + LDA);
        nrd += 3;
      }
      if (two && j + 1 + LDA < NF) {
        rd(j + 1 + LDA);
        nrd += 3;
      }
      const b3_u4(&b)[3] = bq[j % RING];
      const b3_u4(&c)[3] = bq[(j + 1) % RING];
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        floatx4 x = acc[i][j], y = two ? acc[i][j + 1] : x;
        x = b3_mfma(afc[i][1], b[1], x);
        if (two) y = b3_mfma(afc[i][1], c[1], y);
        x = b3_mfma(afc[i][0], b[2], x);
        if (two) y = b3_mfma(afc[i][0], c[2], y);
        x = b3_mfma(afc[i][2], b[0], x);
        if (two) y = b3_mfma(afc[i][2], c[0], y);
        x = b3_mfma(afc[i][0], b[1], x);
        if (two) y = b3_mfma(afc[i][0], c[1], y);
        x = b3_mfma(afc[i][1], b[0], x);
        if (two) y = b3_mfma(afc[i][1], c[0], y);
        x = b3_mfma(afc[i][0], b[0], x);
        if (two) y = b3_mfma(afc[i][0], c[0], y);
        acc[i][j] = x;
        if (two) acc[i][j + 1] = y;
      }
      // this pair's share of the load slots and of the B stores
      int nvm = 0, nst = 0;
      const int s0 = p * NLS / NP, s1 = (p + 1) * NLS / NP;
#pragma unroll
      for (int s = 0; s < NLS; ++s)
        if (s >= s0 && s < s1) {
          load_slot(s);
          nvm += s < NAS ? AV : 1;
        }
      if (!(CGR_B3_LAB & 8)) {
        const int w0 = p * BPT / NP, w1 = (p + 1) * BPT / NP;
#pragma unroll
        for (int q = 0; q < BPT; ++q)
          if (q >= w0 && q < w1) {
            storeB1(xb, q, wb);
            ++nst;
          }
        if (p == NP / 2) splitA(xa, afn, ksn);
      }
      constexpr int MQ = 4 * RF;  // a third of a pair's MFMAs
      b3_sgb<0x100>(nrd);                                    // ds_read
      if (two) b3_sgb<0x008>(MQ); else b3_sgb<0x008>(MQ / 2);  // MFMA
      b3_sgb<0x020>(nvm);                                    // global load
      if (two) b3_sgb<0x008>(MQ); else b3_sgb<0x008>(MQ / 2);
      b3_sgb<0x200>(nst);                                    // ds_write
      if (two) b3_sgb<0x008>(MQ); else b3_sgb<0x008>(MQ);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!(CGR_B3_LAB & 2)) __syncthreads();
  };

  {  // prologue: buffers 0, 1 <- B(0), B(1); afr0 <- A(0); raw set 0 <- A(1), B(2)
    ARaw a0, xa0, xa1;
    BRaw b0, b1, xb0, xb1;
    fetchA(a0, 0);
    fetchB(b0, 0);
    fetchB(b1, 1);
    fetchA(xa0, 1);
    fetchB(xb0, 2);
    b3_u4 afr0[RF][3], afr1[RF][3];
    storeB(b0, 0);
    storeB(b1, 1);
    splitA(a0, afr0, 0);
    __syncthreads();
    B3_STAMP(1)
    int cb = 0;  // LDS buffer of step ks (ks % 3)
    for (int ks = 0; ks < nk; ks += 2) {
      // even step: consume set 0 (A(ks+1), B(ks+2)), fill set 1 with A(ks+2), B(ks+3)
      step(cb, afr0, xb0, cb == 0 ? 2 : cb - 1, xa0, afr1, ks + 1, xa1, ks + 2, xb1, ks + 3);
      if (ks + 1 >= nk) break;
      cb = cb == 2 ? 0 : cb + 1;
      // odd step: consume set 1 (A(ks+2), B(ks+3)), fill set 0 with A(ks+3), B(ks+4)
      step(cb, afr1, xb1, cb == 0 ? 2 : cb - 1, xa1, afr0, ks + 2, xa0, ks + 3, xb0, ks + 4);
      cb = cb == 2 ? 0 : cb + 1;
    }
  }

  B3_STAMP(2)
  // ---- epilogue (the stage buffers are dead after the last barrier) ----
  constexpr int C4 = BN / 4;
  constexpr int EIT = (BM * C4 + NT - 1) / NT;
  const typename EP::Ctx cx = ep.ctx();
  typename EP::Pre pv[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int q = min(tid + it * NT, BM * C4 - 1);
    const int r = q / C4, c4 = q - r * C4;
    pv[it] = ep.pre4(m0 + r, n0 + 4 * c4);
  }
  float* C = reinterpret_cast<float*>(b3_lds);
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[((w * RF + i) * 16 + fg * 4 + r) * S::LDC + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int q = tid + it * NT;
    if (q < BM * C4) {
      const int r = q / C4, c4 = q - r * C4;
      const float4 v = *reinterpret_cast<const float4*>(&C[r * S::LDC + 4 * c4]);
      ep.apply4p(m0 + r, n0 + 4 * c4, v, pv[it], cx);
    }
  }
  B3_STAMP(3)
}

template <int WAVES, int RF, int NF, bool NOMASK, class AL, class EP>
inline hipError_t launch_b3nt_t(const AL& al, const b3_u4* Bimg, int nimg, const EP& ep, int M,
                                int N, int K, int tiles_n, hipStream_t st) {
  using S = B3NtShape<WAVES, RF, NF>;
  auto kern = gemm_b3nt_kernel<WAVES, RF, NF, NOMASK, AL, EP>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int tm = (M + S::BM - 1) / S::BM;
  hipLaunchKernelGGL(kern, dim3(tm * tiles_n), dim3(WAVES * 64), S::LDS_BYTES, st, al, Bimg, nimg,
                     ep, M, N, K, tiles_n);
  return hipGetLastError();
}

// workgroup rows: 8 waves (128 rows) when that still gives ~200+ workgroups, else 4 (64 rows)
#ifndef CGR_B3_WAVES
#define CGR_B3_WAVES 0  // 0: by size; 4 / 8: forced (lab)
#endif
inline int b3nt_waves(int M, int N) {
  if (CGR_B3_WAVES) return CGR_B3_WAVES;
  const int tiles_n = b3_cols(N).tiles;
  return ((M + 127) / 128) * tiles_n >= 192 ? 8 : 4;
}

// C = A B^T with B given as its image (b3_pack of the same N, K).  M, N, K > 0.
template <class AL, class EP>
inline hipError_t launch_b3nt(const AL& al, const b3_u4* Bimg, const EP& ep, int M, int N, int K,
                              hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const B3Cols c = b3_cols(N);
  const bool w8 = b3nt_waves(M, N) == 8;
  // unmasked A when K % 4 == 0: every fetched float4 is either all-valid or past K (clamped to
  // finite in-bounds data, multiplied by the image's zero rows)
  auto go = [&](auto NFc) -> hipError_t {
    constexpr int NF = decltype(NFc)::value;
#ifndef CGR_B3_RF
#define CGR_B3_RF 1  // row fragments per wave of the 128-row tiles (2: 4 waves x 32 rows)
#endif
    constexpr int W8 = 8 / CGR_B3_RF;
    if (K % 4 == 0)
      return w8 ? launch_b3nt_t<W8, CGR_B3_RF, NF, true>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st)
                : launch_b3nt_t<4, 1, NF, true>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st);
    return w8 ? launch_b3nt_t<W8, CGR_B3_RF, NF, false>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st)
              : launch_b3nt_t<4, 1, NF, false>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st);
  };
  switch (c.nf) {
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    case 4: return go(std::integral_constant<int, 4>{});
    case 6: return go(std::integral_constant<int, 6>{});
    case 8: return go(std::integral_constant<int, 8>{});
    case 11: return go(std::integral_constant<int, 11>{});
    case 13: return go(std::integral_constant<int, 13>{});
  }
  return hipErrorInvalidValue;
}

}  // namespace cgr
