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

#include "epilogues.hpp"
#include "gemm.hpp"
#include "handoff.hpp"
#include "reduce.hpp"
#include "stamps.hpp"

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
// the instantiated fragment counts per tile (launch_b3nt's switch)
inline int b3_nf_snap(int nf) {
  static const int sizes[] = {1, 2, 3, 4, 6, 7, 8, 11, 13};
  for (int s : sizes)
    if (s >= nf) return s;
  return 13;
}
inline B3Cols b3_cols(int N) {
  const int nft = (N + 15) / 16;
  const int tiles = (nft + 12) / 13;
  int nf = (nft + tiles - 1) / tiles;
  nf = b3_nf_snap(nf);
  return B3Cols{tiles, nf, tiles * nf * 16};
}
inline int b3_nk(int K) { return (K + B3_BK - 1) / B3_BK; }
// b3_u4 elements of an image (3 pieces) in the column tiling c
inline size_t b3_img_u4(const B3Cols& c, int K) { return (size_t)b3_nk(K) * 3 * c.nimg * 4; }
inline size_t b3_img_u4(int N, int K) { return b3_img_u4(b3_cols(N), K); }

// one pack job: image rows [n_begin, n_begin + rows) from B(n, k) = src[n * ldn + k * ldk]
// (n < N real rows of this job, zero beyond; k < K real, zero beyond), times kscale[k] when set
struct B3PackJob {
  const float* src;
  int64_t ldn, ldk;
  b3_u4* img;
  int n_begin, rows, N, K, nimg, nk;
  const float* kscale;
};
constexpr int kMaxB3PackJobs = 24;  // per launch (kernel-argument size); b3_pack_all splits
struct B3PackJobs {
  B3PackJob job[kMaxB3PackJobs];
  int n;
};
// small independent jobs that ride in a pack launch (the forward start, gnn_fwd.hip: one launch
// per queue instead of three); each part is off when its pointer is null
struct B3PackRiders {
  // t_dst[c * t_ld_dst + r] = t_src[r * t_ld_src + c], r < t_rows, c < t_cols
  const float* t_src = nullptr;
  int64_t t_ld_src = 0;
  float* t_dst = nullptr;
  int64_t t_ld_dst = 0;
  int t_rows = 0, t_cols = 0;
  // z_u4 16-byte words of zeros at z_dst
  void* z_dst = nullptr;
  int64_t z_u4 = 0;
  // p_dst[r, :p_ld] = p_src[r, :p_F] then zeros, r < p_rows (pad_rows; p_ld % 4 == 0)
  const float* p_src = nullptr;
  float* p_dst = nullptr;
  int64_t p_rows = 0;
  int p_F = 0, p_ld = 0;
};
hipError_t b3_pack(const B3PackJobs& jobs, hipStream_t st, const B3PackRiders* riders = nullptr);
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
inline B3PackJob b3_job(const float* src, int64_t ldn, int64_t ldk, int N, int K, void* img,
                        const B3Cols& c) {
  return B3PackJob{src, ldn, ldk, static_cast<b3_u4*>(img), 0, c.nimg, N, K, c.nimg, b3_nk(K)};
}
inline B3PackJob b3_job(const float* src, int64_t ldn, int64_t ldk, int N, int K, void* img) {
  return b3_job(src, ldn, ldk, N, K, img, b3_cols(N));
}

// ------------------------------------------------------------------------------------------
// NT kernel
// ------------------------------------------------------------------------------------------
// epilogue functors with kTile = true take the whole accumulator tile (EpLayerBwdSeg)
template <class EP, class = void>
struct b3_ep_tile : std::false_type {};
template <class EP>
struct b3_ep_tile<EP, std::void_t<decltype(EP::kTile)>> : std::bool_constant<EP::kTile> {};

// epilogue functors with kAddend = true take their addend (bias, skip term, Q, ...) into the
// accumulators in MFMA layout: its loads are issued in the last k step (EpLayer, EpReadoutQ)
template <class EP, class = void>
struct b3_ep_addend : std::false_type {};
template <class EP>
struct b3_ep_addend<EP, std::void_t<decltype(EP::kAddend)>> : std::bool_constant<EP::kAddend> {};
#ifdef CGR_NO_ADDEND
template <class EP>
struct b3_ep_addend_off : std::false_type {};
#define b3_ep_addend b3_ep_addend_off
#endif

// epilogue functors with kAct = true apply an activation `act`: the kernel switches on it once,
// outside its epilogue loop, and hands it to the functor as a template constant
template <class EP, class = void>
struct b3_ep_act : std::false_type {};
template <class EP>
struct b3_ep_act<EP, std::void_t<decltype(EP::kAct)>> : std::bool_constant<EP::kAct> {};

// epilogue functors with kSideBlock = true may carry one workgroup of independent work (EpSplit2:
// the graph bookkeeping beside the x-GEMM, prep_one.hpp): when ep.side_on, the launch has one
// extra, LAST workgroup (the tiles keep their XCD mapping) that runs ep.side(lds) instead of a
// tile, with the tile's LDS
template <class EP, class = void>
struct b3_ep_side : std::false_type {};
template <class EP>
struct b3_ep_side<EP, std::void_t<decltype(EP::kSideBlock)>> : std::bool_constant<EP::kSideBlock> {};

// dynamic LDS bytes of a BM x BN NT workgroup (B3NtShape::LDS_BYTES)
constexpr size_t b3nt_lds_bytes(int BM, int BN) {
  const size_t stage = (size_t)3 * (3 * BN * 4) * 16;
  const size_t epi = (size_t)BM * (BN + 4) * 4 + (size_t)(BM + 2) * 4 + 64 + (size_t)(BM + 1) * 4;
  return stage > epi ? stage : epi;
}

template <int WAVES, int RF, int NF>
struct B3NtShape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RF, BN = NF * 16;
  static constexpr int BU4 = 3 * BN * 4;  // b3_u4 per B stage buffer (3 pieces x BN rows x 64 B)
  static constexpr int BPT = (BU4 + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr size_t STAGE_BYTES = 3 * BU4 * 16;
  // + the dst of rows m0 - 1 .. m0 + BM (EpLayerSeg, EpLayerBwdSeg), 16 floats of reduction
  // scratch (EpLayerBwdSeg; kernels with static LDS cannot be given the full 160 KB dynamically)
  // and the tile's segment-start rows + terminator (EpLayerSeg's segment pass)
  static constexpr size_t EPI_BYTES = (size_t)BM * LDC * 4 + (BM + 2) * 4 + 64 + (BM + 1) * 4;
  static constexpr size_t LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
  static_assert(LDS_BYTES == b3nt_lds_bytes(BM, BN), "b3nt_lds_bytes");
};

#ifndef CGR_B3_LDA
#define CGR_B3_LDA 4
#endif
#ifndef CGR_B3_RA_FENCE
#define CGR_B3_RA_FENCE 1
#endif
constexpr int B3_LDA = CGR_B3_LDA;  // B fragment groups read from LDS ahead of the MFMAs using them
constexpr bool kB3ReadAheadFence = CGR_B3_RA_FENCE;
#ifndef CGR_B3_STEP_ACC
#define CGR_B3_STEP_ACC 0
#endif
constexpr bool kB3StepAcc = CGR_B3_STEP_ACC;
#ifndef CGR_B3_FLAT
#define CGR_B3_FLAT 1
#endif
constexpr bool kB3FlatEpilogue = CGR_B3_FLAT;  // flat epilogue passes + compact segment pass
#ifndef CGR_B3_SEGMERGE
#define CGR_B3_SEGMERGE 1
#endif
constexpr bool kB3SegMerge = CGR_B3_SEGMERGE;  // the forward's apply and segment sums in one pass

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
  int nwg = gridDim.x;
  if constexpr (b3_ep_side<EP>::value) {
    if (ep.side_on) {
      if (blockIdx.x == gridDim.x - 1) {
        ep.side(b3_lds);
        return;
      }
      --nwg;
    }
  }
  CGR_STAMP_BEGIN();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (K + B3_BK - 1) / B3_BK;
  const int sw = fg ^ lds_swz(fr);  // lds_swz(16 j + fr) == lds_swz(fr)

  // ---- epilogue mapping: one float4 column group per thread, rows er0 + RPP * it ----
  constexpr int C4 = BN / 4;
  constexpr int RPP = NT / C4;                // rows per pass
  constexpr int EIT = (BM + RPP - 1) / RPP;   // passes
  constexpr bool SEG = EP::kSeg;  // the epilogue also sums the tile's dst segments (EpLayerSeg)
  // the whole tile goes to the functor (EpLayerBwdSeg: ep_bwd.hpp)
  constexpr bool TILE = b3_ep_tile<EP>::value;
  static_assert(NT >= BM + 2 && RPP >= 1, "one dst per thread; one row group per pass");
  const bool eact = tid < RPP * C4;
  const int ec4 = eact ? tid % C4 : 0, er0 = tid / C4;
  const int ecol = n0 + 4 * ec4;
  // Flat passes: epilogues without per-column constants (the addend forms, whose column terms
  // are already in the accumulators; the whole-tile functors) take item q = tid + NT * it of the
  // tile's BM x C4 float4 pieces, row q / C4, column group q % C4 -- every lane busy in every
  // pass (at BM 128 x 52 groups: 13 passes of 512 instead of 15 passes of 468 lanes)
  constexpr bool FLAT = kB3FlatEpilogue && (TILE || b3_ep_addend<EP>::value);
  constexpr int EITF = (BM * C4 + NT - 1) / NT;
  constexpr int EP_IT = FLAT ? EITF : EIT;
  // issued in the prologue behind the first operand loads, used after the main loop: the column
  // group's constants (bias, ...) and, for the segmented epilogues, the dst of rows
  // m0 - 1 .. m0 + BM (one per thread)
  typename EP::Ctx cx;
  int sdv = 0;
  bool sstart = true;  // row tid starts a dst segment in the tile (handoff.hpp seg_*)
  auto epilogue_consts = [&]() {
    if constexpr (b3_ep_addend<EP>::value)
      cx = ep.ctx_add();  // the column constants travel with the addend
    else
      cx = ep.ctx(ecol);
    if constexpr (SEG || TILE) {
      const int r = m0 - 1 + tid;
      const int d = ep.dst_s[min(max(r, 0), M - 1)];
      sdv = (r >= 0 && r < M) ? d : -1 - (r >= M);  // distinct sentinels outside [0, M)
      const int d1 = ep.dst_s[min(r + 1, M - 1)];    // row tid itself
      sstart = tid == 0 || r + 1 >= M || d1 != d;
    }
  };

  // ---- A: RF row fragments per lane, two float4 fetches per fragment per k step ----
  typename AL::Row arow[RF];
#pragma unroll
  for (int i = 0; i < RF; ++i) arow[i] = al.row(m0 + (w * RF + i) * 16 + fr, M);
  typedef typename AL::Raw ARaw[RF][2];
  // unconditional loads: k >= K reads in-bounds element 0 (the loaders clamp), never used
  auto fetchA = [&](ARaw& a, int ks) {
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

  // read-ahead depth: 2 groups at 11 fragment columns (4 spill the gathered-A kernels there)
  constexpr int LDA = NF == 11 ? 2 : (B3_LDA < NF ? B3_LDA : NF - 1);
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
        bq[j % RING][q] = Bs[q * BN * 4 + o];
    };
#pragma unroll
    for (int j = 0; j < LDA; ++j) rd(j);
    // the read-ahead is issued here, ahead of everything (else the scheduler fills each pair's
    // ds_read group with that pair's own reads and waits on them right away)
    if constexpr (kB3ReadAheadFence) __builtin_amdgcn_sched_barrier(0);
    floatx4 carx[RF], cary[RF];  // kB3StepAcc: the previous pair's step sums
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
        // kB3StepAcc: the step's six products into a zero accumulator, then one fp32 add into
        // the running sum (the matrix core aligns every product of an MFMA to its largest
        // operand, accumulator included: the small pieces' products would be rounded at the
        // running sum's ulp, tools/diag/bf16_round_probe.hip).  The add of pair p is issued
        // behind pair p + 1's MFMAs (carry): only two pairs' temporaries are live.
        floatx4 x = kB3StepAcc ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i][j];
        floatx4 y = kB3StepAcc ? x : (two ? acc[i][j + 1] : x);
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
        if constexpr (kB3StepAcc) {
          if (p > 0) {
            acc[i][j - 2] += carx[i];
            acc[i][j - 1] += cary[i];  // the previous pair always has two columns
          }
          carx[i] = x;
          cary[i] = y;
        } else {
          acc[i][j] = x;
          if (two) acc[i][j + 1] = y;
        }
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
      {
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
    if constexpr (kB3StepAcc) {  // the last pair's step sums
      constexpr int jl = 2 * (NP - 1);
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        acc[i][jl] += carx[i];
        if constexpr (jl + 1 < NF) acc[i][jl + 1] += cary[i];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };

  // The last step (tail): no operand loads, B stores or A split are left to issue (the main
  // steps fetch two steps ahead); for an addend epilogue it issues the addend loads in the load
  // slots instead: the addend of fragment column j is loaded beside the MFMAs of pair j / 2, so
  // its HBM traffic overlaps the matrix work instead of following it.  (A two-step tail that
  // also splits A of the last step spilled 16-22 VGPRs on the gathered-A kernels.)
  constexpr bool ADD = b3_ep_addend<EP>::value;
  float arow_v[ADD ? RF : 1][ADD ? NF : 1][4];
  float acol_v[ADD ? NF : 1];
  // the lane coordinates of the addend loads are recomputed behind an opaque copy of the thread
  // id: shared with the prologue's, they would stay live across the main loop (spills)
  int otid = 0;
  auto add_loads = [&](int j) {
    if constexpr (ADD) {
      const int ofr = otid & 15, ofg = (otid & 63) >> 4, ow = otid >> 6;
      const int col = n0 + j * 16 + ofr;
#pragma unroll
      for (int i = 0; i < RF; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          arow_v[i][j][r] = ep.add_row(m0 + (ow * RF + i) * 16 + ofg * 4 + r, col);
    }
  };
  auto tstep = [&](int cb, const b3_u4 (&afc)[RF][3], const ARaw* xa, b3_u4 (&afn)[RF][3],
                   int ksn, bool prefetch, bool last) {
    const b3_u4* Bs = b3_lds + cb * BU4;
    constexpr int RING = LDA + 2;
    b3_u4 bq[RING][3];
    auto rd = [&](int j) {
      const int o = (j * 16 + fr) * 4 + sw;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bq[j % RING][q] = Bs[q * BN * 4 + o];
    };
#pragma unroll
    for (int j = 0; j < LDA; ++j) rd(j);
    if constexpr (kB3ReadAheadFence) __builtin_amdgcn_sched_barrier(0);
    floatx4 carx[RF], cary[RF];  // kB3StepAcc: the previous pair's step sums
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
        // kB3StepAcc: the step's six products into a zero accumulator, then one fp32 add into
        // the running sum (the matrix core aligns every product of an MFMA to its largest
        // operand, accumulator included: the small pieces' products would be rounded at the
        // running sum's ulp, tools/diag/bf16_round_probe.hip).  The add of pair p is issued
        // behind pair p + 1's MFMAs (carry): only two pairs' temporaries are live.
        floatx4 x = kB3StepAcc ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i][j];
        floatx4 y = kB3StepAcc ? x : (two ? acc[i][j + 1] : x);
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
        if constexpr (kB3StepAcc) {
          if (p > 0) {
            acc[i][j - 2] += carx[i];
            acc[i][j - 1] += cary[i];  // the previous pair always has two columns
          }
          carx[i] = x;
          cary[i] = y;
        } else {
          acc[i][j] = x;
          if (two) acc[i][j + 1] = y;
        }
      }
      int nvm = 0;
      if (ADD && prefetch) {
        add_loads(j);
        if (two) add_loads(j + 1);
        nvm = (two ? 2 : 1) * 4 * RF;
      }
      if (xa && p == NP / 2) splitA(*xa, afn, ksn);
      constexpr int MQ = 4 * RF;
      b3_sgb<0x100>(nrd);
      if (two) b3_sgb<0x008>(MQ); else b3_sgb<0x008>(MQ / 2);
      b3_sgb<0x020>(nvm);
      if (two) b3_sgb<0x008>(2 * MQ); else b3_sgb<0x008>(MQ + MQ / 2);
    }
    if constexpr (kB3StepAcc) {  // the last pair's step sums
      constexpr int jl = 2 * (NP - 1);
#pragma unroll
      for (int i = 0; i < RF; ++i) {
        acc[i][jl] += carx[i];
        if constexpr (jl + 1 < NF) acc[i][jl + 1] += cary[i];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (last) __syncthreads();
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
    CGR_STAMP(1);
    epilogue_consts();  // after the prologue barrier: not waited for by it
    int cb = 0;  // LDS buffer of step ks (ks % 3)
    const int nmain = nk - 1;  // steps before the tail (the last step)
    for (int ks = 0; ks < nmain; ks += 2) {
      // even step: consume set 0 (A(ks+1), B(ks+2)), fill set 1 with A(ks+2), B(ks+3)
      step(cb, afr0, xb0, cb == 0 ? 2 : cb - 1, xa0, afr1, ks + 1, xa1, ks + 2, xb1, ks + 3);
      cb = cb == 2 ? 0 : cb + 1;
      if (ks + 1 >= nmain) break;
      // odd step: consume set 1 (A(ks+2), B(ks+3)), fill set 0 with A(ks+3), B(ks+4)
      step(cb, afr1, xb1, cb == 0 ? 2 : cb - 1, xa1, afr0, ks + 2, xa0, ks + 3, xb0, ks + 4);
      cb = cb == 2 ? 0 : cb + 1;
    }
    // tail: the last step uses fragment set nmain % 2 (split by the step before), moved into set
    // 0 so that the tail is one piece of code
    if (nmain & 1) {
#pragma unroll
      for (int i = 0; i < RF; ++i)
#pragma unroll
        for (int q = 0; q < 3; ++q) afr0[i][q] = afr1[i][q];
    }
    if constexpr (ADD) asm volatile("v_mov_b32 %0, %1" : "=v"(otid) : "v"(tid));
    tstep(cb, afr0, nullptr, afr1, 0, true, true);
  }

  CGR_STAMP(2);
  // ---- epilogue (the stage buffers are dead after the last barrier) ----
  ep.finish_ctx(cx);
  if constexpr (ADD) {  // the addend into the accumulators (the operation order of the apply)
#pragma unroll
    for (int j = 0; j < NF; ++j) acol_v[j] = ep.add_col(n0 + j * 16 + fr);  // L2-resident
#pragma unroll
    for (int i = 0; i < RF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[i][j][r] = ep.add_apply(acc[i][j][r], arow_v[i][j][r], acol_v[j], cx);
  }
  typename EP::Pre pv[EP_IT];
  if constexpr (!ADD) {
#pragma unroll
    for (int it = 0; it < EP_IT; ++it) {
      if constexpr (FLAT) {
        const int q = min(tid + NT * it, BM * C4 - 1);
        const int r = q / C4;
        pv[it] = ep.pre4(m0 + r, n0 + 4 * (q - r * C4));
      } else {
        pv[it] = ep.pre4(m0 + min(er0 + RPP * it, BM - 1), ecol);
      }
    }
  }
  float* C = reinterpret_cast<float*>(b3_lds);
  int* sd = reinterpret_cast<int*>(C + BM * S::LDC);  // SEG / TILE: dst of rows m0 - 1 .. m0 + BM
  // segment-start mask of the tile's rows: words 8..11 of the 16 scratch words after sd
  uint32_t* smask = reinterpret_cast<uint32_t*>(sd + BM + 2 + 8);
  if constexpr (SEG || TILE) {
    static_assert(BM == 64 || BM == 128, "segment mask: one or two 64-row words");
    if (tid < BM + 2) sd[tid] = sdv;
    if (tid < BM) {
      const uint64_t b = __ballot(sstart);
      if ((tid & 63) == 0) {
        smask[2 * (tid >> 6)] = (uint32_t)b;
        smask[2 * (tid >> 6) + 1] = (uint32_t)(b >> 32);
      }
      if constexpr (SEG && FLAT) {
        // the segment-start rows of this wave's 64 rows (below the tile's row count), in order,
        // into half tid / 64 of the start list (the halves' counts come from smask)
        const bool real = sstart && tid < M - m0;
        const uint64_t rb = __ballot(real);
        if (real) sd[BM + 2 + 16 + (tid & ~63) + __popcll(rb & ((1ull << (tid & 63)) - 1))] = tid;
      }
    }
    if (BM == 64 && tid == 0) smask[2] = smask[3] = 0xffffffffu;  // rows 64.. (none): starts
  }
#pragma unroll
  for (int i = 0; i < RF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[((w * RF + i) * 16 + fg * 4 + r) * S::LDC + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  CGR_STAMP(3);
  if constexpr (TILE) {
    ep.template tile<BM, BN, NT, S::LDC, EP_IT, FLAT ? 0 : RPP>(pv, C, sd, m0, n0, tile, tid);
  } else {
  // SEG && FLAT: the tile's segment starts, written before the barrier above in two halves
  // (rows 0..63 from slist[0], rows 64..127 from slist[64]); nh0 / nseg from the mask
  const int* slist = sd + BM + 2 + 16;
  const int nrow_t = min(BM, M - m0);
  uint64_t mlo = 0, mhi = 0;
  int nseg = 0, nh0 = 0;
  if constexpr (SEG && FLAT) {
    mlo = smask[0] | ((uint64_t)smask[1] << 32);
    mhi = smask[2] | ((uint64_t)smask[3] << 32);
    // starts among rows < nrow_t (rows past the tile's count are sentinel starts)
    const uint64_t klo = nrow_t >= 64 ? mlo : mlo & ((1ull << nrow_t) - 1);
    const uint64_t khi = nrow_t >= 128 ? mhi : (nrow_t > 64 ? mhi & ((1ull << (nrow_t - 64)) - 1) : 0);
    nh0 = __popcll(klo);
    nseg = nh0 + __popcll(khi);
  }
  auto seg_start = [&](int j) { return slist[j < nh0 ? j : 64 + (j - nh0)]; };
  // segment [r, e) x column group c4 of the tile: a[v] stored, or handed over (crossing)
  auto seg_out = [&](int r, int e, int c4, float4 a) {
    if constexpr (SEG) {
      const int col = n0 + 4 * c4;
      const int v = sd[r + 1];
      float* dst = ep.aout + (int64_t)v * ep.lda + col;
      const bool head = r == 0 && sd[0] == v, tail = e == nrow_t && sd[nrow_t + 1] == v;
      if (tail && !head && ep.znext)  // the tile where a crossing segment starts
        *reinterpret_cast<float4*>(ep.znext + (int64_t)v * ep.lda + col) = f4zero();
      if (head || tail) {
        const int b = ep.dst_ptr[v], ee = ep.dst_ptr[v + 1];
        if (seg_tiles(b, ee, BM) <= 2) {
          atomicAdd(dst, a.x);
          atomicAdd(dst + 1, a.y);
          atomicAdd(dst + 2, a.z);
          atomicAdd(dst + 3, a.w);
        } else {
          sc1_store4(ep.part + ((int64_t)tile * 2 + slot_of(tm, b / BM)) * BN + 4 * c4, a);
        }
      } else {
        st4_nt(dst, a);  // (common.hpp)
      }
    }
  };
  // SEG && FLAT && kB3SegMerge: ONE pass over (segment, column group) items -- each item applies
  // its segment's rows in row order (h stored) and sums them: no h write-back to LDS, no second
  // pass behind a barrier.  The lanes of a wave take consecutive column groups of one or two
  // segments, so they run the same row count but at segment boundaries.
  constexpr bool MERGE = SEG && FLAT && kB3SegMerge;
  auto apply_pass = [&](auto Ac) {
    constexpr int A = decltype(Ac)::value;
    if constexpr (MERGE) {
#pragma unroll
      for (int it = 0; it < EITF; ++it) {
        const int q = tid + NT * it;
        if (q >= nseg * C4) break;
        const int j = q / C4, c4 = q - j * C4, col = n0 + 4 * c4;
        if (col >= ep.N) continue;
        const int r = seg_start(j), e = seg_end(mlo, mhi, r);
        float4 a = f4zero();
        for (int k = r; k < e; ++k)
          a = f4add(a, ep.template apply4z_h<A>(
                           m0 + k, col, *reinterpret_cast<const float4*>(&C[k * S::LDC + 4 * c4]),
                           cx));
        seg_out(r, e, c4, a);
      }
    } else if constexpr (FLAT) {
#pragma unroll
      for (int it = 0; it < EP_IT; ++it) {
        const int q = tid + NT * it;
        if (q >= BM * C4) break;
        const int r = q / C4, c4 = q - r * C4, col = n0 + 4 * c4;
        float4* cp = reinterpret_cast<float4*>(&C[r * S::LDC + 4 * c4]);
        if constexpr (SEG)
          *cp = ep.template apply4z_h<A>(m0 + r, col, *cp, cx);  // keep h for the sums
        else
          ep.template apply4z<A>(m0 + r, col, *cp, cx);
      }
    } else {
#pragma unroll
      for (int it = 0; it < EIT; ++it) {
        const int r = er0 + RPP * it;
        if (eact && r < BM) {
          float4* cp = reinterpret_cast<float4*>(&C[r * S::LDC + 4 * ec4]);
          if constexpr (SEG && ADD)
            *cp = ep.template apply4z_h<A>(m0 + r, ecol, *cp, cx);  // keep h for the sums
          else if constexpr (SEG)
            *cp = ep.template apply4p_h<A>(m0 + r, ecol, *cp, pv[it], cx);
          else if constexpr (ADD)
            ep.template apply4z<A>(m0 + r, ecol, *cp, cx);
          else if constexpr (b3_ep_act<EP>::value)
            ep.template apply4p<A>(m0 + r, ecol, *cp, pv[it], cx);
          else
            ep.apply4p(m0 + r, ecol, *cp, pv[it], cx);
        }
      }
    }
  };
  if constexpr (b3_ep_act<EP>::value) {  // one loop per activation, chosen once
    if (ep.act == ACT_RELU) apply_pass(std::integral_constant<int, ACT_RELU>{});
    else if (ep.act == ACT_SILU) apply_pass(std::integral_constant<int, ACT_SILU>{});
    else apply_pass(std::integral_constant<int, -1>{});  // GELU and the rest
  } else {
    apply_pass(std::integral_constant<int, -1>{});
  }
  CGR_STAMP(4);
  if constexpr (SEG) {
    // a[v] = sum_{dst(i) = v} h[i] for the tile's columns (GNN.py:134): the thread owning the
    // first row of a segment in the tile sums its rows in row order (the segment bounds from the
    // tile's segment-start mask).  A segment inside the tile is stored; one crossing into one
    // neighbouring tile is added atomically to a[v], which edge_init_segsum_fwd zeroed (two
    // partials onto zero: p + q == q + p, deterministic); one over three or more row tiles (a hub
    // node, in-degree > BM + 1) leaves its partial in a slot fixed by the data and its last
    // contributor sums the slots in row-tile order -- deterministic for every in-degree.
    const int nrow = nrow_t;
    // segment [r, e) x column group c4 from the applied h rows in LDS
    auto seg_item = [&](int r, int e, int c4) {
      float4 a = f4zero();
      for (int k = r; k < e; ++k)
        a = f4add(a, *reinterpret_cast<const float4*>(&C[k * S::LDC + 4 * c4]));
      seg_out(r, e, c4, a);
    };
    if constexpr (MERGE) {
      // done by the apply pass
    } else if constexpr (FLAT) {
      __syncthreads();
      // items (segment j, column group c4) of the compact segment list: no lane waits on a
      // row that does not start a segment
#pragma unroll
      for (int it = 0; it < EITF; ++it) {
        const int q = tid + NT * it;
        if (q >= nseg * C4) break;
        const int j = q / C4, c4 = q - j * C4;
        if (n0 + 4 * c4 >= ep.N) continue;
        const int r = seg_start(j);
        seg_item(r, seg_end(mlo, mhi, r), c4);
      }
    } else {
      __syncthreads();
      mlo = smask[0] | ((uint64_t)smask[1] << 32);
      mhi = smask[2] | ((uint64_t)smask[3] << 32);
#pragma unroll
      for (int it = 0; it < EIT; ++it) {
        const int r = er0 + RPP * it;
        if (!eact || r >= nrow || ecol >= ep.N || !seg_bit(mlo, mhi, r)) continue;
        seg_item(r, seg_end(mlo, mhi, r), ec4);
      }
    }
    // hub segments: the last contributor sums the slots of every row tile in order
    const int vh = sd[0] == sd[1] ? sd[0] : -3;               // head segment's node, if any
    const int vt = sd[nrow] == sd[nrow + 1] ? sd[nrow] : -3;  // tail segment's node, if any
    auto hub = [&](int v) {
      return v >= 0 && seg_tiles(ep.dst_ptr[v], ep.dst_ptr[v + 1], BM) >= 3;
    };
    const bool bh = hub(vh), bt = vt != vh && hub(vt);  // uniform over the workgroup
    if (bh || bt) {
      int* scratch = sd + BM + 2;  // 16 words (B3NtShape::EPI_BYTES)
      ep_vm_drain();  // this wave's slot stores
      __syncthreads();
      if (tid == 0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int v = k == 0 ? (bh ? vh : -3) : (bt ? vt : -3);
          int done = 0;
          if (v >= 0) {
            const int cnt = seg_tiles(ep.dst_ptr[v], ep.dst_ptr[v + 1], BM);
            done = __hip_atomic_fetch_add(&ep.cnt[(int64_t)v * ep.tiles_n + tn], 1,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == cnt - 1;
          }
          scratch[14 + k] = done ? v : -1;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int v = scratch[14 + k];
        if (v < 0) continue;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // loads stay below the ticket
        const int t0 = ep.dst_ptr[v] / BM, t1 = (ep.dst_ptr[v + 1] - 1) / BM;
        for (int c4 = tid; c4 < C4; c4 += NT) {
          const int col = n0 + 4 * c4;
          if (col >= ep.N) continue;
          float4 a = f4zero();
          for (int t = t0; t <= t1; ++t)
            a = f4add(a, sc1_load4(ep.part + ((int64_t)(t * tiles_n + tn) * 2 + slot_of(t, t0)) *
                                                 BN + 4 * c4));
          *reinterpret_cast<float4*>(ep.aout + (int64_t)v * ep.lda + col) = a;
        }
        if (tid == 0) ep.cnt[(int64_t)v * ep.tiles_n + tn] = 0;
      }
    }
  }
  }  // !TILE
  CGR_STAMP_END((TILE ? 2 : 0) | (SEG ? 1 : 0) | (NF << 2) | (WAVES << 7));
}

template <int WAVES, int RF, int NF, bool NOMASK, class AL, class EP>
inline hipError_t launch_b3nt_t(const AL& al, const b3_u4* Bimg, int nimg, const EP& ep, int M,
                                int N, int K, int tiles_n, hipStream_t st) {
  using S = B3NtShape<WAVES, RF, NF>;
  auto kern = gemm_b3nt_kernel<WAVES, RF, NF, NOMASK, AL, EP>;
  static LdsLimit lim;
  // the dynamic bytes this launch asks for (a diagnostic build adds static LDS: stamps.hpp)
  const hipError_t e = lim.ensure(reinterpret_cast<const void*>(kern), (int)S::LDS_BYTES);
  if (e != hipSuccess) return e;
  const int tm = (M + S::BM - 1) / S::BM;
  int side = 0;
  if constexpr (b3_ep_side<EP>::value) {
    side = ep.side_on ? 1 : 0;
    // the caller checked b3nt_side_fits; a side workgroup needing more LDS than the tile is a bug
    if (side && ep.side_lds_bytes() > S::LDS_BYTES) return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(kern, dim3(tm * tiles_n + side), dim3(WAVES * 64), S::LDS_BYTES, st, al, Bimg,
                     nimg, ep, M, N, K, tiles_n);
  return hipGetLastError();
}

// workgroup rows: 8 waves (128 rows) when that still gives ~100+ workgroups (the node-row readout
// GEMMs at 120 x 8 waves beat 240 x 4 waves at one wave per SIMD: step A/B +0.8 %), else 4 (64 rows)
inline int b3nt_waves(int M, int N) {
  const int tiles_n = b3_cols(N).tiles;
  return ((M + 127) / 128) * tiles_n >= 96 ? 8 : 4;
}

// rows per workgroup tile of launch_b3nt for an M x N GEMM
inline int b3nt_rows(int M, int N) { return b3nt_waves(M, N) == 8 ? 128 : 64; }

// Column tiling of an M-row NT GEMM whose workgroups would leave CUs idle in b3_cols(N)'s tiling
// (the node-row readout GEMMs of a small batch: 60 row tiles x 2 at cfg2): more, narrower column
// tiles, chosen by a cost model of waves of workgroups x per-k-step cost, a step costing its
// MFMAs (nf fragment columns) plus fixed work worth kB3StepFixed columns (A fetch + split, B
// staging, the barrier: cfg2 layer GEMMs run 1.9 us per 13-column step against 1.3 us of MFMA).
// Every A row is then loaded and split once per column tile (more A traffic, all L2 hits).
// Images are packed in the tiling they are launched with (b3_job(..., cols)).
constexpr int kB3Cus = 256;
constexpr int kB3StepFixed = 6;
inline B3Cols b3nt_cols(int M, int N) {
  const B3Cols c0 = b3_cols(N);
  const int bm = b3nt_rows(M, N);
  const int tm = (M + bm - 1) / bm;
  const int nft = (N + 15) / 16;
  auto cost = [&](const B3Cols& c) {
    const int waves = (tm * c.tiles + kB3Cus - 1) / kB3Cus;
    return waves * (kB3StepFixed + c.nf);
  };
  B3Cols best = c0;
  int bc = cost(c0);
  for (int nf = c0.nf - 1; nf >= 2; --nf) {
    if (b3_nf_snap(nf) != nf) continue;
    const int tiles = (nft + nf - 1) / nf;
    const B3Cols c{tiles, nf, tiles * nf * 16};
    const int k = cost(c);
    if (k < bc) best = c, bc = k;
  }
  return best;
}

// whether launch_b3nt(.., c, .., M, N, ..) can host a side workgroup of lds bytes on a CU no tile
// takes (one NT workgroup per CU: kB3Cus - 1 tiles at most)
inline bool b3nt_side_fits(int M, int N, const B3Cols& c, size_t lds) {
  const int bm = b3nt_rows(M, N);
  return (int64_t)((M + bm - 1) / bm) * c.tiles < kB3Cus && lds <= b3nt_lds_bytes(bm, c.nf * 16);
}

// C = A B^T with B given as its image (b3_pack of the same N, K in the column tiling c).
// M, N, K > 0.
template <class AL, class EP>
inline hipError_t launch_b3nt(const AL& al, const b3_u4* Bimg, const B3Cols& c, const EP& ep,
                              int M, int N, int K, hipStream_t st) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (c.tiles * c.nf * 16 != c.nimg || c.nimg < N || b3_nf_snap(c.nf) != c.nf)
    return hipErrorInvalidValue;
  const bool w8 = b3nt_waves(M, N) == 8;
  // unmasked A when K % 4 == 0: every fetched float4 is either all-valid or past K (clamped to
  // finite in-bounds data, multiplied by the image's zero rows)
  auto go = [&](auto NFc) -> hipError_t {
    constexpr int NF = decltype(NFc)::value;
    if (K % 4 == 0)
      return w8 ? launch_b3nt_t<8, 1, NF, true>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st)
                : launch_b3nt_t<4, 1, NF, true>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st);
    return w8 ? launch_b3nt_t<8, 1, NF, false>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st)
              : launch_b3nt_t<4, 1, NF, false>(al, Bimg, c.nimg, ep, M, N, K, c.tiles, st);
  };
  switch (c.nf) {
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    case 4: return go(std::integral_constant<int, 4>{});
    case 6: return go(std::integral_constant<int, 6>{});
    case 7: return go(std::integral_constant<int, 7>{});
    case 8: return go(std::integral_constant<int, 8>{});
    case 11: return go(std::integral_constant<int, 11>{});
    case 13: return go(std::integral_constant<int, 13>{});
  }
  return hipErrorInvalidValue;
}
// ... in b3_cols(N)'s tiling
template <class AL, class EP>
inline hipError_t launch_b3nt(const AL& al, const b3_u4* Bimg, const EP& ep, int M, int N, int K,
                              hipStream_t st) {
  return launch_b3nt(al, Bimg, b3_cols(N), ep, M, N, K, st);
}

}  // namespace cgr

namespace cgr {

// ------------------------------------------------------------------------------------------
// TN (weight gradients): C[n, k] = sum_{e in split} A(e, n) B(e, k), fp32 partial slabs
// ------------------------------------------------------------------------------------------
// Two-piece split (x = hi + lo, hi = bf16(x), lo = bf16(x - hi)) and three terms per product
// (lo.hi, hi.lo, hi.hi; the dropped lo.lo and the residuals are <= 2^-16 |ab| per product, and a
// weight gradient sums ~10^4 of them with independent signs: fp32-level error against the fp64
// oracle, profiles/r02_split_precision_experiment.txt "b3t").  The kernel (gemm_b3tni_kernel,
// below) takes A pre-split as an e-image and stages B transposed into LDS in the NT image
// geometry ([piece][column row][4 swizzled 16-byte chunks of 8 e-rows]: every fragment read one
// conflict-free ds_read_b128; column c stored at row sigma(c), a rotation inside its 16-column
// block, so a b128 store pass hits four 64-byte bank groups).  Plans: one workgroup per (split of
// the e rows, k-tile of TNK fragments), all Nout columns (TNN n-fragments) per workgroup; splits
// start on 32-row boundaries.
struct B3TnPlan {
  int tiles_k, splits, rows_per_split, tnn;
};
inline B3TnPlan plan_b3tn(int Nout, int Kout, int R, int tnk, int target_wgs) {
  B3TnPlan p;
  p.tnn = (Nout + 15) / 16;
  p.tiles_k = (Kout + 16 * tnk - 1) / (16 * tnk);
  int splits = target_wgs / p.tiles_k;
  const int max_splits = (R + 63) / 64;  // >= 2 steps per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + 31) / 32 * 32;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

// storage row of column c: rotate by its 4-group inside the 16-column block
__device__ __forceinline__ int b3tn_sigma(int c) {
  return (c & ~3) | (((c & 3) + ((c >> 2) & 3)) & 3);
}

// Per operand kind: idx() turns a row into the element rows its loads read (the gather's index
// loads), base()/off() address load i of a job (i < NL; 32-bit element offsets, b3tn_fits checks
// the extents), get() the fp32 value of row j (float4 = the job's 4 columns).  Rows past R read
// row 0 and columns past the operand column 0 (in bounds; discarded or zero-weighted).
template <class L>
struct B3TnSrc;
template <>
struct B3TnSrc<LdPlain<4>> {
  static constexpr int NL = 8;
  static __device__ __forceinline__ void idx(const LdPlain<4>&, int row, int (&ix)[2]) {
    ix[0] = ix[1] = row;
  }
  static __device__ __forceinline__ const float* base(const LdPlain<4>& l, int, int) {
    return l.base;
  }
  static __device__ __forceinline__ uint32_t off(const LdPlain<4>& l, const int (&ix)[2], int,
                                                 int col, int K) {
    return (uint32_t)ix[0] * (uint32_t)l.ld + (uint32_t)(col < K ? col : 0);
  }
  static __device__ __forceinline__ float4 get(const float4 (&v)[16], int j) { return v[j]; }
  static bool fits(const LdPlain<4>& l, int R) { return (double)R * l.ld < 4.0e9; }
};
template <>
struct B3TnSrc<LdConcat<4>> {  // [x | s] (F % 4 == 0)
  static constexpr int NL = 8;
  static __device__ __forceinline__ void idx(const LdConcat<4>&, int row, int (&ix)[2]) {
    ix[0] = ix[1] = row;
  }
  static __device__ __forceinline__ const float* base(const LdConcat<4>& l, int, int col) {
    return col < l.F ? l.x : l.s;
  }
  static __device__ __forceinline__ uint32_t off(const LdConcat<4>& l, const int (&ix)[2], int,
                                                 int col, int K) {
    return col < l.F ? (uint32_t)ix[0] * (uint32_t)l.ldx + (uint32_t)col
                     : (uint32_t)ix[0] * (uint32_t)l.lds + (uint32_t)(col < K ? col - l.F : 0);
  }
  static __device__ __forceinline__ float4 get(const float4 (&v)[16], int j) { return v[j]; }
  static bool fits(const LdConcat<4>& l, int R) {
    return (double)R * l.ldx < 4.0e9 && (double)R * l.lds < 4.0e9;
  }
};
template <bool X>
struct B3TnSrc<LdGatherDiff<X>> {  // a[src] - h[rev]: loads 0..7 the a rows, 8..15 the h rows
  static constexpr int NL = 16;
  static __device__ __forceinline__ void idx(const LdGatherDiff<X>& l, int row, int (&ix)[2]) {
    ix[0] = l.src[row];
    ix[1] = X ? (row ^ 1) : l.rev[row];
  }
  static __device__ __forceinline__ const float* base(const LdGatherDiff<X>& l, int h, int) {
    return h ? l.h : l.a;
  }
  static __device__ __forceinline__ uint32_t off(const LdGatherDiff<X>& l, const int (&ix)[2],
                                                 int h, int col, int K) {
    return (uint32_t)ix[h] * (uint32_t)l.ld + (uint32_t)(col < K ? col : 0);
  }
  static __device__ __forceinline__ float4 get(const float4 (&v)[16], int j) {
    return f4sub(v[j], v[8 + j]);
  }
  static bool fits(const LdGatherDiff<X>& l, int R) { return (double)R * l.ld < 4.0e9; }
};

// k fragments per workgroup: 5 (H = 400: 25 -> 5 tiles exactly); 4 for more than 25 n-fragments
// (H = 512: 32 -> 8 tiles), whose accumulators would not fit beside TNK = 5 (40 B of scratch)
inline int b3tn_tnk(int Nout) { return (Nout + 15) / 16 > 25 ? 4 : 5; }
// workgroups of the layer weight gradient (A/B in the step: 128 -0.8 %, 256 -1.1 % vs 176; the
// side stream shares the GPU with the main chain, fewer splits = smaller slabs)
constexpr int kB3TnTarget = 176;
inline B3TnPlan b3tn_plan(int Nout, int Kout, int R, int target = kB3TnTarget) {
  return plan_b3tn(Nout, Kout, R, b3tn_tnk(Nout), target);
}
// ------------------------------------------------------------------------------------------
// TN with the n-side operand as a pre-split e-image (weight gradients dW = A^T B whose A is
// shared by every k-tile: dpre, dzn, Gs)
// ------------------------------------------------------------------------------------------
// e-image of X [R rows, C cols] (R = the TN's reduction dimension): per 32-row step s and piece p
// (0 = hi = bf16(x), 1 = lo = bf16(x - hi)) a plane of `cimg` columns x 64 bytes, column c
// holding the pieces of rows 32 s .. 32 s + 31 in order; rows >= R and columns >= C are zero.
// Written once per matrix by b3_eimage (b3_pack.hip).  An MFMA A fragment (16 columns x 32 rows)
// is then one coalesced 1 KB global load per piece: lane (fr, fg) takes column fr, rows
// 8 fg .. 8 fg + 7 -- no transposition and no split inside the GEMM (the round-2 kernel re-staged
// and re-split the whole A operand in each of its tiles_k workgroups, 5 at H = 400: 83 % of its
// staging VALU, PMC 7.6 VALU per MFMA).
struct B3EImg {
  const b3_u4* img;  // 16-byte units: ((s * 2 + p) * cimg + c) * 4 + chunk
  int cimg;          // columns, a multiple of 16
};
inline int b3_eimg_cols(int C) { return (C + 15) / 16 * 16; }
inline size_t b3_eimg_bytes(int64_t R, int C) {
  return (size_t)((R + 31) / 32) * 2 * (size_t)b3_eimg_cols(C) * 64;
}
hipError_t b3_eimage(const float* x, int64_t ld, int64_t R, int C, b3_u4* img, hipStream_t st);
// e-image of G = segsum(X) over the CSR (idx, ptr) of R segments, G never stored (b3_pack.hip);
// X rows 16-byte aligned with ld >= round_up(C, 4)
hipError_t b3_segsum_eimage(const float* x, int64_t ld, const int* idx, const int* ptr, int64_t R,
                            int C, b3_u4* img, hipStream_t st);

// Workgroup = CW = 8 compute waves + SW staging waves (warp-specialised: a wave runs one role for
// the whole kernel, so the registers of the two roles are not live together).
//   * compute wave w: n-fragments w, w + CW, ... (RN of them, all TNK k-fragments each) plus RX
//     of the remaining (TNN % CW) x TNK products, dealt round-robin; its A fragments come straight
//     from the e-image, one step ahead of the MFMAs (two register sets, loop unrolled by 2).
//   * staging waves: the k-side operand B (TNK x 16 columns of the tile), split into hi / lo and
//     transposed into LDS in the NT image geometry (chunk c of a column = rows 8 c .. 8 c + 7 of
//     the step, the e-image's order); a job is 4 columns x 4 rows (one 8-byte half of a chunk
//     per column and piece), so the split's VALU is spread over SW = 3 waves on three SIMDs
//     (8-row jobs on 1.25 waves: lab 40 us);  its loads are issued two intervals before they are
//     staged (two register sets) and the gather's index loads one more interval ahead.
//   * one barrier per step: compute reads LDS buffer t & 1 while staging fills (t + 1) & 1.
//   * splits start on 32-row boundaries, so a split's last step reads only its own rows or the
//     image's zero rows: A is never masked; B rows past R read row 0 (finite, times zero A).
//   * bias (column sums of A) from the pieces, hi + lo per element: n-fragment f is summed by
//     the k-tile min(f / TNK, tiles_k - 1), inside the compute wave that loads f (the remainder
//     fragments by the wave holding their k-fragment-0 product).
template <int TNN, int TNK>
struct B3TniShape {
  static constexpr int CW = 8;
  static constexpr int BC = TNK * 16;
  static constexpr int JC = BC / 4;  // 4-column groups
  static constexpr int JB = JC * 8;  // staging jobs: 4 columns x 4 rows (half an 8-row chunk)
  static constexpr int SW = (JB + 63) / 64;
  static constexpr int NT = (CW + SW) * 64;
  static constexpr int RN = TNN / CW;
  static constexpr int REM = (TNN % CW) * TNK;
  static constexpr int RX = (REM + CW - 1) / CW;
  static constexpr int NA = RN + RX;        // A fragments a compute wave loads per step
  static constexpr int SU4 = 2 * BC * 4;    // b3_u4 per LDS stage buffer
  static constexpr size_t LDS_BYTES = (size_t)2 * SU4 * 16;
};

// prev (slab == null: none): the previous weight gradient's split-K slabs, reduced by this
// launch's threads before their own work (the launch-boundary reduce: no reduce launch, and the
// slab read overlaps other workgroups' main loops; prev's slabs are not this launch's)
template <int TNN, int TNK, class BL>
__global__ __launch_bounds__((B3TniShape<TNN, TNK>::NT)) void gemm_b3tni_kernel(
    B3EImg ai, BL bl, float* __restrict__ slab, float* __restrict__ bslab, int Nout, int Kout,
    int R, int rows_per_split, int tiles_k, int want_bias, RedJob prev) {
  typedef B3TnSrc<BL> TB;
  using S = B3TniShape<TNN, TNK>;
  constexpr int CW = S::CW, RN = S::RN, RX = S::RX, NA = S::NA, BC = S::BC, SU4 = S::SU4;
  constexpr int JB = S::JB;
  extern __shared__ b3_u4 b3_lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  CGR_STAMP_BEGIN();
#ifdef CGR_STAMPS
  // diagnostic: per step, the cycles a wave works and the cycles it waits at the step barrier, for
  // compute wave 0 (slots 1, 2) and staging wave 0 (slots 3, 4); slot 5 = main loop end
  unsigned long long st_work = 0, st_wait = 0, st_prev = 0, st_t = 0;
  const bool st_me = tid == 0 || tid == CW * 64;
#define TN_STAMP_PRE() do { if (st_me) { st_t = ::cgr::stamp_now(); st_work += st_t - st_prev; } } while (0)
#define TN_STAMP_POST() do { if (st_me) { st_prev = ::cgr::stamp_now(); st_wait += st_prev - st_t; } } while (0)
#define TN_STAMP_START() do { if (st_me) st_prev = ::cgr::stamp_now(); } while (0)
#else
#define TN_STAMP_PRE() ((void)0)
#define TN_STAMP_POST() ((void)0)
#define TN_STAMP_START() ((void)0)
#endif
  if (prev.slab) {
    const int64_t tot = reduce_items(prev);
    for (int64_t f = (int64_t)blockIdx.x * S::NT + tid; f < tot; f += (int64_t)gridDim.x * S::NT)
      reduce_slab_item(prev, f);
  }
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / tiles_k, tkk = lin - split * tiles_k;
  const int k0 = tkk * TNK * 16;
  const int e_begin = split * rows_per_split;  // a multiple of 32
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + 31) / 32 : 0;

  // staging waves win the SIMD's issue arbitration against the compute wave they share it with
  // (static priority, no per-step flips: cdna_hip_programming.md T5; step A/B +0.5 %,
  // profiles/r03_fold_ab_cfg2.txt)
  if (w >= CW) __builtin_amdgcn_s_setprio(1);
  if (w >= CW) {
    // ================= staging waves: B of step t + 1 into LDS buffer (t + 1) & 1 =============
    // job (4-column group cg, 4-row group hc): rows 4 hc .. 4 hc + 3 of a step, half of the
    // 16-byte chunk hc / 2 of each column (the e-image's row order); lanes run column groups
    // fastest, so a load instruction covers ~3 rows x 320 contiguous bytes
    constexpr int JC = S::JC;
    const int q = tid - CW * 64;
    const bool act = q < JB;
    const int hc = act ? q / JC : 0;
    const int jcol = (act ? q - hc * JC : 0) * 4;  // first of the job's 4 columns in the tile
    const int gcol = k0 + jcol;
    const float* base0 = TB::base(bl, 0, gcol);
    const float* base1 = TB::base(bl, 1, gcol);
    // two register sets: rows j < 4 of a / plain rows in r[j], gathered h rows in r[8 + j]
    float4 raw0[16], raw1[16];
    uint32_t off[TB::NL];
    int ix[4][2];
    auto rowof = [&](int t, int j) {
      const int e = e_begin + t * 32 + 4 * hc + j;
      return e < R ? e : 0;
    };
    auto index = [&](int t) {  // the gather's index loads of step t
#pragma unroll
      for (int j = 0; j < 4; ++j) TB::idx(bl, rowof(t, j), ix[j]);
    };
    auto fetch = [&](float4 (&raw)[16]) {  // addresses from the last index(), then the loads
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < TB::NL / 8; ++h) off[8 * h + j] = TB::off(bl, ix[j], h, gcol, Kout);
#pragma unroll
      for (int i = 0; i < 4; ++i) raw[i] = *reinterpret_cast<const float4*>(base0 + off[i]);
      if constexpr (TB::NL == 16) {
#pragma unroll
        for (int i = 8; i < 12; ++i) raw[i] = *reinterpret_cast<const float4*>(base1 + off[i]);
      }
    };
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    auto put = [&](b3_u4* img, int t, float f0, float f1, float f2, float f3) {
      float a0, a1, a2, a3, c0, c1, c2, c3;
      const uint32_t h01 = b3_cvt2(f0, f1, a0, a1), h23 = b3_cvt2(f2, f3, a2, a3);
      const uint32_t l01 = b3_cvt2(f0 - a0, f1 - a1, c0, c1), l23 = b3_cvt2(f2 - a2, f3 - a3, c2, c3);
      const int row = b3tn_sigma(jcol + t);
      const int slot = (hc >> 1) ^ lds_swz(row);
      char* b = reinterpret_cast<char*>(img) + 8 * (hc & 1);
      *reinterpret_cast<u2v*>(b + (row * 4 + slot) * 16) = u2v{h01, h23};
      *reinterpret_cast<u2v*>(b + ((BC + row) * 4 + slot) * 16) = u2v{l01, l23};
    };
    auto stage = [&](const float4 (&raw)[16], int buf) {
      b3_u4* img = b3_lds + buf * SU4;
      float4 u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = TB::get(raw, j);
      if (act) {
        put(img, 0, u[0].x, u[1].x, u[2].x, u[3].x);
        put(img, 1, u[0].y, u[1].y, u[2].y, u[3].y);
        put(img, 2, u[0].z, u[1].z, u[2].z, u[3].z);
        put(img, 3, u[0].w, u[1].w, u[2].w, u[3].w);
      }
    };
    if (nt > 0) {
      index(0);
      fetch(raw0);  // step 0
      index(1);
      fetch(raw1);  // step 1
      index(2);
      stage(raw0, 0);
      fetch(raw0);  // step 2
      index(3);
      __syncthreads();
      TN_STAMP_START();
      // interval t (compute on step t): stage step t + 1, whose loads were issued two intervals
      // ago, then issue step t + 3's into the freed set (index loads one interval ahead of them)
      for (int t = 0; t < nt; t += 2) {
        if (t + 1 < nt) stage(raw1, 1);
        fetch(raw1);  // step t + 3
        index(t + 4);
        TN_STAMP_PRE();
        __syncthreads();
        TN_STAMP_POST();
        if (t + 1 >= nt) break;
        if (t + 2 < nt) stage(raw0, 0);
        fetch(raw0);  // step t + 4
        index(t + 5);
        TN_STAMP_PRE();
        __syncthreads();
        TN_STAMP_POST();
      }
    }
#ifdef CGR_STAMPS
    if (tid == CW * 64) {
      ::cgr::stamp_val(3, st_work);
      ::cgr::stamp_val(4, st_wait);
    }
#endif
    CGR_STAMP_END(0x4000 | TNN);
    return;
  }

  // ================= compute waves =================
  const int rrow = b3tn_sigma(fr);  // fragment reads: storage row of column fr of a block
  const int sw = fg ^ lds_swz(rrow);
  // this wave's A fragments: f < RN: n-fragment w + f CW; f >= RN: remainder product xq(f - RN)
  auto xq = [&](int x) {
    const int qq = w + x * CW;
    return qq < S::REM ? qq : 0;
  };
  auto frag_n = [&](int f) { return f < RN ? w + f * CW : RN * CW + xq(f - RN) / TNK; };
  // bias ownership (k-tile of n-fragment f) and, for remainder products, k-fragment 0 only
  bool own[NA];
#pragma unroll
  for (int f = 0; f < NA; ++f) {
    const int n = frag_n(f);
    const int tile = min(n / TNK, tiles_k - 1);
    own[f] = want_bias && tile == tkk && n < TNN &&
             (f < RN || (w + (f - RN) * CW < S::REM && xq(f - RN) % TNK == 0));
  }
  float bsum[NA];
#pragma unroll
  for (int f = 0; f < NA; ++f) bsum[f] = 0.f;
  const int s0 = e_begin / 32;
  auto aload = [&](int t, b3_u4 (&a)[NA][2]) {
    const int s = s0 + (t < nt ? t : nt - 1);
    const b3_u4* base = ai.img + (size_t)s * 2 * ai.cimg * 4;
#pragma unroll
    for (int f = 0; f < NA; ++f) {
      const int c = min(frag_n(f) * 16 + fr, ai.cimg - 1);  // fragments past the image: discarded
      a[f][0] = base[c * 4 + fg];
      a[f][1] = base[(ai.cimg + c) * 4 + fg];
    }
  };
  floatx4 acc[RN > 0 ? RN : 1][TNK], accx[RX > 0 ? RX : 1];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < TNK; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int x = 0; x < RX; ++x) accx[x] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf, const b3_u4 (&a)[NA][2]) {
    const b3_u4* img = b3_lds + buf * SU4;
#pragma unroll
    for (int x = 0; x < RX; ++x) {
      const int rb = (xq(x) % TNK) * 16 + rrow;
      const b3_u4 xbh = img[rb * 4 + sw], xbl = img[(BC + rb) * 4 + sw];
      floatx4 c = accx[x];
      c = b3_mfma(a[RN + x][1], xbh, c);
      c = b3_mfma(a[RN + x][0], xbl, c);
      accx[x] = b3_mfma(a[RN + x][0], xbh, c);
    }
#pragma unroll
    for (int j = 0; j < TNK; ++j) {
      if constexpr (RN > 0) {
        const int row = j * 16 + rrow;
        const b3_u4 bh = img[row * 4 + sw], bl_ = img[(BC + row) * 4 + sw];
#pragma unroll
        for (int i = 0; i < RN; ++i) {
          floatx4 c = acc[i][j];
          c = b3_mfma(a[i][1], bh, c);
          c = b3_mfma(a[i][0], bl_, c);
          acc[i][j] = b3_mfma(a[i][0], bh, c);
        }
      }
    }
#pragma unroll
    for (int f = 0; f < NA; ++f)
      if (own[f]) {  // sum of hi + lo over the lane's 8 rows
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t h = a[f][0][k], l = a[f][1][k];
          s += (__uint_as_float(h << 16) + __uint_as_float(l << 16)) +
               (__uint_as_float(h & 0xffff0000u) + __uint_as_float(l & 0xffff0000u));
        }
        bsum[f] += s;
      }
  };
  if (nt > 0) {
    b3_u4 a0[NA][2], a1[NA][2];
    aload(0, a0);
    __syncthreads();  // B(0) staged
    TN_STAMP_START();
    for (int t = 0; t < nt; t += 2) {
      aload(t + 1, a1);
      __builtin_amdgcn_sched_barrier(0);
      compute(0, a0);
      TN_STAMP_PRE();
      __syncthreads();
      TN_STAMP_POST();
      if (t + 1 >= nt) break;
      aload(t + 2, a0);
      __builtin_amdgcn_sched_barrier(0);
      compute(1, a1);
      TN_STAMP_PRE();
      __syncthreads();
      TN_STAMP_POST();
    }
  }
#ifdef CGR_STAMPS
  if (tid == 0) {
    ::cgr::stamp_val(1, st_work);
    ::cgr::stamp_val(2, st_wait);
    ::cgr::stamp_val(5, ::cgr::stamp_now());
  }
#endif

  // ---- epilogue: accumulators straight to the slab (rows n = 16 nf + 4 fg + r, columns
  // k0 + 16 j + fr: 64 contiguous bytes per row and register) ----
  const int ldk = (Kout + 3) & ~3;
  float* out = slab + (int64_t)split * Nout * ldk;
  auto store = [&](int nf, int kf, const floatx4& c) {
    const int col = k0 + kf * 16 + fr;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = nf * 16 + fg * 4 + r;
      if (row < Nout && col < Kout) out[(int64_t)row * ldk + col] = c[r];
    }
  };
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < TNK; ++j) store(w + i * CW, j, acc[i][j]);
#pragma unroll
  for (int x = 0; x < RX; ++x) {
    const int qq = w + x * CW;
    if (qq < S::REM) store(RN * CW + qq / TNK, qq % TNK, accx[x]);
  }
  if (want_bias) {
#pragma unroll
    for (int f = 0; f < NA; ++f) {
      float v = bsum[f];
      v += __shfl_xor(v, 16, 64);  // (g0 + g1), (g2 + g3)
      v += __shfl_xor(v, 32, 64);  // (g0 + g1) + (g2 + g3), the same in every group
      const int n = frag_n(f) * 16 + fr;
      if (own[f] && fg == 0 && n < Nout) bslab[(int64_t)split * Nout + n] = v;
    }
  }
  CGR_STAMP_END(0x4000 | TNN);
}
#undef TN_STAMP_PRE
#undef TN_STAMP_POST
#undef TN_STAMP_START

// splits of the e-image TN: rows_per_split a multiple of 32 (plan_b3tn rounds it)
template <int TNN, int TNK, class BL>
inline hipError_t launch_b3tni_t(const B3EImg& ai, const BL& bl, const B3TnPlan& p, float* slab,
                                 float* bslab, int Nout, int Kout, int R, bool want_bias,
                                 hipStream_t st, const RedJob& prev) {
  using S = B3TniShape<TNN, TNK>;
  auto kern = gemm_b3tni_kernel<TNN, TNK, BL>;
  static LdsLimit lim;
  const hipError_t e = lim.ensure(reinterpret_cast<const void*>(kern), (int)S::LDS_BYTES);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3(p.tiles_k * p.splits), dim3(S::NT), S::LDS_BYTES, st, ai, bl,
                     slab, bslab, Nout, Kout, R, p.rows_per_split, p.tiles_k, want_bias ? 1 : 0,
                     prev);
  return hipGetLastError();
}

// the e-image TN covers Nout up to 32 fragments (H <= 512) and B operands whose extents fit the
// 32-bit element offsets; A = the e-image of an [R, >= Nout] matrix
template <class BL>
inline bool b3tni_ok(const BL& bl, int Nout, int R) {
  const int t = (Nout + 15) / 16;
  return t >= 1 && t <= 32 && B3TnSrc<BL>::fits(bl, R);
}

template <class BL>
inline hipError_t launch_b3tni(const B3EImg& ai, const BL& bl, const B3TnPlan& p, float* slab,
                               float* bslab, int Nout, int Kout, int R, bool want_bias,
                               hipStream_t st, const RedJob& prev = RedJob{}) {
  constexpr int TNK = 5;
  if (!b3tni_ok(bl, Nout, R) || p.rows_per_split % 32) return hipErrorInvalidValue;
  if (p.tiles_k != (Kout + 16 * b3tn_tnk(Nout) - 1) / (16 * b3tn_tnk(Nout)))
    return hipErrorInvalidValue;  // a plan from b3tn_plan
  switch (p.tnn) {
    case 25: return launch_b3tni_t<25, TNK>(ai, bl, p, slab, bslab, Nout, Kout, R, want_bias, st, prev);
    case 32: return launch_b3tni_t<32, 4>(ai, bl, p, slab, bslab, Nout, Kout, R, want_bias, st, prev);
    default: break;
  }
  // other widths: the smallest instantiated fragment count that covers Nout (extra fragments
  // read the image's zero columns and are not stored)
  const int t = p.tnn;
  B3TnPlan q = p;
  if (t <= 2) { q.tnn = 2; return launch_b3tni_t<2, TNK>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev); }
  if (t <= 4) { q.tnn = 4; return launch_b3tni_t<4, TNK>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev); }
  if (t <= 8) { q.tnn = 8; return launch_b3tni_t<8, TNK>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev); }
  if (t <= 16) { q.tnn = 16; return launch_b3tni_t<16, TNK>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev); }
  if (t <= 25) { q.tnn = 25; return launch_b3tni_t<25, TNK>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev); }
  q.tnn = 32;
  return launch_b3tni_t<32, 4>(ai, bl, q, slab, bslab, Nout, Kout, R, want_bias, st, prev);
}

}  // namespace cgr
