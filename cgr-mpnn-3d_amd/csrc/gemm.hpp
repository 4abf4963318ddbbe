// fp32 MFMA GEMM templates for the D-MPNN path (gfx950, v_mfma_f32_16x16x4_f32).
//
// Two shapes cover every GEMM of the forward and backward (SURVEY.md §2a K3,K7,K10 and their
// backward):
//
//   gemm_nt:  C[m, n] = sum_k A(m, k) * B(n, k)      A rows produced by a *loader* (plain rows,
//             gathered a[src]-h[rev] rows, or the [x | s] concat), B = rows of a weight matrix
//             ([out, in] = nn.Linear layout); an *epilogue* functor consumes C as float4 row
//             pieces (bias / skip / activation / dropout / stores).
//   gemm_tn:  C[n, k] = sum_e A(e, n) * B(e, k)      weight gradients dW = dZ^T Q, reduction over
//             the (long) edge / node dimension, split into row ranges with fp32 partial slabs
//             (deterministic: reduce_slabs sums them in a fixed order).  Workgroups of k-tile 0
//             also emit the column sums of A (= the bias gradient) per split.
//
// Tiling (one workgroup = WAVES waves of 64 lanes; RM row / RN column 16x16 fragments per wave):
//   NT: BM = 16*WAVES*RM, BN = 16*RN (H = 400 -> RN = 5 tiles the hidden dim exactly), BK = 16*KT.
//       LDS tile = [k16][row][4 x float4], chunk c of row r stored at slot c ^ swz(r): every
//       ds_read_b128 fragment read is bank-conflict free (PMC SQ_LDS_BANK_CONFLICT = 0).  The
//       MFMA's 4-deep k is mapped so lane group g = lane>>4 owns k = 4g..4g+3 of a 16-deep slice:
//       one b128 read feeds four MFMAs.
//   TN: e-major LDS tiles ([BE][BM + pad], stride == 16 mod 32 floats) read with conflict-free
//       ds_read_b32; global loads stay coalesced float4 along n / k.
//   Loads are software-pipelined one k-tile ahead through registers.  Loaders are BRANCH-FREE:
//   fetch() issues every global load unconditionally from a clamped, in-bounds address and
//   combine() applies masks / the a[src]-h[rev] subtraction when the tile is written to LDS, so
//   the compiler's s_waitcnt vmcnt lands after the MFMAs instead of in front of them (with
//   guarded loads hipcc branched around each load and waited vmcnt(0) per load, serialising the
//   prefetch: cdna_hip_programming.md §5 trap (c)).  Row state that needs an index load (gathered
//   rows) is computed one tile earlier still.
//   Epilogue: accumulators -> LDS [BM][BN+4] -> coalesced float4 rows -> ep.apply4 / slab store.
//   Grid: 1-D (+ split index for TN), bijective XCD remap so the tiles of one row panel share an
//   XCD's L2.
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

// unconditional VEC-wide loads of elements [k, k+4) of a row; sub-chunks starting at >= K read
// element 0 instead (always in bounds) and are zeroed later by mask4
template <int VEC>
__device__ __forceinline__ float4 fetch4(const float* __restrict__ p, int k, int K) {
  if constexpr (VEC == 4) {
    return *reinterpret_cast<const float4*>(p + (k < K ? k : 0));
  } else if constexpr (VEC == 2) {
    const float2 u = *reinterpret_cast<const float2*>(p + (k < K ? k : 0));
    const float2 w = *reinterpret_cast<const float2*>(p + (k + 2 < K ? k + 2 : 0));
    return make_float4(u.x, u.y, w.x, w.y);
  } else {
    return make_float4(p[k < K ? k : 0], p[k + 1 < K ? k + 1 : 0], p[k + 2 < K ? k + 2 : 0],
                       p[k + 3 < K ? k + 3 : 0]);
  }
}

__device__ __forceinline__ float4 mask4(float4 v, bool ok, int k, int K) {
  v.x = (ok && k < K) ? v.x : 0.f;
  v.y = (ok && k + 1 < K) ? v.y : 0.f;
  v.z = (ok && k + 2 < K) ? v.z : 0.f;
  v.w = (ok && k + 3 < K) ? v.w : 0.f;
  return v;
}

// ------------------------------------------------------------------------------------------
// Row loaders.  Row row(int r, int limit): per-row state (rows >= limit read row 0, masked);
// Raw fetch(const Row&, int k, int K): the global loads of elements k..k+3;
// float4 combine(const Raw&, const Row&, int k, int K): masks / arithmetic (0 beyond K).
// ------------------------------------------------------------------------------------------
template <int VEC>
struct LdPlain {
  const float* base;
  int64_t ld;
  struct Row {
    const float* p;
    bool ok;
  };
  typedef float4 Raw;
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    return Row{base + (int64_t)(ok ? r : 0) * ld, ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    return fetch4<VEC>(rw.p, k, K);
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(v, rw.ok, k, K);
  }
  // no masks (K % 4 == 0, finite data: rows past the end and k >= K read finite in-bounds
  // elements whose products meet zero weights or are discarded by the epilogue)
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const { return v; }
  typedef float Raw1;  // single element k (column-blocked staging of the split-bf16 TN kernel)
  __device__ __forceinline__ Raw1 fetch1(const Row& rw, int k, int K) const {
    return rw.p[k < K ? k : 0];
  }
  __device__ __forceinline__ float combine1(Raw1 v, const Row& rw, int k, int K) const {
    return (rw.ok && k < K) ? v : 0.f;
  }
};

// rows gathered through an index: A(r, :) = base[idx[r], :]  (internal buffers, ld % 4 == 0).
// The layer backward's dm GEMM reads dpre[rev(r)] so that its output row r is dm[rev(r)]: rows
// grouped by dst(r), the segments its fused epilogue sums (ep_bwd.hpp).
struct LdGatherRows {
  const float* base;
  const int* idx;
  int64_t ld;
  struct Row {
    int i;
    bool ok;
  };
  typedef float4 Raw;
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    return Row{idx[ok ? r : 0], ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    return *reinterpret_cast<const float4*>(base + (int64_t)rw.i * ld + (k < K ? k : 0));
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(v, rw.ok, k, K);
  }
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const { return v; }
};

// the activation-derivative factor of the readout backward's dzn (GNN.py:134-136 reversed):
// A(v, k) = act'(m[v, k]) with m = hn (ReLU: hn > 0) or zn (internal [M, ld] buffers, ld % 4 == 0).
// dzn = dy[graph(v)] wf[k] act'(zn[v, k]) factors into this, a per-k scale folded into the weight
// image (B3PackJob::kscale) and a per-row scale applied by the epilogue (EpStoreRowScale).
template <int ACT = -1>  // ACT >= 0: the activation as a compile-time constant (main-loop code)
struct LdActGradT {
  const float* m;
  int64_t ld;
  int act;
  struct Row {
    const float* p;
    bool ok;
  };
using LdActGrad = LdActGradT<-1>;
  typedef float4 Raw;
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    return Row{m + (int64_t)(ok ? r : 0) * ld, ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    return *reinterpret_cast<const float4*>(rw.p + (k < K ? k : 0));
  }
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const {
    const int ac = ACT < 0 ? act : ACT;
    return make_float4(act_grad(v.x, ac), act_grad(v.y, ac), act_grad(v.z, ac),
                       act_grad(v.w, ac));
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(combine_nm(v), rw.ok, k, K);
  }
};

// B rows of two stacked weight matrices: rows [0, n0) from base0 (ld0), rows [n0, ...) from base1
// (ld1).  Used for the merged x-GEMM  x @ [W0[:, :F]; W_n[:, :F]]^T.  VEC divides ld0, ld1, K.
template <int VEC>
struct LdTwoRows {
  const float* base0;
  int64_t ld0;
  const float* base1;
  int64_t ld1;
  int n0;
  struct Row {
    const float* p;
    bool ok;
  };
  typedef float4 Raw;
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    const int rr = ok ? r : 0;
    return Row{rr < n0 ? base0 + (int64_t)rr * ld0 : base1 + (int64_t)(rr - n0) * ld1, ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    return fetch4<VEC>(rw.p, k, K);
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(v, rw.ok, k, K);
  }
  // no masks (K % 4 == 0, finite data: rows past the end and k >= K read finite in-bounds
  // elements whose products meet zero weights or are discarded by the epilogue)
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const { return v; }
  typedef float Raw1;  // single element k (column-blocked staging of the split-bf16 TN kernel)
  __device__ __forceinline__ Raw1 fetch1(const Row& rw, int k, int K) const {
    return rw.p[k < K ? k : 0];
  }
  __device__ __forceinline__ float combine1(Raw1 v, const Row& rw, int k, int K) const {
    return (rw.ok && k < K) ? v : 0.f;
  }
};

// m[e, :] = a[src[e], :] - h[rev[e], :]   (GNN.py:136-141).  Internal buffers, ld = Hp (% 4 == 0).
// REV_XOR: rev[e] = e ^ 1 (caller's original edge order, no index array).  Row keeps the raw
// indices; addresses are formed in fetch() so the index loads are waited for only there.
template <bool REV_XOR>
struct LdGatherDiff {
  const float* a;
  const float* h;
  const int* src;
  const int* rev;
  int64_t ld;
  struct Row {
    int s, r;
    bool ok;
  };
  struct Raw {
    float4 a, h;
  };
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    const int rr = ok ? r : 0;
    return Row{src[rr], REV_XOR ? (rr ^ 1) : rev[rr], ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    const int kk = k < K ? k : 0;
    return Raw{*reinterpret_cast<const float4*>(a + (int64_t)rw.s * ld + kk),
               *reinterpret_cast<const float4*>(h + (int64_t)rw.r * ld + kk)};
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(f4sub(v.a, v.h), rw.ok, k, K);
  }
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const { return f4sub(v.a, v.h); }
  struct Raw1 {
    float a, h;
  };
  __device__ __forceinline__ Raw1 fetch1(const Row& rw, int k, int K) const {
    const int kk = k < K ? k : 0;
    return Raw1{a[(int64_t)rw.s * ld + kk], h[(int64_t)rw.r * ld + kk]};
  }
  __device__ __forceinline__ float combine1(const Raw1& v, const Row& rw, int k, int K) const {
    return (rw.ok && k < K) ? v.a - v.h : 0.f;
  }
};

// q[v, :] = [x[v, :F] | s[v, :H]]  (GNN.py:106).  VEC divides F and ldx (so no VEC sub-chunk
// straddles F); s rows are internal (16-byte aligned, ld % 4 == 0).
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
    bool ok;
  };
  typedef float4 Raw;
  __device__ __forceinline__ Row row(int r, int limit) const {
    const bool ok = r < limit;
    const int rr = ok ? r : 0;
    return Row{x + (int64_t)rr * ldx, s + (int64_t)rr * lds, ok};
  }
  __device__ __forceinline__ Raw fetch(const Row& rw, int k, int K) const {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; j += VEC) {
      const int kk = k + j;
      const float* p = kk < F ? rw.px + kk : (kk < K ? rw.ps + (kk - F) : rw.px);
      if constexpr (VEC == 4) {
        const float4 u = *reinterpret_cast<const float4*>(p);
        v[0] = u.x;
        v[1] = u.y;
        v[2] = u.z;
        v[3] = u.w;
      } else if constexpr (VEC == 2) {
        const float2 u = *reinterpret_cast<const float2*>(p);
        v[j] = u.x;
        v[j + 1] = u.y;
      } else {
        v[j] = *p;
      }
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ float4 combine(const Raw& v, const Row& rw, int k, int K) const {
    return mask4(v, rw.ok, k, K);
  }
  // no masks (K % 4 == 0, finite data: rows past the end and k >= K read finite in-bounds
  // elements whose products meet zero weights or are discarded by the epilogue)
  __device__ __forceinline__ float4 combine_nm(const Raw& v) const { return v; }
  typedef float Raw1;  // single element k (column-blocked staging of the split-bf16 TN kernel)
  __device__ __forceinline__ Raw1 fetch1(const Row& rw, int k, int K) const {
    return *(k < F ? rw.px + k : (k < K ? rw.ps + (k - F) : rw.px));
  }
  __device__ __forceinline__ float combine1(Raw1 v, const Row& rw, int k, int K) const {
    return (rw.ok && k < K) ? v : 0.f;
  }
};

// ------------------------------------------------------------------------------------------
// NT GEMM
// ------------------------------------------------------------------------------------------
template <int WAVES, int RM, int RN, int KT>
struct NTShape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RM, BN = RN * 16, BK = 16 * KT;
  static constexpr int CPR = 4 * KT;  // float4 chunks per row per k-tile
  static constexpr int ACH = BM * CPR, BCH = BN * CPR;
  static constexpr int APT = ACH / NT;
  static constexpr int BPT = (BCH + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr int STAGE_F4 = 2 * (ACH + BCH);
  static constexpr int EPI_F4 = (BM * LDC + 3) / 4;
  static constexpr int LDS_F4 = STAGE_F4 > EPI_F4 ? STAGE_F4 : EPI_F4;
  static_assert(ACH % NT == 0, "A chunks per thread must be integral");
};

// the next tile's global loads spread over the MFMAs, one per kNtIl (lab: layer NT gather 65.7 ->
// 59.0 us, plain 58.3 -> 53.8; step A/B -2 %; 4: -1.5 %)
constexpr int kNtIl = 5;
// OCC > 0 asks the compiler for OCC waves per SIMD (register budget 512 / OCC per lane)
template <int WAVES, int RM, int RN, int KT, int PF, int OCC, class AL, class BL, class EP>
__global__ __attribute__((amdgpu_flat_work_group_size(1, WAVES * 64),
                          amdgpu_waves_per_eu(OCC > 0 ? OCC : 1))) void
gemm_nt_kernel(AL al, BL bl, EP ep, int M, int N, int K, int tiles_n) {
  using S = NTShape<WAVES, RM, RN, KT>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BK = S::BK, CPR = S::CPR;
  constexpr int ACH = S::ACH, BCH = S::BCH, APT = S::APT, BPT = S::BPT;
  __shared__ float4 lds[S::LDS_F4];
  float4* As = lds;
  float4* Bs = lds + 2 * ACH;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  typename AL::Row arow[APT];
  int adst[APT], akof[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT;
    const int r = q / CPR, kc = q % CPR;
    arow[p] = al.row(m0 + r, M);
    akof[p] = kc * 4;
    adst[p] = ((kc >> 2) * BM + r) * 4 + ((kc & 3) ^ lds_swz(r));
  }
  typename BL::Row brow[BPT];
  int bdst[BPT], bkof[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    const int r = q / CPR, kc = q % CPR;
    const bool in = q < BCH;
    brow[p] = bl.row(in ? n0 + r : N, N);
    bkof[p] = kc * 4;
    bdst[p] = in ? ((kc >> 2) * BN + r) * 4 + ((kc & 3) ^ lds_swz(r)) : -1;
  }

  typename AL::Raw ra[APT];
  typename BL::Raw rb[BPT];
  floatx4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = fg ^ lds_swz(fr);

  auto fetch = [&](typename AL::Raw(&xa)[APT], typename BL::Raw(&xb)[BPT], int kb) {
#pragma unroll
    for (int p = 0; p < APT; ++p) xa[p] = al.fetch(arow[p], kb + akof[p], K);
#pragma unroll
    for (int p = 0; p < BPT; ++p) xb[p] = bl.fetch(brow[p], kb + bkof[p], K);
  };
  auto sstore = [&](const typename AL::Raw(&xa)[APT], const typename BL::Raw(&xb)[BPT], int buf,
                    int kb) {
    float4* An = As + buf * ACH;
    float4* Bn = Bs + buf * BCH;
#pragma unroll
    for (int p = 0; p < APT; ++p) An[adst[p]] = al.combine(xa[p], arow[p], kb + akof[p], K);
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bdst[p] >= 0) Bn[bdst[p]] = bl.combine(xb[p], brow[p], kb + bkof[p], K);
  };
  auto compute = [&](int buf) {
    const float4* Ac = As + buf * ACH;
    const float4* Bc = Bs + buf * BCH;
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
  };

  if constexpr (PF == 1) {
    fetch(ra, rb, 0);
    sstore(ra, rb, 0, 0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      const int kb = (kt + 1) * BK;
      if (more) fetch(ra, rb, kb);
      compute(cur);
      if (more) sstore(ra, rb, cur ^ 1, kb);
      __syncthreads();
    }
  } else {
    // prefetch distance 2: the global loads of tile t+2 are issued before tile t is computed and
    // consumed (written to LDS) only at the end of iteration t+1, so each load has two
    // iterations of MFMA work to land.  Register sets alternate by tile parity (loop unrolled
    // by 2 so they stay static); two LDS buffers suffice because a buffer is rewritten only
    // after the barrier that ends its readers' iteration.
    // Fetches are unconditional (tiles past K read in-bounds addresses and are zero-masked by
    // combine), so no branch separates a load from its consumer and the waitcnt pass can count.
    typename AL::Raw ra2[APT];
    typename BL::Raw rb2[BPT];
    fetch(ra, rb, 0);
    fetch(ra2, rb2, BK);
    sstore(ra, rb, 0, 0);
    __syncthreads();
    int kt = 0;
    // the loads of tile t+2 are spread over tile t's MFMAs (one per kNtIl) instead of issued as
    // one burst ahead of them
    auto il = [&]() {
      __builtin_amdgcn_sched_group_barrier(0x100, KT * (RM + RN), 0);  // fragment ds_reads
#pragma unroll
      for (int q = 0; q < APT * (sizeof(typename AL::Raw) / 16) + BPT; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, kNtIl, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    };
    for (; kt + 2 <= nk; kt += 2) {  // buf 0 holds tile kt, set 2 holds tile kt + 1
      fetch(ra, rb, (kt + 2) * BK);
      compute(0);
      il();
      __builtin_amdgcn_sched_barrier(0);
      sstore(ra2, rb2, 1, (kt + 1) * BK);
      __syncthreads();
      fetch(ra2, rb2, (kt + 3) * BK);
      compute(1);
      il();
      __builtin_amdgcn_sched_barrier(0);
      sstore(ra, rb, 0, (kt + 2) * BK);
      __syncthreads();
    }
    if (kt < nk) {
      compute(0);
      __syncthreads();  // the epilogue reuses the stage buffers
    }
  }

  // epilogue: accumulators -> LDS [BM][LDC] -> coalesced float4 rows -> ep.apply4p.  Every
  // operand load of the epilogue (h0 / Q rows, bias) is issued first, from clamped in-bounds
  // addresses, so they land while the accumulators go through LDS: one memory round trip per
  // tile instead of one per float4 piece.
  constexpr int C4 = BN / 4;
  constexpr int EIT = (BM * C4 + NT - 1) / NT;
  typename EP::Pre pv[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int q = min(tid + it * NT, BM * C4 - 1);
    const int r = q / C4, c4 = q - r * C4;
    pv[it] = ep.pre4(m0 + r, n0 + 4 * c4);
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
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int q = tid + it * NT;
    if (q < BM * C4) {
      const int r = q / C4, c4 = q - r * C4;
      const float4 v = *reinterpret_cast<const float4*>(&C[r * S::LDC + 4 * c4]);
      typename EP::Ctx cx = ep.ctx(n0 + 4 * c4);
      ep.finish_ctx(cx);
      ep.apply4p(m0 + r, n0 + 4 * c4, v, pv[it], cx);
    }
  }
}

template <int WAVES, int RM, int RN, int KT, class AL, class BL, class EP, int PF = 2, int OCC = 0>
inline hipError_t launch_gemm_nt(const AL& al, const BL& bl, const EP& ep, int M, int N, int K,
                                 hipStream_t st) {
  using S = NTShape<WAVES, RM, RN, KT>;
  if (M <= 0 || N <= 0) return hipSuccess;
  const int tm = (M + S::BM - 1) / S::BM, tn = (N + S::BN - 1) / S::BN;
  hipLaunchKernelGGL((gemm_nt_kernel<WAVES, RM, RN, KT, PF, OCC, AL, BL, EP>), dim3(tm * tn),
                     dim3(WAVES * 64), 0, st, al, bl, ep, M, N, K, tn);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// TN split-K GEMM (weight gradients)
// ------------------------------------------------------------------------------------------
struct TnPlan {
  int tiles_n, tiles_k, splits, rows_per_split;
};

template <int WAVES, int RM, int RN, int KT>
struct TNShape {
  static constexpr int NT = WAVES * 64;
  static constexpr int BM = WAVES * 16 * RM, BN = RN * 16, BE = 16 * KT;
  static constexpr int SA = BM + (((16 - BM % 32) % 32) + 32) % 32;  // == 16 (mod 32)
  static constexpr int SB = BN + (((16 - BN % 32) % 32) + 32) % 32;
  static constexpr int ACH = BE * BM / 4, BCH = BE * BN / 4;
  static constexpr int APT = ACH / NT;
  static constexpr int BPT = (BCH + NT - 1) / NT;
  static constexpr int LDC = BN + 4;
  static constexpr int STAGE_F = 2 * BE * (SA + SB);
  static constexpr int EPI_F = BM * LDC;
  static constexpr int LDS_F = STAGE_F > EPI_F ? STAGE_F : EPI_F;
  static_assert(ACH % NT == 0, "A chunks per thread must be integral");
};

template <int WAVES, int RM, int RN, int KT, class AL, class BL, int PF>
__global__ __launch_bounds__(WAVES * 64) void gemm_tn_kernel(
    AL al, BL bl, float* __restrict__ slab, float* __restrict__ bslab, int Nout, int Kout, int R,
    int rows_per_split, int tiles_k, int want_bias) {
  using S = TNShape<WAVES, RM, RN, KT>;
  constexpr int NT = S::NT, BM = S::BM, BN = S::BN, BE = S::BE, SA = S::SA, SB = S::SB;
  constexpr int BCH = S::BCH, APT = S::APT, BPT = S::BPT;
  __shared__ __attribute__((aligned(16))) float lds[S::LDS_F];
  float* At = lds;
  float* Bt = lds + 2 * BE * SA;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // 1-D grid of tiles x splits; the XCD-contiguous remap puts all output tiles of one split (which
  // read the same rows) on one XCD, so their re-reads of those rows hit that XCD's L2
  const int ntiles = ((Nout + BM - 1) / BM) * tiles_k;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles, tile = lin - split * ntiles;
  const int tnn = tile / tiles_k, tkk = tile - tnn * tiles_k;
  const int n0 = tnn * BM, k0 = tkk * BN;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);
  const int nt = e_end > e_begin ? (e_end - e_begin + BE - 1) / BE : 0;

  int ae[APT], ac[APT];
#pragma unroll
  for (int p = 0; p < APT; ++p) {
    const int q = tid + p * NT;
    ae[p] = q / (BM / 4);
    ac[p] = (q % (BM / 4)) * 4;
  }
  int be[BPT], bc[BPT];
  bool bin[BPT];
#pragma unroll
  for (int p = 0; p < BPT; ++p) {
    const int q = tid + p * NT;
    bin[p] = q < BCH;
    be[p] = bin[p] ? q / (BN / 4) : 0;
    bc[p] = bin[p] ? (q % (BN / 4)) * 4 : 0;
  }
  // rows of the next tile to fetch (computed one tile ahead: index loads have a tile to land)
  typename AL::Row arow[APT];
  typename BL::Row brow[BPT];
  auto mkrows = [&](int t) {
    const int e0 = e_begin + t * BE;
#pragma unroll
    for (int p = 0; p < APT; ++p) arow[p] = al.row(e0 + ae[p], e_end);
#pragma unroll
    for (int p = 0; p < BPT; ++p) brow[p] = bl.row(e0 + be[p], bin[p] ? e_end : 0);
  };
  // one tile in registers: the rows it was fetched with (for combine) and the raw loads
  struct Set {
    typename AL::Row ar[APT];
    typename BL::Row br[BPT];
    typename AL::Raw ra[APT];
    typename BL::Raw rb[BPT];
  };
  auto fetch = [&](Set& x) {
#pragma unroll
    for (int p = 0; p < APT; ++p) {
      x.ar[p] = arow[p];
      x.ra[p] = al.fetch(arow[p], n0 + ac[p], Nout);
    }
#pragma unroll
    for (int p = 0; p < BPT; ++p) {
      x.br[p] = brow[p];
      x.rb[p] = bl.fetch(brow[p], k0 + bc[p], Kout);
    }
  };
  auto sstore = [&](const Set& x, int buf) {
    float* Ab = At + buf * BE * SA;
    float* Bb = Bt + buf * BE * SB;
#pragma unroll
    for (int p = 0; p < APT; ++p)
      *reinterpret_cast<float4*>(&Ab[ae[p] * SA + ac[p]]) =
          al.combine(x.ra[p], x.ar[p], n0 + ac[p], Nout);
#pragma unroll
    for (int p = 0; p < BPT; ++p)
      if (bin[p])
        *reinterpret_cast<float4*>(&Bb[be[p] * SB + bc[p]]) =
            bl.combine(x.rb[p], x.br[p], k0 + bc[p], Kout);
  };

  floatx4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const bool do_bias = want_bias && tkk == 0 && tid < BM;
  const int fr = lane & 15, fg = lane >> 4;
  auto compute = [&](int cur) {
    const float* Ab = At + cur * BE * SA;
    const float* Bb = Bt + cur * BE * SB;
#pragma unroll
    for (int s = 0; s < 4 * KT; ++s) {
      const int er = 4 * s + fg;
      float av[RM], bv[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) av[i] = Ab[er * SA + w * 16 * RM + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < RN; ++j) bv[j] = Bb[er * SB + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (do_bias) {
#pragma unroll
      for (int e = 0; e < BE; ++e) bsum += Ab[e * SA + tid];
    }
  };

  if constexpr (PF == 1) {
    Set x;
    if (nt > 0) {
      mkrows(0);
      fetch(x);
      mkrows(1);
      sstore(x, 0);
    }
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      const bool more = t + 1 < nt;
      if (more) {
        fetch(x);       // tile t+1, rows prepared during the previous iteration
        mkrows(t + 2);  // index loads for tile t+2
      }
      compute(cur);
      if (more) sstore(x, cur ^ 1);
      __syncthreads();
    }
  } else if (nt > 0) {
    // prefetch distance 2: tile t+2 is fetched before tile t is computed and written to LDS at
    // the end of iteration t+1.  Fetches are unconditional (rows past e_end read row 0, masked by
    // combine), so no branch separates a load from its consumer; register sets alternate by tile
    // parity (loop unrolled by 2).
    Set x0, x1;
    mkrows(0);
    fetch(x0);
    mkrows(1);
    fetch(x1);
    mkrows(2);
    sstore(x0, 0);
    __syncthreads();
    int t = 0;
    for (; t + 2 <= nt; t += 2) {
      fetch(x0);  // tile t+2
      mkrows(t + 3);
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      sstore(x1, 1);  // tile t+1 (t + 1 < nt here)
      __syncthreads();
      fetch(x1);  // tile t+3
      mkrows(t + 4);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nt) sstore(x0, 0);  // tile t+2
      __syncthreads();
    }
    if (t < nt) {
      compute(0);
      __syncthreads();
    }
  } else {
    __syncthreads();
  }

  float* C = lds;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        C[(w * 16 * RM + i * 16 + fg * 4 + r) * S::LDC + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  // slab rows are padded to ldk = round_up(Kout, 4) floats so every store is a float4
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

template <int WAVES, int RM, int RN, int KT>
inline TnPlan plan_tn(int Nout, int Kout, int R, int target_wgs) {
  using S = TNShape<WAVES, RM, RN, KT>;
  TnPlan p;
  p.tiles_n = (Nout + S::BM - 1) / S::BM;
  p.tiles_k = (Kout + S::BN - 1) / S::BN;
  const int tiles = p.tiles_n * p.tiles_k;
  // floor, not ceil: the grid must not exceed the target (a whole number of workgroups per CU);
  // one workgroup past it puts an extra one on a few CUs, and those CUs set the kernel's time
  int splits = target_wgs / tiles;
  const int max_splits = (R + 4 * S::BE - 1) / (4 * S::BE);  // >= 4 k-tiles per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + S::BE - 1) / S::BE * S::BE;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

// TN prefetch distance (2: same-box A/B +1 % step time, layer wgrad slower, node/readout faster)
constexpr int kTnPf = 1;
template <int WAVES, int RM, int RN, int KT, class AL, class BL, int PF = kTnPf>
inline hipError_t launch_gemm_tn(const AL& al, const BL& bl, const TnPlan& p, float* slab,
                                 float* bslab, int Nout, int Kout, int R, bool want_bias,
                                 hipStream_t st) {
  hipLaunchKernelGGL((gemm_tn_kernel<WAVES, RM, RN, KT, AL, BL, PF>),
                     dim3(p.tiles_n * p.tiles_k * p.splits), dim3(WAVES * 64), 0, st, al, bl, slab,
                     bslab, Nout, Kout, R, p.rows_per_split, p.tiles_k, want_bias ? 1 : 0);
  return hipGetLastError();
}

}  // namespace cgr
