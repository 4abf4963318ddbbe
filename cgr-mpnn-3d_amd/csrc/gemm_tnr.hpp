// Register-direct TN GEMM for the weight gradients (gfx950, fp32 MFMA, no LDS in the main loop).
//
//   C[n, k] = sum_e A(e, n) * B(e, k)          (dW = dZ^T Q: A = dZ rows, B = Q rows)
//
// "Strided fragments": with the reduction index e as the MFMA k dimension, lane (fr, fg) of a
// v_mfma_f32_16x16x4_f32 supplies A(e = e0 + fg, m = fr) and B(e0 + fg, n = fr).  Output row
// fragment i of a wave tile is mapped to the rows n0 + FA * m + i (m = 0..15), so the FA
// consecutive values A(e, n0 + FA*fr .. + FA-1) that ONE lane loads with a 16-byte (+4-byte)
// load are exactly its operands for the FA row fragments; likewise FB column fragments.  A wave
// therefore streams its operands straight from L2 into registers, FA*FB MFMAs per 4 rows of e,
// with no LDS traffic and no barrier in the loop.
//
// Decomposition: a workgroup = 4 waves = one (16 FA x 16 FB) output tile and one split (row range)
// of e; the 4 waves take interleaved 4-row steps of the split and their partial tiles are combined
// through LDS in a fixed order ((w0 + w1) + (w2 + w3)) before the split's fp32 slab is written
// (same slab layout as gemm_tn_kernel, so reduce_slabs is shared).  Deterministic.
#pragma once

#include "common.hpp"
#include "gemm.hpp"

namespace cgr {

// F consecutive floats p[0 .. F-1] (4-byte aligned: gfx950 global loads need no 16-byte alignment)
template <int F>
__device__ __forceinline__ void tnr_ld(const float* __restrict__ p, float (&v)[F]) {
  if constexpr (F >= 4) {
    float4 q;
    __builtin_memcpy(&q, p, 16);
    v[0] = q.x;
    v[1] = q.y;
    v[2] = q.z;
    v[3] = q.w;
#pragma unroll
    for (int i = 4; i < F; ++i) v[i] = p[i];
  } else {
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] = p[i];
  }
}

// plain rows: value(e, c) = p[e * ld + c]
struct TnrRows {
  const float* p;
  int64_t ld;
  struct Idx {};
  __device__ __forceinline__ Idx idx(int) const { return Idx{}; }
  template <int F>
  struct Raw {
    float v[F];
  };
  template <int F>
  __device__ __forceinline__ void fetch(int e, const Idx&, int c, Raw<F>& r) const {
    tnr_ld<F>(p + (int64_t)e * ld + c, r.v);
  }
  template <int F>
  __device__ __forceinline__ void combine(const Raw<F>& r, float (&v)[F]) const {
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] = r.v[i];
  }
};

// message rows of a layer: value(e, c) = a[src[e], c] - h[rev[e], c]   (GNN.py:136-141)
struct TnrDiff {
  const float* a;
  const float* h;
  const int* src;
  const int* rev;
  int64_t ld;
  struct Idx {
    int s, r;
  };
  __device__ __forceinline__ Idx idx(int e) const { return Idx{src[e], rev[e]}; }
  template <int F>
  struct Raw {
    float va[F], vh[F];
  };
  template <int F>
  __device__ __forceinline__ void fetch(int, const Idx& x, int c, Raw<F>& r) const {
    tnr_ld<F>(a + (int64_t)x.s * ld + c, r.va);
    tnr_ld<F>(h + (int64_t)x.r * ld + c, r.vh);
  }
  template <int F>
  __device__ __forceinline__ void combine(const Raw<F>& r, float (&v)[F]) const {
#pragma unroll
    for (int i = 0; i < F; ++i) v[i] = r.va[i] - r.vh[i];
  }
};

// [x | s] rows of the readout (GNN.py:106): value(e, c) = c < F ? x[e, c] : s[e, c - F]; F % 4 == 0
// (x padded to 16-byte rows), so a lane's run of FB <= 4 columns never straddles the seam
struct TnrConcat {
  const float* x;
  int64_t ldx;
  const float* s;
  int64_t lds;
  int F;
  struct Idx {};
  __device__ __forceinline__ Idx idx(int) const { return Idx{}; }
  template <int F_>
  struct Raw {
    float v[F_];
  };
  template <int F_>
  __device__ __forceinline__ void fetch(int e, const Idx&, int c, Raw<F_>& r) const {
    tnr_ld<F_>(c < F ? x + (int64_t)e * ldx + c : s + (int64_t)e * lds + (c - F), r.v);
  }
  template <int F_>
  __device__ __forceinline__ void combine(const Raw<F_>& r, float (&v)[F_]) const {
#pragma unroll
    for (int i = 0; i < F_; ++i) v[i] = r.v[i];
  }
};

struct TnrPlan {
  int tiles_n, tiles_k, splits, rows_per_split;
};

constexpr int TNR_WAVES = 4;
// data loads 2 steps (8 rows) ahead of the MFMAs, row indices 3
constexpr int kTnrPf = 2;

template <int FA, int FB, class SA, class SB>
__global__ __launch_bounds__(TNR_WAVES * 64, 2) void gemm_tnr_kernel(
    SA sa, SB sb, float* __restrict__ slab, float* __restrict__ bslab, int Nout, int Kout, int R,
    int rows_per_split, int tiles_k, int want_bias) {
  constexpr int TM = 16 * FA, TK = 16 * FB;
  __shared__ __attribute__((aligned(16))) float red[2][64 * FA * FB * 4];  // two partial tiles
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int tiles_n = (Nout + TM - 1) / TM;
  const int ntiles = tiles_n * tiles_k;
  // XCD-contiguous remap: the tiles of one split (same rows of A and B) share an XCD's L2
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / ntiles, tile = lin - split * ntiles;
  const int tn = tile / tiles_k, tk = tile - tn * tiles_k;
  const int n0 = tn * TM, k0 = tk * TK;
  const int e_begin = split * rows_per_split;
  const int e_end = min(R, e_begin + rows_per_split);

  // this lane's FA rows of the tile, FB columns.  Nout % FA == 0 and Kout % FB == 0 (launcher
  // checks), so a lane's run is either fully valid or fully past the end; the latter is clamped in
  // bounds and only reaches outputs that are never stored
  const int na = min(n0 + FA * fr, Nout - FA);
  const int kb = min(k0 + FB * fr, Kout - FB);

  floatx4 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bs[FA];
#pragma unroll
  for (int i = 0; i < FA; ++i) bs[i] = 0.f;

  // wave w takes steps w, w + 4, ... of 4 rows each; lane group fg row e = base + fg
  const int nrows = max(e_end - e_begin, 0);
  const int nsteps = (nrows + 3) >> 2;
  const int my_steps = nsteps > w ? (nsteps - w + TNR_WAVES - 1) / TNR_WAVES : 0;
  // step t of this wave -> row e (clamped to a valid row; ok = inside the split)
  auto row_of = [&](int t, bool& ok) {
    const int e = e_begin + 4 * (w + TNR_WAVES * t) + fg;
    ok = e < e_end;
    return ok ? e : (e_begin < R ? e_begin : 0);
  };
  // index rows (gathered sources) are loaded one step ahead of the data loads, which are one step
  // ahead of the MFMAs: no load waits on another load inside a step
  constexpr int NB = kTnrPf + 1;  // register sets: data kTnrPf steps ahead
  typename SA::template Raw<FA> ra[NB];
  typename SB::template Raw<FB> rb[NB];
  typename SA::Idx ia[NB];
  typename SB::Idx ib[NB];
  int er[NB];
  bool ok[NB], okn[NB];
  auto fetch_idx = [&](int t, int buf) {
    er[buf] = row_of(t, okn[buf]);
    ia[buf] = sa.idx(er[buf]);
    ib[buf] = sb.idx(er[buf]);
  };
  auto fetch = [&](int buf) {  // data of the step whose indices sit in idx buffer buf
    ok[buf] = okn[buf];
    sa.template fetch<FA>(er[buf], ia[buf], na, ra[buf]);
    sb.template fetch<FB>(er[buf], ib[buf], kb, rb[buf]);
  };
  auto compute = [&](int buf) {
    float av[FA], bv[FB];
    sa.template combine<FA>(ra[buf], av);
    sb.template combine<FB>(rb[buf], bv);
#pragma unroll
    for (int i = 0; i < FA; ++i) av[i] = ok[buf] ? av[i] : 0.f;  // rows past the split: 0
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < FA; ++i) bs[i] += av[i];
  };
  if (my_steps > 0) {
    // steps past my_steps re-read a valid row (never consumed)
    auto cl = [&](int t) { return t < my_steps ? t : my_steps - 1; };
    int t = 0;
    fetch_idx(0, 0);
    fetch_idx(cl(1), 1);
    fetch_idx(cl(2), 2);
    fetch(0);
    fetch(1);
    for (; t + 3 <= my_steps; t += 3) {
      fetch(2);
      fetch_idx(cl(t + 3), 0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      fetch(0);
      fetch_idx(cl(t + 4), 1);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      fetch(1);
      fetch_idx(cl(t + 5), 2);
      compute(2);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < my_steps) compute(0);
    if (t + 1 < my_steps) compute(1);
  }

  // ---- fixed-order combine of the 4 waves' partial tiles: (w0 + w1) + (w2 + w3) ----
  constexpr int NV = FA * FB * 4;  // accumulator values per lane
  auto put = [&](float* dst) {
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[((i * FB + j) * 4 + r) * 64 + lane] = acc[i][j][r];
  };
  auto add = [&](const float* src) {
#pragma unroll
    for (int i = 0; i < FA; ++i) {
#pragma unroll
      for (int j = 0; j < FB; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += src[((i * FB + j) * 4 + r) * 64 + lane];
      __builtin_amdgcn_sched_barrier(0);  // bound the LDS values in flight (registers)
    }
  };
  (void)NV;
  if (w & 1) put(red[w >> 1]);
  __syncthreads();
  if (!(w & 1)) add(red[w >> 1]);
  __syncthreads();
  if (w == 2) put(red[0]);
  __syncthreads();
  if (w == 0) {
    add(red[0]);
    // slab [split][Nout][ldk]: element (n0 + FA*(4fg + r) + i, k0 + FB*fr + j)
    const int ldk = (Kout + 3) & ~3;
    float* out = slab + (int64_t)split * Nout * ldk;
    const int kc = k0 + FB * fr;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < FA; ++i) {
        const int n = n0 + FA * (4 * fg + r) + i;
        if (n >= Nout) continue;
        float* o = out + (int64_t)n * ldk + kc;
        if (FB == 4 && kc + 4 <= Kout) {
          *reinterpret_cast<float4*>(o) =
              make_float4(acc[i][0][r], acc[i][1 % FB][r], acc[i][2 % FB][r], acc[i][3 % FB][r]);
        } else {
#pragma unroll
          for (int j = 0; j < FB; ++j)
            if (kc + j < Kout) o[j] = acc[i][j][r];
        }
      }
  }
  // bias column sums (tiles of the first column block): per lane sum over its rows, combined
  // over the lane groups and then the waves in fixed orders
  if (want_bias && tk == 0) {
#pragma unroll
    for (int i = 0; i < FA; ++i) {
      float v = bs[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      bs[i] = v;
    }
    __syncthreads();
    float* bred = red[0];
    if (fg == 0) {
#pragma unroll
      for (int i = 0; i < FA; ++i) bred[(w * FA + i) * 16 + fr] = bs[i];
    }
    __syncthreads();
    if (w == 0 && fg == 0) {
#pragma unroll
      for (int i = 0; i < FA; ++i) {
        const int n = n0 + FA * fr + i;
        const float v = (bred[(0 * FA + i) * 16 + fr] + bred[(1 * FA + i) * 16 + fr]) +
                        (bred[(2 * FA + i) * 16 + fr] + bred[(3 * FA + i) * 16 + fr]);
        if (n < Nout && n0 + FA * fr + i < n0 + TM) bslab[(int64_t)split * Nout + n] = v;
      }
    }
  }
}

// splits: floor(target / tiles) workgroups (no CU gets an extra one), >= 16 rows per wave step set
template <int FA, int FB>
inline TnrPlan plan_tnr(int Nout, int Kout, int R, int target_wgs) {
  TnrPlan p;
  p.tiles_n = (Nout + 16 * FA - 1) / (16 * FA);
  p.tiles_k = (Kout + 16 * FB - 1) / (16 * FB);
  const int tiles = p.tiles_n * p.tiles_k;
  int splits = target_wgs / tiles;
  const int max_splits = (R + 63) / 64;  // >= 64 rows (4 steps per wave) per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int rps = (R + splits - 1) / splits;
  rps = (rps + 15) / 16 * 16;
  p.splits = R > 0 ? (R + rps - 1) / rps : 1;
  p.rows_per_split = rps;
  return p;
}

// requires Nout % FA == 0, Kout % FB == 0 (tnr_ok)
template <int FA, int FB>
inline bool tnr_ok(int Nout, int Kout) {
  return Nout >= FA && Kout >= FB && Nout % FA == 0 && Kout % FB == 0;
}
template <int FA, int FB, class SA, class SB>
inline hipError_t launch_gemm_tnr(const SA& sa, const SB& sb, const TnrPlan& p, float* slab,
                                  float* bslab, int Nout, int Kout, int R, bool want_bias,
                                  hipStream_t st) {
  hipLaunchKernelGGL((gemm_tnr_kernel<FA, FB, SA, SB>), dim3(p.tiles_n * p.tiles_k * p.splits),
                     dim3(TNR_WAVES * 64), 0, st, sa, sb, slab, bslab, Nout, Kout, R,
                     p.rows_per_split, p.tiles_k, want_bias ? 1 : 0);
  return hipGetLastError();
}

}  // namespace cgr
