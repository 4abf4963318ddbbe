#include <algorithm>
#include <type_traits>
// Non-GEMM kernels of the D-MPNN path: segmented sums (the sum-scatter of GNN.py:134 / :110),
// edge init, pooling + ffn head, backward activation kernels, deterministic split-K reduction.
// All are HBM/L2-streaming kernels: float4 per lane along the hidden dimension, rows of one
// segment are contiguous (dst-sorted edges) so every wave reads whole 1.6 KB rows.
#include "common.hpp"
#include "kernels.hpp"
#include "bwd_rows.hpp"
#include "reduce.hpp"

namespace cgr {

// ------------------------------------------------------------------------------------------
// segmented sum
// ------------------------------------------------------------------------------------------
// one thread per ITEMS (segment, float4 column) items; each segment's rows are summed in index
// order (deterministic), the loads of its first three rows issued together (a runtime-trip-count
// loop would serialise them: ptr -> row -> add -> next row); segments average ~2 rows on
// T1x-shaped graphs
// Items are spaced a grid apart; every index load of all items is issued first, then the first
// three rows of each (clamped), then the adds: a thread keeps ITEMS x 3 row loads in flight
// (one item per thread streamed 3.5 TB/s from HBM at cfg2, the round-4 VERDICT's cold-cache
// question).
template <bool GATHER, int ITEMS>
__global__ __launch_bounds__(256) void k_segsum_v4m(const float* __restrict__ vals, int64_t ldv,
                                                    const int* __restrict__ idx,
                                                    const int* __restrict__ ptr, int64_t nseg,
                                                    int C4, float* __restrict__ out, int64_t ldo) {
  const int64_t tot = nseg * C4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t v[ITEMS];
  int c[ITEMS], b[ITEMS], e[ITEMS];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int64_t t = t0 + k * stride;
    const bool ok = t < tot;
    v[k] = ok ? t / C4 : 0;
    c[k] = ok ? (int)(t - v[k] * C4) : 0;
    b[k] = ok ? ptr[v[k]] : 0;
    e[k] = ok ? ptr[v[k] + 1] : 0;
  }
  auto row = [&](int j) -> int64_t { return GATHER ? (int64_t)idx[j] : (int64_t)j; };
  float4 x[ITEMS][3];
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int last = e[k] > b[k] ? e[k] - 1 : b[k];
    const float* base = vals + 4 * c[k];
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // an empty segment (or a thread past the end) loads nothing:
      const int jj = min(b[k] + j, last);  // `vals` may have no rows at all
      x[k][j] = e[k] > b[k] ? *reinterpret_cast<const float4*>(base + row(jj) * ldv) : f4zero();
    }
  }
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    if (t0 + k * stride >= tot) continue;
    const int n = e[k] - b[k];
    float4 acc = f4zero();
    if (n > 0) acc = f4add(acc, x[k][0]);
    if (n > 1) acc = f4add(acc, x[k][1]);
    if (n > 2) acc = f4add(acc, x[k][2]);
    const float* base = vals + 4 * c[k];
    for (int j = b[k] + 3; j < e[k]; ++j)
      acc = f4add(acc, *reinterpret_cast<const float4*>(base + row(j) * ldv));
    *reinterpret_cast<float4*>(out + v[k] * ldo + 4 * c[k]) = acc;
  }
}

template <bool GATHER>
__global__ __launch_bounds__(256) void k_segsum_s(const float* __restrict__ vals, int64_t ldv,
                                                  const int* __restrict__ idx,
                                                  const int* __restrict__ ptr, int64_t nseg,
                                                  int W, float* __restrict__ out, int64_t ldo) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nseg * W) return;
  const int64_t v = t / W;
  const int c = (int)(t - v * W);
  const int b = ptr[v], e = ptr[v + 1];
  float acc = 0.f;
  for (int j = b; j < e; ++j) {
    const int64_t row = GATHER ? idx[j] : j;
    acc += vals[row * ldv + c];
  }
  out[v * ldo + c] = acc;
}

hipError_t segment_sum(const float* vals, int64_t ldv, const int* idx, const int* ptr,
                       int64_t nseg, int64_t width, float* out, int64_t ldo, hipStream_t st) {
  if (nseg <= 0 || width <= 0) return hipSuccess;
  const bool v4 = (width % 4 == 0) && (ldv % 4 == 0) && (ldo % 4 == 0) &&
                  ((uintptr_t)vals % 16 == 0) && ((uintptr_t)out % 16 == 0);
  const int T = 256;
  if (v4) {  // two items per thread (scatter lab, r05: cold 10.6 -> 9.6 us at cfg2; 4: 10.3)
    const int C4 = (int)(width / 4);
    const int64_t tot = nseg * C4;
    const int64_t grid = cdiv(cdiv(tot, 2), T);
    if (idx)
      hipLaunchKernelGGL((k_segsum_v4m<true, 2>), dim3(grid), dim3(T), 0, st, vals, ldv, idx, ptr,
                         nseg, C4, out, ldo);
    else
      hipLaunchKernelGGL((k_segsum_v4m<false, 2>), dim3(grid), dim3(T), 0, st, vals, ldv, idx,
                         ptr, nseg, C4, out, ldo);
  } else {
    const int64_t tot = nseg * width;
    if (idx)
      hipLaunchKernelGGL(k_segsum_s<true>, dim3(cdiv(tot, T)), dim3(T), 0, st, vals, ldv, idx,
                         ptr, nseg, (int)width, out, ldo);
    else
      hipLaunchKernelGGL(k_segsum_s<false>, dim3(cdiv(tot, T)), dim3(T), 0, st, vals, ldv, idx,
                         ptr, nseg, (int)width, out, ldo);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// batched 32x32-tiled transpose
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_transpose(TransposeJobs jobs) {
  const TransposeJob jb = jobs.job[blockIdx.y];
  const int tr = (jb.rows + 31) / 32, tc = (jb.cols + 31) / 32;
  const int tile = blockIdx.x;
  if (tile >= tr * tc) return;
  const int r0 = (tile / tc) * 32, c0 = (tile % tc) * 32;
  __shared__ float s[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    s[i][tx] = (r < jb.rows && c < jb.cols) ? jb.src[(int64_t)r * jb.ld_src + jb.col_off + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (r < jb.rows && c < jb.cols) jb.dst[(int64_t)c * jb.ld_dst + r] = s[tx][i];
  }
}

hipError_t transpose_batch(const TransposeJobs& jobs, hipStream_t st) {
  if (jobs.n <= 0) return hipSuccess;
  int maxt = 1;
  for (int j = 0; j < jobs.n; ++j) {
    const int t = (int)(cdiv(jobs.job[j].rows, 32) * cdiv(jobs.job[j].cols, 32));
    maxt = t > maxt ? t : maxt;
  }
  hipLaunchKernelGGL(k_transpose, dim3(maxt, jobs.n), dim3(256), 0, st, jobs);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// edge init (GNN.py:85-87) after the node-level GEMM P = x @ W0[:, :F]^T
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_edge_init(const float* __restrict__ P,
                                                   const int* __restrict__ src_s,
                                                   const float* __restrict__ e_s, int Fe, int Fep,
                                                   const float* __restrict__ w0eT,
                                                   const float* __restrict__ b0, int64_t E, int H,
                                                   int Hp, int act, float* __restrict__ h0,
                                                   float* __restrict__ pre0) {
  const int C4 = Hp >> 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * C4) return;
  const int64_t i = t / C4;
  const int c = (int)(t - i * C4);
  const int n = 4 * c;
  float4 z = *reinterpret_cast<const float4*>(P + (int64_t)src_s[i] * Hp + n);
  z.x += b0[min(n, H - 1)];
  z.y += b0[min(n + 1, H - 1)];
  z.z += b0[min(n + 2, H - 1)];
  z.w += b0[min(n + 3, H - 1)];
  const float* er = e_s + i * Fep;
  for (int q = 0; q < Fe; ++q) {
    const float ev = er[q];
    const float4 w = *reinterpret_cast<const float4*>(w0eT + (int64_t)q * Hp + n);
    z.x += ev * w.x;
    z.y += ev * w.y;
    z.z += ev * w.z;
    z.w += ev * w.w;
  }
  const int64_t o = i * Hp + n;
  if (pre0) *reinterpret_cast<float4*>(pre0 + o) = z;
  float4 h;
  h.x = act_fwd(z.x, act);
  h.y = act_fwd(z.y, act);
  h.z = act_fwd(z.z, act);
  h.w = act_fwd(z.w, act);
  *reinterpret_cast<float4*>(h0 + o) = h;
}

hipError_t edge_init_fwd(const float* P, const int* src_s, const float* e_s, int Fe, int Fep,
                         const float* w0eT, const float* b0, int64_t E, int H, int Hp, int act,
                         float* h0, float* pre0, hipStream_t st) {
  if (E <= 0) return hipSuccess;
  const int64_t tot = E * (Hp / 4);
  hipLaunchKernelGGL(k_edge_init, dim3(cdiv(tot, 256)), dim3(256), 0, st, P, src_s, e_s, Fe, Fep,
                     w0eT, b0, E, H, Hp, act, h0, pre0);
  return hipGetLastError();
}

// Edge init fused with the first dst segmented sum: a_0[v] = sum_{dst(i) = v} h0[i].  A block
// owns kEiNodes consecutive nodes, i.e. the contiguous dst-sorted edge range of their in-edges;
// thread c owns float4 column c, keeps its slice of W0[:, F:]^T (Fe x 4) in registers across
// all those edges (the per-edge kernel reloaded it for every edge: 14 float4 + 14 scalar loads
// per output float4), and sums its edges' h0 into a_0 in edge order -- the same adds, in the same
// order, as k_edge_init followed by k_segsum_v4m<false, 2>, so h0 / pre0 / a_0 are bitwise unchanged.
constexpr int kEiNodes = 4;  // (2: A/B -0.5 %)
constexpr int kEiMaxFe = 16;

template <bool REG>
__global__ __launch_bounds__(128) void k_edge_init_seg(
    const float* __restrict__ P, const int* __restrict__ src_s, const float* __restrict__ e_s,
    int Fe, int Fep, const float* __restrict__ w0eT, const float* __restrict__ b0,
    const int* __restrict__ dst_ptr, int64_t N, int H, int Hp, int act, float* __restrict__ h0,
    float* __restrict__ pre0, float* __restrict__ a, SegZero zero) {
  const int C4 = Hp >> 2;
  const int c = threadIdx.x;
  if (c >= C4) return;  // no barriers below
  const int n = 4 * c;
  const float4 bias = make_float4(b0[min(n, H - 1)], b0[min(n + 1, H - 1)],
                                  b0[min(n + 2, H - 1)], b0[min(n + 3, H - 1)]);
  float4 w[REG ? kEiMaxFe : 1];
  if constexpr (REG) {
#pragma unroll
    for (int q = 0; q < kEiMaxFe; ++q)
      w[q] = q < Fe ? *reinterpret_cast<const float4*>(w0eT + (int64_t)q * Hp + n) : f4zero();
  }
  const int64_t v0 = (int64_t)blockIdx.x * kEiNodes;
  const int64_t v1 = v0 + kEiNodes < N ? v0 + kEiNodes : N;
  // one edge: P row (gathered) + bias + e W0e^T -> pre0, h0 (loads come from ld())
  struct EdgeIn {
    float4 p;
    float4 e[kEiMaxFe / 4];
  };
  auto ld = [&](int i) {
    EdgeIn x;
    x.p = *reinterpret_cast<const float4*>(P + (int64_t)src_s[i] * Hp + n);
    if constexpr (REG) {
      const float* er = e_s + (int64_t)i * Fep;
#pragma unroll
      for (int q4 = 0; q4 < kEiMaxFe / 4; ++q4)
        x.e[q4] = 4 * q4 < Fe ? *reinterpret_cast<const float4*>(er + 4 * q4) : f4zero();
    }
    return x;
  };
  auto edge = [&](int i, const EdgeIn& x) {
    float4 z = x.p;
    z.x += bias.x;
    z.y += bias.y;
    z.z += bias.z;
    z.w += bias.w;
    if constexpr (REG) {
#pragma unroll
      for (int q4 = 0; q4 < kEiMaxFe / 4; ++q4) {
        if (4 * q4 >= Fe) break;
        const float e4[4] = {x.e[q4].x, x.e[q4].y, x.e[q4].z, x.e[q4].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (4 * q4 + k >= Fe) break;
          const float4 wq = w[4 * q4 + k];
          z.x += e4[k] * wq.x;
          z.y += e4[k] * wq.y;
          z.z += e4[k] * wq.z;
          z.w += e4[k] * wq.w;
        }
      }
    } else {
      const float* er = e_s + (int64_t)i * Fep;
      for (int q = 0; q < Fe; ++q) {
        const float ev = er[q];
        const float4 wq = *reinterpret_cast<const float4*>(w0eT + (int64_t)q * Hp + n);
        z.x += ev * wq.x;
        z.y += ev * wq.y;
        z.z += ev * wq.z;
        z.w += ev * wq.w;
      }
    }
    const int64_t o = (int64_t)i * Hp + n;
    if (pre0) *reinterpret_cast<float4*>(pre0 + o) = z;
    float4 h;
    h.x = act_fwd(z.x, act);
    h.y = act_fwd(z.y, act);
    h.z = act_fwd(z.z, act);
    h.w = act_fwd(z.w, act);
    *reinterpret_cast<float4*>(h0 + o) = h;
    return h;
  };
  for (int64_t v = v0; v < v1; ++v) {
    float4 acc = f4zero();
    const int ib = dst_ptr[v], ie = dst_ptr[v + 1];
    // the node's edges two at a time, both edges' loads issued before either is used (a chain
    // of single edges serialised src index -> P row -> store per edge); summed in edge order
    int i = ib;
    for (; i + 2 <= ie; i += 2) {
      const EdgeIn x0 = ld(i), x1 = ld(i + 1);
      acc = f4add(acc, edge(i, x0));
      acc = f4add(acc, edge(i + 1, x1));
    }
    if (i < ie) acc = f4add(acc, edge(i, ld(i)));
    *reinterpret_cast<float4*>(a + v * Hp + n) = acc;
    if (zero.n > 0) {
      if (ie == ib || ib / zero.tile_rows != (ie - 1) / zero.tile_rows)
        for (int l = 0; l < zero.n; ++l)
          *reinterpret_cast<float4*>(zero.a[l] + v * Hp + n) = f4zero();
    }
  }
}

hipError_t edge_init_segsum_fwd(const float* P, const int* src_s, const float* e_s, int Fe,
                                int Fep, const float* w0eT, const float* b0, const int* dst_ptr,
                                int64_t N, int H, int Hp, int act, float* h0, float* pre0,
                                float* a, hipStream_t st, const SegZero* zero) {
  if (N <= 0) return hipSuccess;
  if (Hp % 4 || Hp / 4 > 128) return hipErrorInvalidValue;  // one thread per float4 column
  SegZero z{};
  if (zero) {
    if (zero->n > 32 || zero->tile_rows <= 0) return hipErrorInvalidValue;
    z = *zero;
  }
  const int threads = (Hp / 4 + 63) / 64 * 64;
  const int nb = (int)cdiv(N, kEiNodes);
  if (Fe <= kEiMaxFe && (Fe == 0 || Fep % 4 == 0))
    hipLaunchKernelGGL(k_edge_init_seg<true>, dim3(nb), dim3(threads), 0, st, P, src_s, e_s, Fe,
                       Fep, w0eT, b0, dst_ptr, N, H, Hp, act, h0, pre0, a, z);
  else
    hipLaunchKernelGGL(k_edge_init_seg<false>, dim3(nb), dim3(threads), 0, st, P, src_s, e_s, Fe,
                       Fep, w0eT, b0, dst_ptr, N, H, Hp, act, h0, pre0, a, z);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// add-pool + ffn head (GNN.py:110): one workgroup per graph
// ------------------------------------------------------------------------------------------
// one workgroup per graph, one thread per float4 column; the node rows of a graph are read
// kPoolBatch at a time (all of a batch's loads issued before its adds, summed in node order: a
// 30-atom reaction is two round trips instead of eight)
constexpr int kPoolThreads = 128;
constexpr int kPoolBatch = 16;

__global__ __launch_bounds__(kPoolThreads) void k_pool_head(const float* __restrict__ hn, int Hp,
                                                            const int* __restrict__ gptr, int H,
                                                            const float* __restrict__ wf,
                                                            const float* __restrict__ bf,
                                                            float* __restrict__ g,
                                                            float* __restrict__ y,
                                                            const float* __restrict__ inv_cnt,
                                                            int* __restrict__ pool_arg,
                                                            bool pool_first) {
  const int b = blockIdx.x;
  const int v0 = gptr[b], v1 = gptr[b + 1];
  const int C4 = Hp >> 2;
  const float gs = inv_cnt ? inv_cnt[b] : 1.f;  // global_mean_pool: the sum / node count
  float dot = 0.f;
  for (int c = threadIdx.x; c < C4; c += kPoolThreads) {
    const float* col = hn + 4 * c;
    float4 s = f4zero();
    if (pool_arg) {  // global_max_pool: the largest value, its first node and its tie count
      float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      int arg[4] = {-1, -1, -1, -1}, cnt[4] = {0, 0, 0, 0};
      for (int v = v0; v < v1; ++v) {
        const float4 x = *reinterpret_cast<const float4*>(col + (int64_t)v * Hp);
        const float xv[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (xv[k] > m[k] || arg[k] < 0) {
            m[k] = xv[k];
            arg[k] = v;
            cnt[k] = 1;
          } else if (xv[k] == m[k]) {
            ++cnt[k];
          }
      }
      if (v1 <= v0) m[0] = m[1] = m[2] = m[3] = 0.f;  // (empty graph: 0, entry -1, never read)
      s = make_float4(m[0], m[1], m[2], m[3]);
      int rec[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)  // torch's amax backward also counts the zero `self` at a 0 max
        rec[k] = pool_first || arg[k] < 0 ? arg[k] : -(cnt[k] + (m[k] == 0.f ? 1 : 0));
      *reinterpret_cast<int4*>(pool_arg + (int64_t)b * Hp + 4 * c) =
          make_int4(rec[0], rec[1], rec[2], rec[3]);
    } else {
      for (int v = v0; v < v1; v += kPoolBatch) {
        float4 x[kPoolBatch];
#pragma unroll
        for (int u = 0; u < kPoolBatch; ++u)
          x[u] = v + u < v1 ? *reinterpret_cast<const float4*>(col + (int64_t)(v + u) * Hp)
                            : f4zero();
#pragma unroll
        for (int u = 0; u < kPoolBatch; ++u)
          if (v + u < v1) s = f4add(s, x[u]);
      }
    }
    if (inv_cnt) s = make_float4(s.x * gs, s.y * gs, s.z * gs, s.w * gs);
    *reinterpret_cast<float4*>(g + (int64_t)b * Hp + 4 * c) = s;
    const int n = 4 * c;
    const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (n + k < H) dot += sv[k] * wf[n + k];
  }
  __shared__ float red[kPoolThreads / 64];
  dot = wave_sum(dot);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dot;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = red[0];
#pragma unroll
    for (int k = 1; k < kPoolThreads / 64; ++k) t += red[k];
    y[b] = t + bf[0];
  }
}

hipError_t pool_head_fwd(const float* hn, int Hp, const int* gptr, int64_t B, int H,
                         const float* wf, const float* bf, float* g, float* y, hipStream_t st,
                         const float* inv_cnt, int* pool_arg, bool pool_first) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pool_head, dim3(B), dim3(kPoolThreads), 0, st, hn, Hp, gptr, H, wf, bf, g,
                     y, inv_cnt, pool_arg, pool_first);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// mean aggregation / mean pooling (PyG scatter mean: sum / max(count, 1))
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mean_scales(const int* __restrict__ dst_ptr, int64_t N,
                                                     const int* __restrict__ gptr, int64_t B,
                                                     float* __restrict__ inv_deg,
                                                     float* __restrict__ inv_cnt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (inv_deg && t < N) inv_deg[t] = 1.f / (float)max(dst_ptr[t + 1] - dst_ptr[t], 1);
  if (inv_cnt && t < B) inv_cnt[t] = 1.f / (float)max(gptr[t + 1] - gptr[t], 1);
}

hipError_t mean_scales(const int* dst_ptr, int64_t N, const int* gptr, int64_t B, float* inv_deg,
                       float* inv_cnt, hipStream_t st) {
  const int64_t n = std::max(inv_deg ? N : 0, inv_cnt ? B : 0);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mean_scales, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, dst_ptr, N,
                     gptr, B, inv_deg, inv_cnt);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_scale_rows(float* __restrict__ a, int Hp, int64_t N,
                                                    const float* __restrict__ s) {
  const int C4 = Hp >> 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * C4) return;
  const int64_t v = t / C4;
  float4* p = reinterpret_cast<float4*>(a) + t;
  const float4 x = *p;
  const float f = s[v];
  *p = make_float4(x.x * f, x.y * f, x.z * f, x.w * f);
}

hipError_t scale_rows(float* a, int Hp, int64_t N, const float* s, hipStream_t st) {
  const int64_t tot = N * (Hp >> 2);
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scale_rows, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, st, a, Hp, N, s);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// backward: ffn head + add-pool + edge_to_node activation
//   dwf[n] = sum_b dy[b] g[b, n] ; dbf = sum_b dy[b]            (k_head_bwd, column reduction)
//   dzn[v, n] = dy[graph(v)] * wf[n] * act'(zn[v, n])           (k_readout_bwd; dg never stored)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_head_bwd(const float* __restrict__ dy,
                                                   const float* __restrict__ g, int64_t B, int H,
                                                   int Hp, float* __restrict__ dwf,
                                                   float* __restrict__ dbf) {
  // block = 64 columns x 16 row phases
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + tx;
  float acc = 0.f, sdy = 0.f;
  for (int64_t b = ty; b < B; b += 16) {
    const float d = dy[b];
    if (n < H) acc += d * g[b * Hp + n];
    sdy += d;
  }
  __shared__ float red[16][65];
  red[ty][tx] = acc;
  __syncthreads();
  if (ty == 0) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    if (n < H) dwf[n] = s;
  }
  if (blockIdx.x == 0) {
    __syncthreads();
    red[ty][tx] = sdy;  // every tx of a row phase summed the same dy values
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red[k][0];
      dbf[0] = s;
    }
  }
}

hipError_t head_bwd(const float* dy, const float* g, const float* wf, int64_t B, int H, int Hp,
                    float* dg, float* dwf, float* dbf, hipStream_t st) {
  (void)wf;
  (void)dg;
  hipLaunchKernelGGL(k_head_bwd, dim3(cdiv(H, 64)), dim3(1024), 0, st, dy, g, B, H, Hp, dwf, dbf);
  return hipGetLastError();
}

// (k_readout_bwd_img, the dzn kernel, lives in b3_pack.hip: it writes the e-image too)

// ------------------------------------------------------------------------------------------
// backward: D-MPNN layer activation / skip / dropout (GNN.py:94-102 reversed)
// ------------------------------------------------------------------------------------------
// (the top layer's activation backward, k_layer_bwd_img, lives in b3_pack.hip: it writes the
// weight gradient's e-image of dpre as well)

// ------------------------------------------------------------------------------------------
// x rows padded to a multiple of 4 floats (F = 846 -> 848): every GEMM that reads x then issues
// 16-byte loads instead of 8-byte ones
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pad_rows(const float* __restrict__ x, int64_t N, int F,
                                                  float* __restrict__ xp, int ldp, int vec2) {
  const int c4n = ldp >> 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * c4n) return;
  pad_row4(x, F, xp, ldp, c4n, t, vec2 != 0);
}

hipError_t pad_rows(const float* x, int64_t N, int F, float* xp, int ldp, hipStream_t st) {
  const int64_t tot = N * (ldp >> 2);
  if (tot <= 0) return hipSuccess;
  const int vec2 = (F % 2 == 0) && ((uintptr_t)x & 7) == 0;
  hipLaunchKernelGGL(k_pad_rows, dim3(cdiv(tot, 256)), dim3(256), 0, st, x, N, F, xp, ldp, vec2);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// deterministic split-K reduction of weight-gradient slabs
// ------------------------------------------------------------------------------------------
// slab layout [splits][Nout][ldk], ldk = round_up(Kout, 4) (gemm_tn_kernel).  The output is
// small (a weight matrix) and the split dimension long (up to ~200), so a workgroup owns 32
// float4 outputs and spreads the splits over 8 thread groups (group g sums splits g, g + 8, ...
// in order), then combines the 8 partials in a fixed order through LDS: deterministic, and
// ~40k outputs still give >1000 workgroups.  The bias slabs [splits][Nout] ride along as extra
// float4-less columns in the last workgroups.
constexpr int kRedCols = 32, kRedGroups = 8;

// one logical block of one reduction job
__device__ __forceinline__ void reduce_slab_block(const RedJob& J, int blk, float4 (*part)[kRedCols],
                                                  float (*bpart)[kRedCols]) {
  const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
  const int ldk = (J.Kout + 3) & ~3;
  const int c4n = ldk >> 2;
  const int64_t nf = (int64_t)J.Nout * c4n;
  if (J.splits < kRedGroups) {
    // fewer splits than groups: the grouped form would idle kRedGroups - splits groups, so each
    // thread takes one float4 output (or bias element) and sums its splits in order
    reduce_slab_item(J, (int64_t)blk * (kRedCols * kRedGroups) + threadIdx.x);
    return;  // uniform over the block: no LDS used, the next logical block may follow at once
  }
  if (blk < J.main_blocks) {
    const int64_t f = (int64_t)blk * kRedCols + col;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (f < nf) {
      const float4* s4 = reinterpret_cast<const float4*>(J.slab) + f;
#pragma unroll 4
      for (int p = grp; p < J.splits; p += kRedGroups) {
        const float4 v = s4[(int64_t)p * nf];
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
    }
    part[grp][col] = s;
    __syncthreads();
    if (grp == 0 && f < nf) {
      float4 t = part[0][col];
#pragma unroll
      for (int g = 1; g < kRedGroups; ++g) {
        const float4 u = part[g][col];
        t.x += u.x;
        t.y += u.y;
        t.z += u.z;
        t.w += u.w;
      }
      const int64_t n = f / c4n;
      const int k = (int)(f - n * c4n) * 4;
      float* o = J.dst + n * J.ld_dst + J.col_off;
      const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kk = k + q;
        if (kk >= J.Kout || (kk >= J.gap_at && kk < J.gap_at + J.gap_len)) continue;
        o[kk >= J.gap_at + J.gap_len ? kk - J.gap_len : kk] = tv[q];
      }
    }
  } else {
    const int n = (blk - J.main_blocks) * kRedCols + col;
    float s = 0.f;
    if (n < J.Nout)
      for (int p = grp; p < J.splits; p += kRedGroups) s += J.bslab[(int64_t)p * J.Nout + n];
    bpart[grp][col] = s;
    __syncthreads();
    if (grp == 0 && n < J.Nout) {
      float t = bpart[0][col];
#pragma unroll
      for (int g = 1; g < kRedGroups; ++g) t += bpart[g][col];
      J.bias_dst[n] = t;
    }
  }
  __syncthreads();  // part / bpart reused by the next logical block
}

// several reductions in one launch (the backward batches every side-stream weight gradient):
// logical blocks are numbered job by job; the grid strides over all of them
__global__ __launch_bounds__(kRedCols * kRedGroups) void k_reduce_slabs(RedJobs jobs) {
  __shared__ float4 part[kRedGroups][kRedCols];
  __shared__ float bpart[kRedGroups][kRedCols];
  for (int blk = blockIdx.x; blk < jobs.total; blk += gridDim.x) {
    int j = 0, base = 0;
    while (j + 1 < jobs.n && blk >= base + jobs.j[j].nblk) base += jobs.j[j++].nblk;
    reduce_slab_block(jobs.j[j], blk - base, part, bpart);
  }
}

bool add_reduce_job(RedJobs& jobs, const float* slab, const float* bslab, int splits, int Nout,
                    int Kout, float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                    int gap_at, int gap_len) {
  const int64_t nf = (int64_t)Nout * (((Kout + 3) & ~3) >> 2);
  if (nf <= 0) return true;
  if (jobs.n >= kMaxRedJobs) return false;
  RedJob& J = jobs.j[jobs.n++];
  if (gap_len <= 0) gap_at = 0x7fffffff, gap_len = 0;
  J.slab = slab;
  J.bslab = bslab;
  J.dst = dst;
  J.bias_dst = bias_dst;
  J.ld_dst = ld_dst;
  J.col_off = col_off;
  J.splits = splits;
  J.Nout = Nout;
  J.Kout = Kout;
  J.gap_at = gap_at;
  J.gap_len = gap_len;
  red_job_set_splits(J, splits);
  jobs.total += J.nblk;
  return true;
}

void red_job_set_splits(RedJob& J, int splits) {
  J.splits = splits;
  const int64_t nf = (int64_t)J.Nout * (((J.Kout + 3) & ~3) >> 2);
  if (splits < kRedGroups) {  // flat logical blocks (reduce_slab_block)
    J.main_blocks = (int)cdiv(nf + (J.bias_dst ? J.Nout : 0), kRedCols * kRedGroups);
    J.nblk = J.main_blocks;
  } else {
    J.main_blocks = (int)cdiv(nf, kRedCols);
    J.nblk = J.main_blocks + (J.bias_dst ? (int)cdiv(J.Nout, kRedCols) : 0);
  }
}

hipError_t reduce_slabs_batched(const RedJobs& jobs, int max_blocks, hipStream_t st) {
  if (jobs.n <= 0 || jobs.total <= 0) return hipSuccess;
  const int grid = std::min(jobs.total, max_blocks);
  hipLaunchKernelGGL(k_reduce_slabs, dim3(grid), dim3(kRedCols * kRedGroups), 0, st, jobs);
  return hipGetLastError();
}

// One thread per float4 output (and per bias element): reduce_slab_item (reduce.hpp)
__global__ __launch_bounds__(256) void k_reduce_slabs_flat(RedJob J) {
  reduce_slab_item(J, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// flat form (one thread per output, every split in flight) for short split counts: the grouped
// form leaves 8 - splits thread groups idle.  For every side-stream reduction the flat form was
// serially faster (106 -> 97 us / step) but the step 3.5 % slower (A/B): it crowds the main chain.
constexpr int kReduceFlatMaxSplits = 8;

hipError_t reduce_slabs(const float* slab, const float* bslab, int splits, int Nout, int Kout,
                        float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                        hipStream_t st, int gap_at, int gap_len, bool flat) {
  RedJobs jobs{};
  if (flat || splits <= kReduceFlatMaxSplits) {
    if (!add_reduce_job(jobs, slab, bslab, splits, Nout, Kout, dst, ld_dst, col_off, bias_dst,
                        gap_at, gap_len) || jobs.n == 0)
      return hipSuccess;
    const RedJob& J = jobs.j[0];
    const int64_t nf = (int64_t)Nout * (((Kout + 3) & ~3) >> 2);
    const int64_t tot = nf + (bias_dst ? Nout : 0);
    hipLaunchKernelGGL(k_reduce_slabs_flat, dim3(cdiv(tot, 256)), dim3(256), 0, st, J);
    return hipGetLastError();
  }
  add_reduce_job(jobs, slab, bslab, splits, Nout, Kout, dst, ld_dst, col_off, bias_dst, gap_at,
                 gap_len);
  return reduce_slabs_batched(jobs, kReduceMaxBlocks, st);
}

__global__ __launch_bounds__(256) void k_reduce_partials(const float* __restrict__ part, int nb,
                                                         ScalarReduceJobs jobs) {
  const int j = blockIdx.x;
  float s = 0.f;
  for (int b = threadIdx.x; b < jobs.count[j]; b += blockDim.x) s += part[(int64_t)j * nb + b];
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) jobs.out[j][0] = (red[0] + red[1]) + (red[2] + red[3]);
}

hipError_t reduce_partials(const float* part, int nb, const ScalarReduceJobs& jobs,
                           hipStream_t st) {
  if (jobs.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_reduce_partials, dim3(jobs.n), dim3(256), 0, st, part, nb, jobs);
  return hipGetLastError();
}

}  // namespace cgr
