// Graph bookkeeping of one collated batch in ONE workgroup (graph_prep.hip's six launches as six
// phases of one block, counters in LDS): the extra, last workgroup of the x-GEMM launch
// (epilogues.hpp EpSplit2, gemm_b3.hpp kSideBlock), so that at small batches the bookkeeping
// runs beside the x-GEMM on its own CU with no second queue and no cross-queue join.  Same
// outputs, bit for bit, as cgr_graph_prep_impl (graph_prep.hip; oracle/dmpnn_numpy.py): the
// counting sorts claim slots with LDS atomics in arbitrary order and every bucket is then
// insertion-sorted, so the stable order is unique.
#pragma once

#include "common.hpp"

namespace cgr {

__device__ __forceinline__ void insertion_sort(int* __restrict__ buf, int b, int e) {
  for (int i = b + 1; i < e; ++i) {
    const int x = buf[i];
    int j = i - 1;
    while (j >= b && buf[j] > x) {
      buf[j + 1] = buf[j];
      --j;
    }
    buf[j + 1] = x;
  }
}

struct PrepOne {
  const int64_t* ei;      // [2, E]
  const int64_t* batch;   // [N] or null (one graph)
  const int64_t* gptr64;  // [B + 1] or null (derived from batch)
  const float* ea;        // [E, Fe]
  int E, N, B, Fe, Fep;
  int *src_c, *dst_c, *perm, *inv, *src_s, *dst_s, *rev_s, *src_list;
  int *dst_ptr, *src_ptr, *graph_ptr, *node_graph, *status;
  float* e_s;
  int want_key;
  uint64_t seed;
  uint64_t* counter;
  uint64_t* key_out;
};

// LDS ints the block needs (see graph_prep_one's layout)
__host__ __device__ inline int64_t prep_one_lds_ints(int64_t N, int64_t E, int64_t B) {
  return (N + 1) + (E > N + 1 ? E : N + 1) + (B + 1) + 1 + 16;
}
// Where one workgroup is the faster form: its phases cost a few us each beside the running
// x-GEMM and its stores go through one CU, so it pays only while the batch is small (same-box
// A/B, profiles/r04_c_prep_one_ab.txt: train.py's default batch, 1,920 edges, x-GEMM + side
// 27 us and the step +4..9 %; cfg2, 15,360 edges, 129 us and the step -8 %).  The packed
// dst-sorted entries (edge << 16 | src) need E < 32768 and N < 65536 anyway.
constexpr int64_t kPrepOneMaxEdges = 4096;
__host__ __device__ inline bool prep_one_fits(int64_t N, int64_t E, int64_t Fep) {
  return E <= kPrepOneMaxEdges && N < 65536 && Fep <= 16;
}
// items per thread with their loads in flight together (a round trip costs several us beside a
// running GEMM): index phases, and the feature-row phase
constexpr int kPrepU = 16, kPrepUR = 8;

// exclusive scan of c[0, n) in place (c[n] = total) by the whole block, also written to out[]
__device__ __forceinline__ void prep_one_scan(int* c, int n, int* out, int* wsum) {
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, w = t >> 6, nw = nt >> 6;
  const int chunk = (n + nt - 1) / nt;
  const int b = min(n, t * chunk), e = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += c[i];
  int x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    int v = lane < nw ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane < nw) wsum[lane] = v;  // inclusive over waves
  }
  __syncthreads();
  int run = (x - s) + (w ? wsum[w - 1] : 0);
  for (int i = b; i < e; ++i) {
    const int k = c[i];
    c[i] = run;
    out[i] = run;
    run += k;
  }
  if (t == nt - 1) {
    c[n] = wsum[nw - 1];
    out[n] = wsum[nw - 1];
  }
  __syncthreads();
}

// The whole bookkeeping by one block (blockDim.x a multiple of 64, <= 1024; E even, as the
// forward requires).  LDS (prep_one_lds_ints), R = max(E, N + 1):
//   [0, N + 1)          in-degrees -> dst CSR offsets -> dst cursors (phases 1-4)
//   [N + 1, N + 1 + R)  out-degrees -> src CSR offsets (1-2); the dst-sorted edges packed as
//                       edge << 16 | src (3-4); from phase 5 on [R, R + N + 1) holds the src
//                       cursors and [0, E) the src lists (5-7)
//   then B + 1 graph counts, the status bits and 16 per-wave scan totals.
__device__ __forceinline__ void graph_prep_one(const PrepOne& a, int* lds) {
  const int t = threadIdx.x, nt = blockDim.x;
  const int E = a.E, N = a.N, B = a.B;
  const int R = E > N + 1 ? E : N + 1;
  int* ldst = lds;
  int* lr = lds + N + 1;
  int* lg = lr + R;
  int* lstat = lg + B + 1;
  int* wsum = lstat + 1;
  int* lcur = lds + R;  // phase 5 on
  int* lsl = lds;       // phase 5 on
  for (int i = t; i < (int)prep_one_lds_ints(N, E, B); i += nt) lds[i] = 0;
  if (a.want_key && t == 0) {  // rng_key semantics (kernels.hip), as k_prep_count
    uint64_t k = a.seed;
    if (a.counter) {
      const uint64_t c = a.counter[0];
      k = a.seed + 0xD1B54A32D192ED03ull * (c + 1);
      a.counter[0] = c + 1;
    }
    a.key_out[0] = k;
  }
  __syncthreads();
  // phase 1: endpoints (clamped: status bit 1), degrees, and the pairing check of the reverse
  // edge (status bit 4: src(e ^ 1) != dst(e), k_rev_place's test): e ^ 1 sits in lane t ^ 1
  for (int e0 = t; e0 < E; e0 += nt * kPrepU) {
    int64_t s64[kPrepU], d64[kPrepU];
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int e = e0 + u * nt;
      s64[u] = e < E ? a.ei[e] : 0;
      d64[u] = e < E ? a.ei[(int64_t)E + e] : 0;
    }
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int e = e0 + u * nt;
      const int64_t s = s64[u], d = d64[u];
      const bool bad = s < 0 || s >= N || d < 0 || d >= N;
      const int si = (s < 0 || s >= N) ? 0 : (int)s, di = (d < 0 || d >= N) ? 0 : (int)d;
      const int sr = __shfl_xor(si, 1, 64);  // e and e ^ 1 are both < E or both >= E (E even)
      if (e < E) {
        if (bad) atomicOr(lstat, 1);
        if (sr != di) atomicOr(lstat, 4);
        a.src_c[e] = si;
        a.dst_c[e] = di;
        atomicAdd(&ldst[di], 1);
        atomicAdd(&lr[si], 1);
      }
    }
  }
  // node -> graph (status bit 2: out of range or batch not sorted)
  for (int v0 = t; v0 < N; v0 += nt * kPrepU) {
    int64_t g64[kPrepU], gn[kPrepU];
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int v = v0 + u * nt;
      g64[u] = (a.batch && v < N) ? a.batch[v] : 0;
      gn[u] = (a.batch && v + 1 < N) ? a.batch[v + 1] : INT64_MAX;  // no successor: never smaller
    }
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int v = v0 + u * nt;
      if (v < N) {
        int64_t g = g64[u];
        if (g < 0 || g >= B) {
          atomicOr(lstat, 2);
          g = g < 0 ? 0 : B - 1;
        }
        if (gn[u] < g64[u]) atomicOr(lstat, 2);
        a.node_graph[v] = (int)g;
        if (!a.gptr64) atomicAdd(&lg[g], 1);
      }
    }
  }
  if (a.gptr64)
    for (int b = t; b <= B; b += nt) a.graph_ptr[b] = (int)a.gptr64[b];
  __syncthreads();
  // phase 2: CSR offsets
  prep_one_scan(ldst, N, a.dst_ptr, wsum);
  prep_one_scan(lr, N, a.src_ptr, wsum);
  if (!a.gptr64) prep_one_scan(lg, B, a.graph_ptr, wsum);
  // phase 3: dst counting sort of the edges, slots claimed in arbitrary order (this thread's own
  // phase-1 stores read back)
  for (int e0 = t; e0 < E; e0 += nt * kPrepU) {
    int sv[kPrepU], dv[kPrepU];
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int e = e0 + u * nt;
      sv[u] = e < E ? a.src_c[e] : 0;
      dv[u] = e < E ? a.dst_c[e] : 0;
    }
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const int e = e0 + u * nt;
      if (e < E) lr[atomicAdd(&ldst[dv[u]], 1)] = (e << 16) | sv[u];
    }
  }
  __syncthreads();
  // phase 4: per dst bucket: stable order (by edge id, the high half), then the permutation, its
  // inverse and the sorted endpoints
  for (int v = t; v < N; v += nt) {
    const int b = v ? ldst[v - 1] : 0, e = ldst[v];
    insertion_sort(lr, b, e);
    for (int i = b; i < e; ++i) {
      const int x = lr[i], p = x >> 16;
      a.perm[i] = p;
      a.inv[p] = i;
      a.src_s[i] = x & 0xffff;
      a.dst_s[i] = v;
    }
  }
  __syncthreads();
  for (int v = t; v <= N; v += nt) lcur[v] = a.src_ptr[v];
  __syncthreads();
  // phase 5: per edge p (original order): rev_s[inv[p]] = inv[p ^ 1] (lane t ^ 1), its sorted
  // feature row (8-byte loads when Fe is even), and its src-list slot (claimed in arbitrary order)
  const bool fe2 = !(a.Fe & 1) && !((uintptr_t)a.ea & 7);
  for (int p0 = t; p0 < E; p0 += nt * kPrepUR) {
    int iv[kPrepUR], sv[kPrepUR];
    float f[kPrepUR][16];
#pragma unroll
    for (int u = 0; u < kPrepUR; ++u) {
      const int p = p0 + u * nt;
      iv[u] = p < E ? a.inv[p] : 0;
      sv[u] = p < E ? a.src_c[p] : 0;
      const float* row = a.ea + (int64_t)p * a.Fe;
      if (fe2) {
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const float2 v2 = (p < E && q < a.Fe) ? *reinterpret_cast<const float2*>(row + q)
                                                : make_float2(0.f, 0.f);
          f[u][q] = v2.x;
          f[u][q + 1] = v2.y;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) f[u][q] = (p < E && q < a.Fe) ? row[q] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < kPrepUR; ++u) {
      const int p = p0 + u * nt;
      const int ir = __shfl_xor(iv[u], 1, 64);
      if (p < E) {
        const int i = iv[u];
        a.rev_s[i] = ir;
        float* dst = a.e_s + (int64_t)i * a.Fep;
#pragma unroll
        for (int q = 0; q < 16; q += 4)
          if (q < a.Fep)
            *reinterpret_cast<float4*>(dst + q) =
                make_float4(f[u][q], f[u][q + 1], f[u][q + 2], f[u][q + 3]);
        lsl[atomicAdd(&lcur[sv[u]], 1)] = i;
      }
    }
  }
  __syncthreads();
  // phase 6: per src bucket: stable order (ascending sorted position)
  for (int v = t; v < N; v += nt) insertion_sort(lsl, v ? lcur[v - 1] : 0, lcur[v]);
  __syncthreads();
  // phase 7: the src lists out, coalesced
  for (int i = t; i < E; i += nt) a.src_list[i] = lsl[i];
  if (t == 0 && lstat[0]) atomicOr(a.status, lstat[0]);
}

}  // namespace cgr
