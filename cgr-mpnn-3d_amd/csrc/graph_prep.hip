// Graph bookkeeping for one collated batch (integer work, bit-exact vs oracle/dmpnn_numpy.py).
//
// Replaces the implicit index handling of the reference forward:
//   row, col = edge_index                      (GNN.py:85, GNN.py:132)
//   scatter_add(h, col, dim_size=max(col)+1)   (GNN.py:134 via PyG propagate)
//   flip(h.view(E/2, 2, H), [1])               (GNN.py:136-138, reverse edge = e ^ 1)
//   global_add_pool(h, batch)                  (GNN.py:110)
//
// Outputs (int32, sorted edge space = stable sort of edges by dst):
//   perm[i]      original edge id of sorted position i        (np.argsort(dst, kind=stable))
//   src_s, dst_s endpoints of sorted edge i
//   rev_s[i]     sorted position of the reverse edge perm[i]^1
//   dst_ptr[N+1] CSR offsets of sorted positions per destination node
//   src_ptr[N+1], src_list[E]  CSR of sorted positions per source node (stable by position)
//   graph_ptr[B+1], node_graph[N]  node ranges per reaction graph
//   status       bit0: edge index out of range, bit1: batch not sorted/out of range,
//                bit2: edges not reverse-paired (src(e ^ 1) != dst(e) for some e; informational:
//                the reference's flip pairs e with e ^ 1 whatever they hold, and so does rev_s,
//                but the backward's fused src sum takes its paired fast form only when clear)
//
// Determinism: the counting sort claims slots with atomics (arbitrary order inside a bucket) and
// then insertion-sorts every bucket by key, so the result is the unique stable order.  Buckets are
// atom in/out-degrees (<= ~10 for molecules), so the per-bucket sort is a few compares.
#include "common.hpp"
#include "gnn_internal.hpp"
#include "prep_one.hpp"

namespace cgr {

// Phase 1 (one launch): edge endpoints + degree counts [0, E), node -> graph ids [E, E+N),
// graph_ptr copy [E+N, E+N+B+1) when the caller has PyG's ptr; thread 0 also writes the dropout
// key of this forward (rng_key semantics, kernels.hip) when asked to.
__global__ void k_prep_count(const int64_t* __restrict__ ei, int E, int N, int B,
                             const int64_t* __restrict__ batch,
                             const int64_t* __restrict__ gptr64, int* __restrict__ deg_dst,
                             int* __restrict__ deg_src, int* __restrict__ src_c,
                             int* __restrict__ dst_c, int* __restrict__ graph_cnt,
                             int* __restrict__ node_graph, int* __restrict__ gptr,
                             int* __restrict__ status, int want_key, uint64_t seed,
                             uint64_t* __restrict__ counter, uint64_t* __restrict__ key_out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (want_key && t == 0) {
    uint64_t k = seed;
    if (counter) {
      const uint64_t c = counter[0];
      k = seed + 0xD1B54A32D192ED03ull * (c + 1);
      counter[0] = c + 1;
    }
    key_out[0] = k;
  }
  if (t < E) {
    const int e = t;
    int64_t s = ei[e], d = ei[(int64_t)E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) {
      atomicOr(status, 1);
      s = (s < 0 || s >= N) ? 0 : s;  // clamp so no kernel ever faults; status reports it
      d = (d < 0 || d >= N) ? 0 : d;
    }
    src_c[e] = (int)s;
    dst_c[e] = (int)d;
    atomicAdd(&deg_dst[d], 1);
    atomicAdd(&deg_src[s], 1);
  } else if (t < E + N) {
    const int v = t - E;
    int64_t g = batch ? batch[v] : 0;
    if (g < 0 || g >= B) {
      atomicOr(status, 2);
      g = g < 0 ? 0 : B - 1;
    }
    if (batch && v + 1 < N && batch[v + 1] < batch[v]) atomicOr(status, 2);
    node_graph[v] = (int)g;
    if (!gptr64) atomicAdd(&graph_cnt[g], 1);
  } else if (gptr64 && t < E + N + B + 1) {
    const int b = t - E - N;
    gptr[b] = (int)gptr64[b];
  }
}

// Exclusive scan of `n` ints into out[0..n] (out[n] = total).  One 1024-thread block per array
// (blockIdx.x picks the job): contiguous per-thread chunks, wave scans with shuffles, one LDS
// pass over the 16 wave totals.
struct ScanJob {
  const int* in;
  int* out;
  int n;
};
struct ScanJobs {
  ScanJob job[3];
};

__global__ __launch_bounds__(1024) void k_scan(ScanJobs jobs) {
  const ScanJob jb = jobs.job[blockIdx.x];
  if (jb.in == nullptr) return;
  __shared__ int wsum[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int chunk = (jb.n + 1023) / 1024;
  const int b = min(jb.n, t * chunk), e = min(jb.n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += jb.in[i];
  // inclusive wave scan of the chunk sums
  int x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (w == 0) {
    int v = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane < 16) wsum[lane] = v;  // inclusive over waves
  }
  __syncthreads();
  int run = (x - s) + (w ? wsum[w - 1] : 0);  // exclusive prefix of this thread's chunk
  for (int i = b; i < e; ++i) {
    jb.out[i] = run;
    run += jb.in[i];
  }
  if (t == 1023) jb.out[jb.n] = wsum[15];
}

// slot claim: tmp[ptr[key[j]] + k] = j  for j in [0, n)
__global__ void k_place(const int* __restrict__ key, int n, const int* __restrict__ ptr,
                        int* __restrict__ cursor, int* __restrict__ tmp) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int k = key[j];
  const int slot = atomicAdd(&cursor[k], 1);
  tmp[ptr[k] + slot] = j;
}

// per bucket insertion sort (ascending) -> stable order
__global__ void k_bucket_sort(const int* __restrict__ ptr, int nb, int* __restrict__ buf) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nb) return;
  insertion_sort(buf, ptr[v], ptr[v + 1]);
}

// dst buckets: sort (-> stable perm) and, for the bucket's own sorted positions, the inverse
// permutation and sorted endpoints (no cross-bucket dependency, so one pass)
__global__ void k_sort_inv(const int* __restrict__ dst_ptr, int N, int* __restrict__ perm,
                           const int* __restrict__ src_c, int* __restrict__ inv,
                           int* __restrict__ src_s, int* __restrict__ dst_s) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= N) return;
  const int b = dst_ptr[v], e = dst_ptr[v + 1];
  insertion_sort(perm, b, e);
  for (int i = b; i < e; ++i) {
    const int p = perm[i];
    inv[p] = i;
    src_s[i] = src_c[p];
    dst_s[i] = v;
  }
}

// rev_s, the sorted zero-padded edge_attr ([E, Fep]) and the src-CSR slot claim
__global__ void k_rev_place(const int* __restrict__ perm, const int* __restrict__ inv, int E,
                            int* __restrict__ rev_s, const float* __restrict__ ea, int Fe,
                            int Fep, float* __restrict__ e_s, const int* __restrict__ src_s,
                            const int* __restrict__ src_ptr, int* __restrict__ cursor2,
                            int* __restrict__ src_list, const int* __restrict__ src_c,
                            const int* __restrict__ dst_s, int* __restrict__ status) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E) return;
  const int p = perm[i];
  rev_s[i] = inv[p ^ 1];
  if (src_c[p ^ 1] != dst_s[i]) atomicOr(status, 4);
  if (Fep) {
    const float* src = ea + (int64_t)p * Fe;
    float* dst = e_s + (int64_t)i * Fep;
    for (int q = 0; q < Fep; ++q) dst[q] = q < Fe ? src[q] : 0.f;
  }
  const int k = src_s[i];
  const int slot = atomicAdd(&cursor2[k], 1);
  src_list[src_ptr[k] + slot] = i;
}

}  // namespace cgr

using namespace cgr;

int cgr_graph_prep_impl(const PrepArgs& a, hipStream_t st) {
  const int E = (int)a.E, N = (int)a.N, B = (int)a.B;
  IndexView iv = a.idx;
  // zero counters + status (one contiguous block, see arena layout)
  if (!a.zeroed) HIP_RET(hipMemsetAsync(iv.zero_block, 0, iv.zero_bytes, st));
  const int T = 256;
  const int nt = E + N + (a.graph_ptr ? B + 1 : 0);
  hipLaunchKernelGGL(k_prep_count, dim3(cdiv(nt > 0 ? nt : 1, T)), dim3(T), 0, st, a.edge_index,
                     E, N, B, a.batch, a.graph_ptr, iv.deg_dst, iv.deg_src, iv.src_c, iv.dst_c,
                     iv.graph_cnt, iv.node_graph, iv.graph_ptr, iv.status, a.want_key ? 1 : 0,
                     a.seed, a.rng_counter, iv.rng);
  ScanJobs sj{};
  sj.job[0] = ScanJob{iv.deg_dst, iv.dst_ptr, N};
  sj.job[1] = ScanJob{iv.deg_src, iv.src_ptr, N};
  sj.job[2] = a.graph_ptr ? ScanJob{nullptr, nullptr, 0} : ScanJob{iv.graph_cnt, iv.graph_ptr, B};
  hipLaunchKernelGGL(k_scan, dim3(3), dim3(1024), 0, st, sj);
  if (E > 0) {
    // dst counting sort of original edge ids -> perm (+ inverse and sorted endpoints)
    hipLaunchKernelGGL(k_place, dim3(cdiv(E, T)), dim3(T), 0, st, iv.dst_c, E, iv.dst_ptr,
                       iv.cursor, iv.perm);
    hipLaunchKernelGGL(k_sort_inv, dim3(cdiv(N, T)), dim3(T), 0, st, iv.dst_ptr, N, iv.perm,
                       iv.src_c, iv.inv, iv.src_s, iv.dst_s);
    // reverse map, sorted edge features, src CSR over sorted positions (stable by position)
    hipLaunchKernelGGL(k_rev_place, dim3(cdiv(E, T)), dim3(T), 0, st, iv.perm, iv.inv, E,
                       iv.rev_s, a.edge_attr, (int)a.Fe, (int)a.Fep, a.e_s, iv.src_s,
                       iv.src_ptr, iv.cursor2, iv.src_list, iv.src_c, iv.dst_s, iv.status);
    hipLaunchKernelGGL(k_bucket_sort, dim3(cdiv(N, T)), dim3(T), 0, st, iv.src_ptr, N,
                       iv.src_list);
  }
  HIP_RET(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------
// Generic pieces reused by the standalone DMPNNConv (caller's edge order).
// ------------------------------------------------------------------------------------------
namespace cgr {

__global__ void k_split_edges(const int64_t* __restrict__ ei, int E, int N, int* __restrict__ src_c,
                              int* __restrict__ dst_c) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  int64_t s = ei[e], d = ei[(int64_t)E + e];
  src_c[e] = (s < 0 || s >= N) ? 0 : (int)s;
  dst_c[e] = (d < 0 || d >= N) ? 0 : (int)d;
}

__global__ void k_count_keys(const int* __restrict__ key, int n, int* __restrict__ deg) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) atomicAdd(&deg[key[j]], 1);
}

int split_edges(const int64_t* ei, int E, int N, int* src_c, int* dst_c, hipStream_t st) {
  if (E > 0)
    hipLaunchKernelGGL(k_split_edges, dim3(cdiv(E, 256)), dim3(256), 0, st, ei, E, N, src_c, dst_c);
  HIP_RET(hipGetLastError());
  return 0;
}

// Stable CSR of positions j in [0, n) grouped by key[j] in [0, nb): ptr[nb+1], list[n].
// deg/cursor: caller-provided int[nb] scratch, zeroed here.
int csr_from_keys(const int* key, int n, int nb, int* deg, int* cursor, int* ptr, int* list,
                  hipStream_t st) {
  HIP_RET(hipMemsetAsync(deg, 0, sizeof(int) * nb, st));
  HIP_RET(hipMemsetAsync(cursor, 0, sizeof(int) * nb, st));
  if (n > 0)
    hipLaunchKernelGGL(k_count_keys, dim3(cdiv(n, 256)), dim3(256), 0, st, key, n, deg);
  ScanJobs sj{};
  sj.job[0] = ScanJob{deg, ptr, nb};
  sj.job[1] = ScanJob{nullptr, nullptr, 0};
  sj.job[2] = ScanJob{nullptr, nullptr, 0};
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, sj);
  if (n > 0) {
    hipLaunchKernelGGL(k_place, dim3(cdiv(n, 256)), dim3(256), 0, st, key, n, ptr, cursor, list);
    hipLaunchKernelGGL(k_bucket_sort, dim3(cdiv(nb, 256)), dim3(256), 0, st, ptr, nb, list);
  }
  HIP_RET(hipGetLastError());
  return 0;
}

}  // namespace cgr
