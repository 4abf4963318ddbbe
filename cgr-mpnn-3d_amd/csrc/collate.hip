// On-device collation of a batch of reaction graphs from a device-resident graph store
// (replaces torch_geometric.loader.DataLoader / Batch.from_data_list as
// used by trainer.py:105-118 over the per-reaction Data of ChemDataset.py:81-94).
//
// The store is every graph of the dataset collated once (PyG layout): node rows of graph g are
// [node_ptr[g], node_ptr[g+1]) of x, its edges [edge_ptr[g], edge_ptr[g+1]) of edge_index /
// edge_attr with GLOBAL node ids.  Collating graph ids gid[0..B) gives exactly what
// Batch.from_data_list produces for those graphs in that order: node blocks concatenated, edge
// ids re-based to the running node count, batch[v] = position b, ptr = node offsets, y gathered.
//
// kCollateSlices workgroups per output graph: each sums the node / edge counts of the graphs
// before it (a block reduction over gid[0..b), O(B) reads -- no separate scan launch), then
// copies its slice of the graph's node rows (one contiguous block of x) and edge rows as 8-byte
// or 4-byte words, re-bases its edge ids, fills batch; slice 0 writes ptr and y.  Pure data
// movement: HBM-bound, bit-exact.
#include "gnn_internal.hpp"

namespace cgr {

constexpr int kCollateThreads = 256;
constexpr int kCollateSlices = 4;  // 4 workgroups per graph: ~1000 for a 256-graph batch

__device__ __forceinline__ int64_t block_sum_i64(int64_t v, int64_t* red) {
  // 256 threads = 4 waves
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const int64_t t = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return t;
}

// contiguous copy of n floats, src/dst offsets in floats; 8-byte words when both are 8-byte
// aligned, else 4-byte words
__device__ __forceinline__ void copy_floats(const float* __restrict__ src, float* __restrict__ dst,
                                            int64_t n, int slice) {
  // slice `slice` of kCollateSlices equal parts (even-sized, so 8-byte alignment is kept)
  const int64_t part = ((n + kCollateSlices - 1) / kCollateSlices + 1) & ~int64_t(1);
  const int64_t lo = min(n, part * slice);
  src += lo;
  dst += lo;
  n = min(n, lo + part) - lo;
  const bool al8 = (((uintptr_t)src | (uintptr_t)dst) & 7) == 0;
  if (al8) {
    const int64_t n2 = n >> 1;
    const float2* s2 = reinterpret_cast<const float2*>(src);
    float2* d2 = reinterpret_cast<float2*>(dst);
    int64_t i = threadIdx.x;
    for (; i + 3 * kCollateThreads < n2; i += 4 * kCollateThreads) {  // 4 loads in flight
      const float2 a = s2[i], b = s2[i + kCollateThreads], c = s2[i + 2 * kCollateThreads],
                   d = s2[i + 3 * kCollateThreads];
      d2[i] = a;
      d2[i + kCollateThreads] = b;
      d2[i + 2 * kCollateThreads] = c;
      d2[i + 3 * kCollateThreads] = d;
    }
    for (; i < n2; i += kCollateThreads) d2[i] = s2[i];
    if ((n & 1) && threadIdx.x == 0) dst[n - 1] = src[n - 1];
  } else {
    for (int64_t i = threadIdx.x; i < n; i += kCollateThreads) dst[i] = src[i];
  }
}

__global__ __launch_bounds__(kCollateThreads) void k_collate(
    const int64_t* __restrict__ gid, int64_t B, const int64_t* __restrict__ node_ptr,
    const int64_t* __restrict__ edge_ptr, const float* __restrict__ x, int64_t F,
    const int64_t* __restrict__ ei, int64_t E_all, const float* __restrict__ ea, int64_t Fe,
    const float* __restrict__ y, float* __restrict__ x_out, int64_t* __restrict__ ei_out,
    int64_t E_out, float* __restrict__ ea_out, int64_t* __restrict__ batch_out,
    int64_t* __restrict__ ptr_out, float* __restrict__ y_out) {
  __shared__ int64_t red[4];
  const int64_t b = blockIdx.x / kCollateSlices;
  const int slice = (int)(blockIdx.x % kCollateSlices);
  // offsets of this graph in the output = counts of the graphs before it
  int64_t pn = 0, pe = 0;
  for (int64_t i = threadIdx.x; i < b; i += kCollateThreads) {
    const int64_t g = gid[i];
    pn += node_ptr[g + 1] - node_ptr[g];
    pe += edge_ptr[g + 1] - edge_ptr[g];
  }
  const int64_t on = block_sum_i64(pn, red);
  const int64_t oe = block_sum_i64(pe, red);
  const int64_t g = gid[b];
  const int64_t n0 = node_ptr[g], nn = node_ptr[g + 1] - n0;
  const int64_t e0 = edge_ptr[g], ne = edge_ptr[g + 1] - e0;
  if (threadIdx.x == 0 && slice == 0) {
    ptr_out[b] = on;
    if (b == B - 1) ptr_out[B] = on + nn;
    if (y) y_out[b] = y[g];
  }
  copy_floats(x + n0 * F, x_out + on * F, nn * F, slice);
  if (Fe > 0) copy_floats(ea + e0 * Fe, ea_out + oe * Fe, ne * Fe, slice);
  const int t = slice * kCollateThreads + threadIdx.x, T = kCollateSlices * kCollateThreads;
  for (int64_t v = t; v < nn; v += T) batch_out[on + v] = b;
  const int64_t shift = on - n0;
  for (int64_t e = t; e < ne; e += T) {
    ei_out[oe + e] = ei[e0 + e] + shift;
    ei_out[E_out + oe + e] = ei[E_all + e0 + e] + shift;
  }
}

}  // namespace cgr

using namespace cgr;

extern "C" int cgr_collate(const int64_t* graph_ids, int64_t num_ids, const int64_t* node_ptr,
                           const int64_t* edge_ptr, const float* x, int64_t num_node_features,
                           const int64_t* edge_index, int64_t num_edges_all,
                           const float* edge_attr, int64_t num_edge_features, const float* y,
                           float* x_out, int64_t* edge_index_out, int64_t num_edges_out,
                           float* edge_attr_out, int64_t* batch_out, int64_t* ptr_out,
                           float* y_out, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(num_ids >= 0, "cgr_collate: negative batch size");
  if (num_ids == 0) return 0;
  CGR_CHECK(graph_ids && node_ptr && edge_ptr && x && edge_index && x_out && edge_index_out &&
                batch_out && ptr_out,
            "cgr_collate: NULL pointer");
  CGR_CHECK(num_edge_features == 0 || (edge_attr && edge_attr_out),
            "cgr_collate: edge_attr pointers missing");
  CGR_CHECK(!y || y_out, "cgr_collate: y_out missing");
  CGR_CHECK(num_node_features >= 0 && num_edge_features >= 0 && num_edges_all >= 0 &&
                num_edges_out >= 0,
            "cgr_collate: bad sizes");
  CGR_CHECK(num_ids < (1LL << 28), "cgr_collate: too many graphs");
  hipLaunchKernelGGL(k_collate, dim3((unsigned)(num_ids * kCollateSlices)), dim3(kCollateThreads), 0,
                     (hipStream_t)stream, graph_ids, num_ids, node_ptr, edge_ptr, x,
                     num_node_features, edge_index, num_edges_all, edge_attr, num_edge_features,
                     y, x_out, edge_index_out, num_edges_out, edge_attr_out, batch_out, ptr_out,
                     y_out);
  HIP_RET(hipGetLastError());
  return 0;
}
