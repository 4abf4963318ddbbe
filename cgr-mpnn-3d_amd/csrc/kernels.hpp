// Host wrappers of the non-GEMM kernels (kernels.hip).  All enqueue on `st`, no sync.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cgr_mpnn3d.h"  // CGR_MAX_DEPTH

namespace cgr {

// out[s, :w] = sum_{j in [ptr[s], ptr[s+1])} vals[idx ? idx[j] : j, :w]
hipError_t segment_sum(const float* vals, int64_t ldv, const int* idx, const int* ptr,
                       int64_t nseg, int64_t width, float* out, int64_t ldo, hipStream_t st);

struct TransposeJob {
  const float* src;  // [rows, ld_src], columns [col_off, col_off + cols)
  int64_t ld_src;
  int64_t col_off;
  float* dst;  // [cols, ld_dst]
  int64_t ld_dst;
  int rows, cols;
};
constexpr int kMaxTransposeJobs = 40;
struct TransposeJobs {
  TransposeJob job[kMaxTransposeJobs];
  int n;
};
hipError_t transpose_batch(const TransposeJobs& jobs, hipStream_t st);

// h0 = act(P[src_s] + e_s @ W0e^T + b0) ; pre0 stored if non-null
// edge init + a_0 = segsum_dst(h0) in one pass (Hp <= 512); hipErrorInvalidValue otherwise.
// `zero` (may be null): the rows of a_1 .. a_n the layer GEMMs' segmented-sum epilogue
// (EpLayerSeg, row tiles of tile_rows) does not store -- nodes without in-edges and nodes whose
// in-edges cross a tile boundary (accumulated atomically) -- are zeroed here.
struct SegZero {
  float* a[32];
  int n;
  int tile_rows;
};
hipError_t edge_init_segsum_fwd(const float* P, const int* src_s, const float* e_s, int Fe,
                                int Fep, const float* w0eT, const float* b0, const int* dst_ptr,
                                int64_t N, int H, int Hp, int act, float* h0, float* pre0,
                                float* a, hipStream_t st, const SegZero* zero = nullptr);
hipError_t edge_init_fwd(const float* P, const int* src_s, const float* e_s, int Fe, int Fep,
                         const float* w0eT, const float* b0, int64_t E, int H, int Hp, int act,
                         float* h0, float* pre0, hipStream_t st);

// g[b] = sum_{v in graph b} hn[v] (* inv_cnt[b]: mean pooling, nullable; pool_arg non-null:
// max pooling, per column the max into g and into pool_arg [B, Hp] what its gradient needs:
// pool_first (batch=None: PyG's x.max(dim=-2), torch.max's first index) the first arg-max node,
// else (scatter_reduce "amax", include_self=False) -count, count = the nodes holding the max plus
// one when the max is 0 (the zero `self` torch's backward also counts));  y[b] = g[b].wf + bf
hipError_t pool_head_fwd(const float* hn, int Hp, const int* gptr, int64_t B, int H,
                         const float* wf, const float* bf, float* g, float* y, hipStream_t st,
                         const float* inv_cnt = nullptr, int* pool_arg = nullptr,
                         bool pool_first = false);

// mean aggregation / pooling factors: inv_deg[v] = 1 / max(in-degree, 1) from the dst CSR,
// inv_cnt[b] = 1 / max(nodes of graph b, 1) (either nullable: not computed)
hipError_t mean_scales(const int* dst_ptr, int64_t N, const int* gptr, int64_t B, float* inv_deg,
                       float* inv_cnt, hipStream_t st);
// a[v, :Hp] *= s[v]  (a summed aggregate -> the mean, in place)
hipError_t scale_rows(float* a, int Hp, int64_t N, const float* s, hipStream_t st);

// dwf = sum_b dy[b] g[b] ; dbf = sum_b dy[b]   (dg is folded into readout_act_bwd)
hipError_t head_bwd(const float* dy, const float* g, const float* wf, int64_t B, int H, int Hp,
                    float* dg, float* dwf, float* dbf, hipStream_t st);

// dzn[v] = dy[graph(v)] * wf * act'(zn[v])   (ReLU: hn > 0)
// dzn (may be null: not materialised) and/or its e-image `img` (gemm_b3.hpp B3EImg; null: none)
// gscale (nullable): per-graph factor of dy (mean pooling: inv_cnt); pool_arg (nullable): max
// pooling (pool_head_fwd's record): dzn[v, n] kept only where v is the column's first arg-max node
// (entry >= 0) or, for an entry -count, where hn[v, n] equals the pooled g[graph(v), n], divided
// by count (torch's scatter_reduce amax backward: ties share the gradient)
hipError_t readout_act_bwd(const float* dy, const float* wf, const int* node_graph,
                           const float* hn, const float* zn, int64_t N, int H, int Hp, int act,
                           float* dzn, void* img, hipStream_t st, const float* gscale = nullptr,
                           const int* pool_arg = nullptr, const float* gpool = nullptr);

struct LayerBwdArgs {
  // dh_{l+1}: top layer (l == D-1, layer_act_bwd): ds[dst_s[i]]; below (the fused dm GEMM,
  // ep_bwd.hpp): da[dst(i)] - dm[rev_s[i]], da = segsum_src(dm)
  const float* ds;
  const float* dm;
  const int* dst_s;
  const int* rev_s;
  const float* hnext;  // h_{l+1} (ReLU mask)
  const float* pre;    // pre_{l} (non-ReLU)
  const float* h0;
  const float* sigma;  // skip weight (nullptr -> 1)
  const uint64_t* seed;  // device dropout key (arena "rng")
  uint32_t thresh;
  float scale;
  int layer;
  int act;
  int64_t E;
  int H, Hp;
  float* dpre;
  float* dh0;         // edge init: dpre0 (written in place of dh0, the buffer it names)
  float* dsig_part;   // [gridDim] partial sums of dpre*h0 (nullable)
  // edge init: dh0 = sum_l sigma_l dpre_l over the layers' dpre buffers (dpre_l at
  // dpre_all + l * dpre_stride), summed l = D-1 .. 0; sig[l] nullptr -> 1
  const float* dpre_all;
  int64_t dpre_stride;
  int nlayers;
  const float* sig[CGR_MAX_DEPTH];
  // top layer (layer_act_bwd): the entries of dag and of the ticket counters cnt
  // ([cnt_nodes * cnt_tiles + CGR_MAX_DEPTH]: segment tickets, then the unpaired form's grid
  // counter of each fused launch) the fused layer-backward GEMMs use (nodes whose dst segment
  // crosses a tile_rows row-tile boundary, ep_bwd.hpp) are zeroed (nullable)
  float* dag;
  int* cnt;
  int64_t cnt_nodes;
  int tile_rows, cnt_tiles;
};
// nblocks: grid size if larger than needed (the learnable-skip partial slots to fill), else 0
// img (nullable): the e-image of dpre for the layer's weight-gradient TN, written beside it
hipError_t layer_act_bwd(const LayerBwdArgs& a, int nblocks, void* img, hipStream_t st);
int layer_act_bwd_blocks(int64_t E, int Hp);
// dst[n, col_off + k] = sum_s slab[s, n, k] ; bias_dst[n] = sum_s bslab[s, n]
// gap_len > 0: slab columns [gap_at, gap_at + gap_len) are padding and skipped; later columns
// shift down by gap_len in dst (the x | s concat of the readout with x padded to 4 floats)
// batched split-K slab reductions (one launch for several weight gradients)
constexpr int kMaxRedJobs = 40;
struct RedJob {
  const float* slab;
  const float* bslab;
  float* dst;
  float* bias_dst;
  int64_t ld_dst, col_off;
  int splits, Nout, Kout, gap_at, gap_len, main_blocks, nblk;
};
struct RedJobs {
  RedJob j[kMaxRedJobs];
  int n, total;
};
bool add_reduce_job(RedJobs& jobs, const float* slab, const float* bslab, int splits, int Nout,
                    int Kout, float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                    int gap_at = 0, int gap_len = 0);
// set a job's split count and size its logical blocks for it (jobs made before their TN plan)
void red_job_set_splits(RedJob& J, int splits);
// grouped form grid (A/B: beats 64 and unbounded 4096 by 4-8 %)
constexpr int kReduceMaxBlocks = 256;
hipError_t reduce_slabs_batched(const RedJobs& jobs, int max_blocks, hipStream_t st);
// flat: one thread per output with every split's load in flight (the critical-path tail) instead
// of the bounded-grid grouped form that shares the GPU with the other stream
hipError_t reduce_slabs(const float* slab, const float* bslab, int splits, int Nout, int Kout,
                        float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                        hipStream_t st, int gap_at = 0, int gap_len = 0, bool flat = false);

// xp[N, ldp] = x[N, F] with zero padding columns [F, ldp) (16-byte rows for the GEMM loaders)
hipError_t pad_rows(const float* x, int64_t N, int F, float* xp, int ldp, hipStream_t st);

// out[j][0] = sum_{b < count[j]} part[j * nb + b]   for j < njobs (scalar grads of skip weights)
// (the first count[j] of the nb slots of job j)
struct ScalarReduceJobs {
  float* out[64];
  int count[64];
  int n;
};
hipError_t reduce_partials(const float* part, int nb, const ScalarReduceJobs& jobs,
                           hipStream_t st);

}  // namespace cgr
