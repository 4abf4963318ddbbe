// Internal (non-ABI) declarations: arena layout, index views, launch helpers.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/cgr_mpnn3d.h"

namespace cgr {

void set_error(const std::string& msg);

#define HIP_RET(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      ::cgr::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + __FILE__ + \
                       ":" + std::to_string(__LINE__));                                       \
      return CGR_ERR_HIP;                                                                     \
    }                                                                                         \
  } while (0)

#define CGR_CHECK(cond, msg)           \
  do {                                 \
    if (!(cond)) {                     \
      ::cgr::set_error(msg);           \
      return CGR_ERR_INVALID_ARGUMENT; \
    }                                  \
  } while (0)

constexpr size_t kAlign = 256;

// Every launching entry point starts with this: hipGetLastError() is per thread and sticky, so an
// error left by an unrelated earlier HIP call (e.g. a caller's aborted stream capture) would
// otherwise be reported by our first post-launch check as if our launch had failed.
inline void clear_stale_hip_error() { (void)hipGetLastError(); }

// Index bookkeeping inside the arena (all int32).
struct IndexView {
  // zero block (zeroed each forward: a rider of the pack launch, or a memset with caller images):
  // deg_dst, deg_src, cursor, cursor2, graph_cnt, status, fcnt
  int* deg_dst;
  int* deg_src;
  int* cursor;
  int* cursor2;
  int* graph_cnt;
  int* status;
  int* fcnt;     // [N * column tiles] hub-segment tickets of the layer GEMMs (in the zero block)
  float* fpart;  // [tiles, 2, BN] hub-segment partial sums of the layer GEMMs
  uint64_t* rng;  // effective dropout key of this forward (read by every dropout kernel)
  void* zero_block;
  size_t zero_bytes;
  int* perm;
  int* src_s;
  int* dst_s;
  int* rev_s;
  int* src_list;
  int* inv;
  int* src_c;
  int* dst_c;
  int* dst_ptr;
  int* src_ptr;
  int* graph_ptr;
  int* node_graph;
};

// Forward-saved float state inside the arena.
struct FloatView {
  float* e_s;   // [E, Fep] sorted, zero padded edge_attr
  float* w0eT;  // [Fe, Hp] transposed edge-feature slice of edge_init.weight
  float* P;     // [N, Hp]  x @ W0[:, :F]^T (node-level half of edge init)
  float* Q;     // [N, Hp]  x @ W_n[:, :F]^T (x-part of the readout, computed beside graph prep)
  float* xp;    // [N, Fp]  x with rows padded to 4 floats (only when F % 4 != 0; else nullptr)
  float* h[CGR_MAX_DEPTH + 1];    // [E, Hp] h_0 .. h_D
  float* a[CGR_MAX_DEPTH + 1];    // [N, Hp] a_l = scatter_add(h_l, dst); a_D = readout s
  float* pre[CGR_MAX_DEPTH + 1];  // [E, Hp] pre-activations (non-ReLU only; else nullptr)
  float* zn;                      // [N, Hp] readout pre-activation (non-ReLU only)
  float* hn;                      // [N, Hp] readout activation
  float* g;                       // [B, Hp] pooled graph embeddings
  float* inv_deg;  // [N] 1 / max(in-degree, 1)   (mean aggregation; else nullptr)
  float* inv_cnt;  // [B] 1 / max(graph nodes, 1) (mean pooling; else nullptr)
  int* pool_arg;   // [B, Hp] max pooling's first arg-max node per column (else nullptr)
  // split-bf16 weight images (gemm_b3.hpp), packed once per step by the forward:
  void* b3x;                      // [W0[:, :F]; W_n[:, :F]]   (x-GEMM)
  void* b3rof;                    // W_n[:, F:]                 (readout forward)
  void* b3rob;                    // W_n[:, F:]^T diag(wf)      (readout backward)
  void* b3lf[CGR_MAX_DEPTH];      // W_l                        (layer forward)
  void* b3lb[CGR_MAX_DEPTH];      // W_l^T                      (layer backward)
};

struct Dims {
  int64_t N, E, B;
  int F, Fe, Fep, Fp, H, Hp, D;  // Fp = round_up(F, 4)
  int act;
  int learnable_skip;
  int aggr, pool;  // enum cgr_aggregation / cgr_pooling
};

struct ArenaLayout {
  size_t off_index_begin;
  size_t bytes;
  // offsets (bytes) for every buffer
  size_t zero_block, zero_bytes, deg_dst, deg_src, cursor, cursor2, graph_cnt, status, rng;
  size_t fcnt, fpart;
  size_t perm, src_s, dst_s, rev_s, src_list, inv, src_c, dst_c, dst_ptr, src_ptr, graph_ptr,
      node_graph;
  size_t e_s, w0eT, P, Q, xp, h[CGR_MAX_DEPTH + 1], a[CGR_MAX_DEPTH + 1],
      pre[CGR_MAX_DEPTH + 1], zn, hn, g;
  size_t inv_deg, inv_cnt;  // mean aggregation / pooling: 1 / max(count, 1) per node / graph
  size_t pool_arg;          // max pooling: [B, Hp] node of each pooled value (-1: empty graph)
  size_t b3x, b3rof, b3rob, b3lf[CGR_MAX_DEPTH], b3lb[CGR_MAX_DEPTH];
};

// Backward workspace.  dpre has one buffer per layer (no side->main wait before a buffer is
// rewritten; the edge-init backward sums dh0 from all of them); dm holds only the rows the fused
// layer-backward GEMM hands to the completer of a tile-crossing segment (ep_bwd.hpp).
struct WorkspaceLayout {
  size_t bytes;
  size_t dpre, dm, dh0, dzn, ds, Gs, slab, bslab, slab2, bslab2, dsig_part, slab_elems,
      bslab_elems;
  size_t slab_b, bslab_b;  // the side stream's second slab pair (reductions folded into TNs)
  // split-bf16 e-images (gemm_b3.hpp B3EImg) of the weight gradients' shared operand: dpre_l and
  // dzn on the side stream (one at a time), Gs on the caller's stream; the top layer's dpre,
  // written by its activation kernel on the caller's stream (img_top)
  size_t img_side, img_main, img_top;
  // 2 x [N, Hp] partial da sums of the dst segments that cross a row tile of the fused
  // layer-backward GEMM (ep_bwd.hpp), alternating by layer
  size_t dag;
  // [N * column tiles + 1] ticket counters of those segments (and of the grid, unpaired form)
  size_t cnt;
  // [row tiles * column tiles, 2, BN] partial sums of the segments over >= 3 row tiles
  size_t part;
  // [F, input_grad_ldw(H)] the stacked, transposed x slices of edge_init / edge_to_node weights
  // (cgr_gnn_input_grads only)
  size_t wxT;
  int dsig_blocks;
};
inline int input_grad_ldw(int H) { return (2 * H + 3) & ~3; }
int bwd_dsig_slots(const Dims& d);
int bwd_seg_tiles(const Dims& d);
struct B3Cols;
B3Cols layer_cols(const Dims& d);  // column tiling of the layer GEMMs (capi.hip)

// Forward variants.  Training (cgr_gnn_forward): every activation the backward reads is saved in
// the arena and the weight images are packed into it by each call.  Eval (cgr_gnn_predict): no
// saved activations -- h_1.. h_D alias a two-buffer ring and a_0 .. a_D a three-buffer ring (the
// fused layer epilogue zeroes the entries it accumulates two layers ahead, gnn_fwd.hip) -- and
// the forward weight images are packed into its arena by every call (the weights may have changed
// by any route: an optimizer writing through raw pointers, a replayed captured step), unless the
// caller hands pre-packed ones (cgr_gnn_pack_images) and vouches for their freshness.
struct FwdMode {
  bool eval = false;
  const void* images = nullptr;
};
struct ImageLayout {
  size_t b3x, b3rof, b3lf[CGR_MAX_DEPTH], bytes;
};
ImageLayout image_layout(const Dims& d);

Dims make_dims(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B);
ArenaLayout arena_layout(const Dims& d);
ArenaLayout eval_arena_layout(const Dims& d);
WorkspaceLayout workspace_layout(const Dims& d);
IndexView index_view(void* arena, const ArenaLayout& L);
FloatView float_view(void* arena, const ArenaLayout& L, const Dims& d);

struct PrepArgs {
  const int64_t* edge_index;
  const int64_t* batch;      // may be null (one graph)
  const int64_t* graph_ptr;  // may be null (derive from batch)
  const float* edge_attr;
  int64_t N, E, B;
  int64_t Fe, Fep;
  IndexView idx;
  float* e_s;
  // dropout key (folded into the first prep kernel): written to idx.rng when want_key
  bool want_key = false;
  uint64_t seed = 0;
  uint64_t* rng_counter = nullptr;
  // idx.zero_block already zeroed on this stream (a pack launch's rider, gnn_fwd.hip)
  bool zeroed = false;
};

}  // namespace cgr

int cgr_graph_prep_impl(const cgr::PrepArgs& a, hipStream_t st);
