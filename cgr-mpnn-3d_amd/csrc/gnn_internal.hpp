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
  // zero block (memset each call): deg_dst, deg_src, cursor, cursor2, graph_cnt, status
  int* deg_dst;
  int* deg_src;
  int* cursor;
  int* cursor2;
  int* graph_cnt;
  int* status;
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

// 1: every NT GEMM (x-GEMM, layer and readout, forward and backward) runs on the bf16 matrix
// cores with three-piece split operands (gemm_b3.hpp); the forward packs the weight images once
// per step.  0: exact fp32 MFMA kernels (gemm.hpp / gemm_rs.hpp).
#ifndef CGR_B3
#define CGR_B3 1
#endif

// Forward-saved float state inside the arena.
struct FloatView {
  float* e_s;   // [E, Fep] sorted, zero padded edge_attr
  float* w0eT;  // [Fe, Hp] transposed edge-feature slice of edge_init.weight
  float* P;     // [N, Hp]  x @ W0[:, :F]^T (node-level half of edge init)
  float* Q;     // [N, Hp]  x @ W_n[:, :F]^T (x-part of the readout, computed beside graph prep)
  float* xp;    // [N, Fp]  x with rows padded to 4 floats (only when F % 4 != 0; else nullptr)
  float* wT;    // [D+1, H, Hp] W_l^T (l < D) and W_n[:, F:]^T for the backward's NT GEMMs, built
                // by the forward on its side stream (weights do not change between the two)
  float* h[CGR_MAX_DEPTH + 1];    // [E, Hp] h_0 .. h_D
  float* a[CGR_MAX_DEPTH + 1];    // [N, Hp] a_l = scatter_add(h_l, dst); a_D = readout s
  float* pre[CGR_MAX_DEPTH + 1];  // [E, Hp] pre-activations (non-ReLU only; else nullptr)
  float* zn;                      // [N, Hp] readout pre-activation (non-ReLU only)
  float* hn;                      // [N, Hp] readout activation
  float* g;                       // [B, Hp] pooled graph embeddings
  // split-bf16 weight images (CGR_B3; gemm_b3.hpp), packed by the forward's side stream:
  void* b3x;                      // [W0[:, :F]; W_n[:, :F]]   (x-GEMM)
  void* b3rof;                    // W_n[:, F:]                 (readout forward)
  void* b3rob;                    // W_n[:, F:]^T               (readout backward)
  void* b3lf[CGR_MAX_DEPTH];      // W_l                        (layer forward)
  void* b3lb[CGR_MAX_DEPTH];      // W_l^T                      (layer backward)
  // the layer messages m_l = a_l[src] - h_l[rev] as bf16 hi / lo planes [round_up(E, 32)][mld]
  // (written by the layer forward when the backward will run; gemm_b3tp.hpp's B operand)
  uint16_t* mhi[CGR_MAX_DEPTH];
  uint16_t* mlo[CGR_MAX_DEPTH];
  int64_t mld;
  // ReLU only (CGR_HBITS): the backward's activation masks h_l > 0 as [E, Hp/4] bytes, bit k of
  // byte (i, c) = h_l[i, 4c + k] > 0, written beside h_l by its producer (edge init / layer
  // epilogue); the backward reads 1/32 of the bytes of h_l for them.  nullptr: read h_l.
  uint8_t* hb[CGR_MAX_DEPTH + 1];
};

struct Dims {
  int64_t N, E, B;
  int F, Fe, Fep, Fp, H, Hp, D;  // Fp = round_up(F, 4)
  int act;
  int learnable_skip;
};

struct ArenaLayout {
  size_t off_index_begin;
  size_t bytes;
  // offsets (bytes) for every buffer
  size_t zero_block, zero_bytes, deg_dst, deg_src, cursor, cursor2, graph_cnt, status, rng;
  size_t perm, src_s, dst_s, rev_s, src_list, inv, src_c, dst_c, dst_ptr, src_ptr, graph_ptr,
      node_graph;
  size_t e_s, w0eT, P, Q, xp, wT, h[CGR_MAX_DEPTH + 1], a[CGR_MAX_DEPTH + 1], pre[CGR_MAX_DEPTH + 1], zn, hn,
      g;
  size_t b3x, b3rof, b3rob, b3lf[CGR_MAX_DEPTH], b3lb[CGR_MAX_DEPTH];
  size_t mhi[CGR_MAX_DEPTH], mlo[CGR_MAX_DEPTH];
  size_t hb[CGR_MAX_DEPTH + 1];
};

// 1: every side-stream weight gradient gets its own split-K slab and all of them are reduced in
// one batched launch at the end of the side stream; 0: one shared slab, reduced after each GEMM.
// Same-box A/B: batched 1.44 ms/step vs 1.34 ms (256 / 4096 blocks no better), so 0.
#ifndef CGR_BATCH_REDUCE
#define CGR_BATCH_REDUCE 0
#endif
#ifndef CGR_BATCH_REDUCE_BLOCKS
#define CGR_BATCH_REDUCE_BLOCKS 1024
#endif
#ifndef CGR_B3TP
#define CGR_B3TP 0  // layer weight gradients from bf16 operand planes the producers write
                    // (gemm_b3tp.hpp; lab 38 vs 50 us, but A/B -2.5 %: in the step the plane TN
                    // runs no faster beside the main chain and the plane writes slow the layer
                    // forward and the activation backward)
#endif
#ifndef CGR_DH0_DEFER
#define CGR_DH0_DEFER 0  // 1: the skip gradient dh0 = sum_l sigma_l dpre_l is summed once by the
                         // edge-init backward from the per-layer dpre buffers (the layer kernels
                         // no longer read + write dh0: 2 x E x H x 4 B each); needs CGR_DPRE_RING 0.
                         // A/B neutral: the layer kernels gain 8 us each, the edge-init backward on
                         // the critical tail loses 28 us reading D buffers (r02 trace)
#endif
#ifndef CGR_DPRE_RING
#define CGR_DPRE_RING (CGR_DH0_DEFER ? 0 : 1)  // 1: two dpre buffers reused across layers (the layer-l+1 weight gradient
                         // must finish reading before the segmented sum of layer l overwrites:
                         // one side->main wait per layer); 0: one buffer per layer, no such wait:
                         // A/B 1.28 -> 1.35 ms (the graph maps the freed main-stream nodes onto
                         // the side stream's queue)
#endif
static_assert(!(CGR_DH0_DEFER && CGR_DPRE_RING), "deferred dh0 needs one dpre buffer per layer");
struct WorkspaceLayout {
  size_t bytes;
  size_t dpre[CGR_MAX_DEPTH], dm, dh0, dzn, ds, Gs, dg, slab, bslab, slab2, bslab2, dsig_part,
      slab_elems, bslab_elems;
  size_t dphi[CGR_MAX_DEPTH], dplo[CGR_MAX_DEPTH];  // dpre bf16 planes (same ring as dpre)
  int dsig_blocks;
};

Dims make_dims(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B);
ArenaLayout arena_layout(const Dims& d);
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
};

}  // namespace cgr

int cgr_graph_prep_impl(const cgr::PrepArgs& a, hipStream_t st);
