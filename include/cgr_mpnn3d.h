/*
 * cgr_mpnn3d.h - C ABI of the MI355X-native CGR-MPNN-3D D-MPNN hot path (libcgr_mpnn3d.so).
 *
 * The reference (tobjec/CGR-MPNN-3D @ 2025-02-27) is pure Python; its hot path is the
 * ``GNN`` / ``DMPNNConv`` pair in ``cgr_mpnn_3D/models/GNN.py`` plus two PyTorch-Geometric
 * sum-scatters.  Each entry point below replaces one of those interfaces (file:line cited) and is
 * bound from Python by ``cgr_mpnn_3D/_amd/native.py`` (ctypes), which keeps the reference's
 * ``nn.Module`` surface so ``train.py`` / ``test.py`` drop in unchanged.
 *
 * Conventions
 *   - plain pointers and sizes only; every pointer argument named d_* / listed as "device" is
 *     device memory on the current HIP device; `stream` is a hipStream_t passed as void*
 *     (NULL = legacy default stream).  Calls only enqueue work: no allocation, no host sync, so
 *     they can be captured into a hipGraph.
 *   - fp32 data, row-major; int64 graph indices exactly as PyG produces them.
 *   - parameters / gradients are passed as a table of device pointers in the reference
 *     ``state_dict`` order (see CGR_PARAM_*), each tensor contiguous in the reference layout
 *     (nn.Linear weight = [out, in]).
 *   - return 0 on success, a CGR_ERR_* code otherwise; cgr_last_error() describes the failure
 *     (thread-local).  Python raises RuntimeError with that text.
 */
#ifndef CGR_MPNN3D_H
#define CGR_MPNN3D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGR_ABI_VERSION 6
#define CGR_MAX_DEPTH 32

enum cgr_status {
  CGR_OK = 0,
  CGR_ERR_INVALID_ARGUMENT = 1,
  CGR_ERR_HIP = 2,
  CGR_ERR_UNSUPPORTED = 3,
};

/* activation_fn of GNN.__init__ (GNN.py:21, applied at GNN.py:86,127: any callable); train.py:284-292
 * offers F.relu / F.silu / F.gelu.  Codes 3-9 are further elementwise activations at torch's
 * default parameters (ELU alpha 1, leaky_relu slope 0.01, softplus beta 1 / threshold 20). */
enum cgr_activation {
  CGR_ACT_RELU = 0, CGR_ACT_SILU = 1, CGR_ACT_GELU = 2, CGR_ACT_TANH = 3, CGR_ACT_SIGMOID = 4,
  CGR_ACT_ELU = 5, CGR_ACT_LEAKY_RELU = 6, CGR_ACT_SOFTPLUS = 7, CGR_ACT_MISH = 8, CGR_ACT_SELU = 9
};

/* GNN.__init__(num_node_features, num_edge_features, depth, hidden_sizes, dropout_ps,
 *              activation_fn, aggr="add", pooling_fn=global_add_pool, use_learnable_skip)
 * (GNN.py:14-74).  The math of the reference requires one uniform hidden size (GNN.py:53-65). */
typedef struct cgr_gnn_config {
  int32_t num_node_features; /* F  (78 CGR + 768 MACE for CGR-MPNN-3D) */
  int32_t num_edge_features; /* Fe (14), may be 0 */
  int32_t hidden;            /* H  = hidden_sizes[i] for all i */
  int32_t depth;             /* D  (1 .. CGR_MAX_DEPTH) */
  int32_t activation;        /* enum cgr_activation */
  int32_t learnable_skip;    /* use_learnable_skip (GNN.py:71-74, :94-97) */
  int32_t aggregation;       /* enum cgr_aggregation: DMPNNConv(aggr=...) (GNN.py:22,63,119) */
  int32_t pooling;           /* enum cgr_pooling: pooling_fn (GNN.py:23,110) */
} cgr_gnn_config;

/* aggr of GNN.__init__ / DMPNNConv (PyG MessagePassing): "add" (= "sum", the default) or "mean"
 * (the sum over a node's in-edges divided by their count, 0 for a node without in-edges) */
enum cgr_aggregation { CGR_AGGR_ADD = 0, CGR_AGGR_MEAN = 1 };
/* pooling_fn: global_add_pool (default), global_mean_pool (the graph's node sum divided by its
 * node count) or global_max_pool (per column the largest node value; with a `batch` its gradient
 * is shared evenly by the nodes holding it, as torch's scatter_reduce("amax", include_self=False)
 * backward does -- the zero `self` counted when the max is 0; with batch == NULL, x.max(dim=-2),
 * it goes to the first node holding it) */
enum cgr_pooling { CGR_POOL_ADD = 0, CGR_POOL_MEAN = 1, CGR_POOL_MAX = 2 };

/* One collated batch, the fields GNN.forward reads from a PyG Batch (GNN.py:77-82). */
typedef struct cgr_batch {
  const float* x;            /* device [N, F]  data.x */
  const int64_t* edge_index; /* device [2, E]  data.edge_index (row 0 = src, row 1 = dst) */
  const float* edge_attr;    /* device [E, Fe] data.edge_attr (NULL allowed when Fe == 0) */
  const int64_t* batch;      /* device [N]     data.batch, sorted graph id per node; NULL = one
                                graph (global_add_pool(h, None), GNN.py:110) */
  const int64_t* graph_ptr;  /* device [B+1]   Batch.ptr node offsets, or NULL (derived from
                                `batch` on the device) */
  int64_t num_nodes;         /* N */
  int64_t num_edges;         /* E (even: reverse edge of e is e ^ 1, GNN.py:136-138) */
  int64_t num_graphs;        /* B (1 when batch == NULL) */
} cgr_batch;

/* Parameter table order = reference state_dict order (GNN.py:53-74):
 *   [0] edge_init.weight [H, F+Fe]   [1] edge_init.bias [H]
 *   [2+2l] convs.l.lin.weight [H, H] [3+2l] convs.l.lin.bias [H]          l = 0..D-1
 *   [2+2D] edge_to_node.weight [H, F+H]  [3+2D] edge_to_node.bias [H]
 *   [4+2D] ffn.weight [1, H]         [5+2D] ffn.bias [1]
 *   [6+2D+l] skip_weights.l []       (only when learnable_skip)                              */
#define CGR_PARAM_EDGE_INIT_W 0
#define CGR_PARAM_EDGE_INIT_B 1
#define CGR_PARAM_CONV_W(l) (2 + 2 * (l))
#define CGR_PARAM_CONV_B(l) (3 + 2 * (l))
#define CGR_PARAM_E2N_W(D) (2 + 2 * (D))
#define CGR_PARAM_E2N_B(D) (3 + 2 * (D))
#define CGR_PARAM_FFN_W(D) (4 + 2 * (D))
#define CGR_PARAM_FFN_B(D) (5 + 2 * (D))
#define CGR_PARAM_SKIP(D, l) (6 + 2 * (D) + (l))

int cgr_abi_version(void);
const char* cgr_last_error(void);

/* number of entries of the parameter / gradient tables for `cfg` */
int cgr_gnn_num_params(const cgr_gnn_config* cfg);

/* Bytes of the per-forward arena (index bookkeeping + activations saved for backward) and of the
 * backward scratch workspace.  The caller owns both (e.g. torch.empty(uint8) on the device). */
int64_t cgr_gnn_arena_bytes(const cgr_gnn_config* cfg, int64_t num_nodes, int64_t num_edges,
                            int64_t num_graphs);
int64_t cgr_gnn_workspace_bytes(const cgr_gnn_config* cfg, int64_t num_nodes, int64_t num_edges,
                                int64_t num_graphs);

/* Byte offset of a named arena buffer (introspection for tests/debugging).  "status" is the graph
 * prep's int32 status word: bit 0 an edge id outside [0, num_nodes), bit 1 an unsorted or
 * out-of-range batch vector, bit 2 edges not reverse-paired (src(e ^ 1) != dst(e) for some e;
 * informational: results stay exact, the backward takes its unpaired form), bit 4 (value 16) the
 * unpaired backward's completion timed out (see cgr_device_errors).  Names: "status", "rng",
 * "perm", "src_s", "dst_s", "rev_s", "src_list", "dst_ptr", "src_ptr", "graph_ptr",
 * "node_graph", "e_s", "P", "h", "a", "pre", "zn", "hn", "g"; `index` selects the layer for
 * "h" / "a" / "pre".  Returns -1 for an unknown or absent buffer. */
int64_t cgr_gnn_arena_offset(const cgr_gnn_config* cfg, int64_t num_nodes, int64_t num_edges,
                             int64_t num_graphs, const char* name, int32_t index);

/* Index bookkeeping only (also run by cgr_gnn_forward): stable dst-sorted edge order, reverse
 * edge map, src/dst CSR, graph node ranges.  Replaces the implicit index handling of
 * GNN.py:85,132-138 and PyG's scatter/pool indexing (GNN.py:110,134). */
int cgr_graph_prep(const cgr_gnn_config* cfg, const cgr_batch* batch, void* arena, void* stream);

/* GNN.forward(data) -> [B] (GNN.py:76-110): edge init, `depth` fused D-MPNN layers
 * (gather -> MFMA GEMM -> bias/skip/act/dropout epilogue -> segmented reduce), edge->node
 * readout, add-pool and ffn.  Dropout (GNN.py:100-102) is applied when `training` != 0 and
 * dropout_p[l] > 0, from a counter-based RNG keyed by `seed` and, when `rng_counter` (device
 * uint64, may be NULL) is given, by its value, which the forward then increments on the device:
 * a captured graph replays with a fresh mask each time (the key is kept in the arena for the
 * backward).  Fills `arena` with what cgr_gnn_backward needs.  `y` device [B].
 * `training` is a bit set (other bits are rejected): CGR_TRAIN_DROPOUT = train-mode dropout
 * (module.training); CGR_TRAIN_FOR_BACKWARD = a backward will follow (the forward then also packs
 * the backward GEMMs' weight images into the arena; cgr_gnn_backward refuses an arena whose
 * forward did not set it).  Pass the same value to cgr_gnn_backward. */
#define CGR_TRAIN_DROPOUT 1
#define CGR_TRAIN_FOR_BACKWARD 2
int cgr_gnn_forward(const cgr_gnn_config* cfg, const float* const* params,
                    const cgr_batch* batch, const float* dropout_p, uint64_t seed,
                    uint64_t* rng_counter, int32_t training, void* arena, float* y,
                    void* stream);

/* Reverse mode of cgr_gnn_forward (what autograd runs for the reference: GNN.py:76-145 under
 * loss.backward(), trainer.py:142-143).  `dy` device [B] = dLoss/dy; writes every parameter
 * gradient into the table `grads` (same order and shapes as `params`, overwritten, not
 * accumulated).  `arena` must come from the matching forward call; `workspace` is scratch.
 *
 * `bucket_events` (NULL, or CGR_GRAD_BUCKETS(depth) hipEvent_t handles passed as void*): event b
 * is recorded on a stream of the backward as soon as every gradient of bucket b is final, so a
 * data-parallel caller can start bucket b's all-reduce while the rest of the backward runs
 * (trainer.py:138-144 has one device).  Buckets, in the order they become ready:
 *   0            edge_to_node.{weight,bias}, ffn.{weight,bias}
 *   1 + k        convs.(depth-1-k).lin.{weight,bias}            k = 0 .. depth-1
 *   depth + 1    edge_init.{weight,bias}, skip_weights.* (end of the backward, caller's stream) */
#define CGR_GRAD_BUCKETS(depth) ((depth) + 2)
int cgr_gnn_backward(const cgr_gnn_config* cfg, const float* const* params,
                     const cgr_batch* batch, const float* dropout_p, uint64_t seed,
                     int32_t training, const void* arena, const float* dy, float* const* grads,
                     void* workspace, void* const* bucket_events, void* stream);

/* Gradients with respect to the inputs (what autograd gives the reference for x / edge_attr
 * tensors that require grad: x enters through x[row] in edge_init, GNN.py:85-86, and through
 * cat([x, s]) in edge_to_node, GNN.py:105-106; edge_attr through edge_init only).  Call after
 * cgr_gnn_backward, on the same stream, with the same config / params / batch / arena / dy and
 * the SAME workspace (it reads the edge-init pre-activation gradient that backward left there).
 * dx: device [num_nodes, num_node_features] (NULL: skipped); dedge_attr: device
 * [num_edges, num_edge_features] in the caller's edge order (NULL: skipped); both overwritten,
 * fp32, 16-byte aligned.  Fails (nothing enqueued) unless `workspace` holds a successful
 * cgr_gnn_backward of `arena`'s latest forward (host-side record, no device sync). */
int cgr_gnn_input_grads(const cgr_gnn_config* cfg, const float* const* params,
                        const cgr_batch* batch, const void* arena, const float* dy,
                        void* workspace, float* dx, float* dedge_attr, void* stream);

/* Forward-only inference (test.py:85-113 and cli_tool/activation_energy_predictor.py:70-80 run
 * GNN.forward under torch.no_grad() in eval mode).  cgr_gnn_predict computes exactly what
 * cgr_gnn_forward computes for `y`, but keeps no activation for a backward (h_1 .. h_D share a
 * two-buffer ring and a_0 .. a_D a three-buffer one: its arena is ~half the training arena).
 * `images` NULL: the split-bf16 forward weight images are packed from `params` into the arena by
 * this call (one launch beside the graph bookkeeping; always current, whatever changed the weights
 * -- an optimizer writing through raw pointers, a replayed captured step).  Non-NULL: images
 * pre-packed by cgr_gnn_pack_images (cgr_gnn_image_bytes bytes, caller-owned), which the caller
 * must re-pack whenever the parameters change.  `training` may only hold CGR_TRAIN_DROPOUT
 * (module in train mode under no_grad).  Sizes: cgr_gnn_predict_arena_bytes. */
int64_t cgr_gnn_image_bytes(const cgr_gnn_config* cfg);
int cgr_gnn_pack_images(const cgr_gnn_config* cfg, const float* const* params, void* images,
                        void* stream);
int64_t cgr_gnn_predict_arena_bytes(const cgr_gnn_config* cfg, int64_t num_nodes,
                                    int64_t num_edges, int64_t num_graphs);
int cgr_gnn_predict(const cgr_gnn_config* cfg, const float* const* params,
                    const cgr_batch* batch, const float* dropout_p, uint64_t seed,
                    uint64_t* rng_counter, int32_t training, const void* images, void* arena,
                    float* y, void* stream);

/* Sticky device-side conditions of `device` (no reference counterpart: the reference's autograd
 * cannot fail this way), read from pinned host memory the kernels write -- no device sync, so a
 * caller can poll it at every step.  A condition becomes visible once the kernel that raised it
 * has run.  Bits (cleared when `clear` != 0):
 *   CGR_DEVERR_UNPAIRED_TIMEOUT  a completer of the unpaired-edge backward (edges not
 *       reverse-paired, status bit 2) gave up waiting for the rest of its launch; the gradients
 *       of that backward are NaN-poisoned, never partial.  An error.
 *   CGR_DEVERR_UNPAIRED_SEEN  a backward ran the unpaired form (slower; informational).
 * Returns 0 before the device's first cgr_gnn_forward / _backward. */
#define CGR_DEVERR_UNPAIRED_SEEN 4
#define CGR_DEVERR_UNPAIRED_TIMEOUT 16
int32_t cgr_device_errors(int32_t device, int32_t clear);

/* Segmented sum, the sum-scatter primitive of the path (PyG propagate aggr="add", GNN.py:134;
 * global_add_pool, GNN.py:110) over a CSR: out[s, :] = sum_{j in [seg_ptr[s], seg_ptr[s+1])}
 * values[index ? index[j] : j, :].  width = row length in floats; ld_* = row strides (floats).
 * Deterministic (fixed summation order, no atomics). */
int cgr_segment_sum(const float* values, int64_t ld_values, const int32_t* index,
                    const int32_t* seg_ptr, int64_t num_segments, int64_t width, float* out,
                    int64_t ld_out, void* stream);

/* DMPNNConv.forward(edge_index, edge_attr) -> (a, h') (GNN.py:131-141), in the caller's edge
 * order: a[v] = sum_{dst(e)=v} h[e] (dim_size = N; aggregation CGR_AGGR_MEAN: divided by
 * max(in-degree, 1)), h'[e] = (a[src(e)] - h[e^1]) W^T + b.
 * `scratch` needs cgr_dmpnn_conv_scratch_bytes(N, E, H). */
int64_t cgr_dmpnn_conv_scratch_bytes(int64_t num_nodes, int64_t num_edges, int64_t hidden);
int cgr_dmpnn_conv_forward(const int64_t* edge_index, int64_t num_nodes, int64_t num_edges,
                           const float* h, int64_t hidden, const float* weight, const float* bias,
                           float* a_out, float* h_out, void* scratch, int32_t aggregation,
                           void* stream);
/* Reverse mode of cgr_dmpnn_conv_forward given dL/da (may be NULL) and dL/dh' (may be NULL):
 * writes dL/dh [E,H], dL/dW [H,H], dL/db [H].  `scratch` must hold the forward's bookkeeping
 * (same scratch buffer, untouched since the forward) plus cgr_dmpnn_conv_scratch_bytes. */
int cgr_dmpnn_conv_backward(const int64_t* edge_index, int64_t num_nodes, int64_t num_edges,
                            const float* h, int64_t hidden, const float* weight,
                            const float* grad_a, const float* grad_h_out, float* grad_h,
                            float* grad_weight, float* grad_bias, void* scratch,
                            int32_t aggregation, void* stream);

/* torch.optim.Adam(params, lr, betas, eps, weight_decay, amsgrad) step (train.py:117-119), fused
 * over every parameter tensor in one launch (+ one tiny launch for the step counter) instead of
 * the ~11 multi-tensor launches of torch's foreach path.  Per element, in the rounding order of
 * torch/optim/adam.py _multi_tensor_adam (hyper-parameters as Python doubles):
 *   g = grad (+ weight_decay * p);  m += (1 - b1) (g - m);  v = b2 v + (1 - b2) g^2;
 *   vmax = max(vmax, v) (amsgrad);  p -= lr / (1 - b1^t) * m / (sqrt(vmax or v) / sqrt(1 - b2^t) + eps)
 * with t = *step + 1 written back to *step: a per-tensor device float, like torch's state["step"]
 * (capturable=True), so a captured graph replays with the right bias corrections.  grad == NULL
 * skips a tensor and leaves its step (p.grad is None).  max_exp_avg_sq may be NULL when
 * amsgrad == 0.  Any number of tensors (launched in groups of CGR_ADAM_GROUP). */
#define CGR_ADAM_GROUP 32
typedef struct cgr_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  float* max_exp_avg_sq;
  float* step; /* device scalar */
  int64_t numel;
} cgr_adam_tensor;
int cgr_adam_step(const cgr_adam_tensor* tensors, int32_t num_tensors, double lr, double beta1,
                  double beta2, double eps, double weight_decay, int32_t amsgrad,
                  int32_t maximize, void* stream);

/* On-device collation (replaces torch_geometric.loader.DataLoader / Batch.from_data_list in
 * trainer.py:105-118 over the per-reaction Data of ChemDataset.py:81-94).  The store holds every
 * graph of a dataset collated once on the device: graph g owns node rows [node_ptr[g],
 * node_ptr[g+1]) of x [*, F] and edges [edge_ptr[g], edge_ptr[g+1]) of edge_index [2,
 * num_edges_all] (global node ids) / edge_attr [*, Fe]; y [G] may be NULL.  For graph_ids[0..B)
 * (device) it writes exactly what Batch.from_data_list would: x_out [sum nodes, F], edge_index_out
 * [2, num_edges_out] re-based to the running node count, edge_attr_out, batch_out [sum nodes]
 * (= position in graph_ids), ptr_out [B+1], y_out [B].  The caller sizes the outputs (the counts
 * are known on the host from its copy of node_ptr / edge_ptr).  Bit-exact; one launch. */
int cgr_collate(const int64_t* graph_ids, int64_t num_ids, const int64_t* node_ptr,
                const int64_t* edge_ptr, const float* x, int64_t num_node_features,
                const int64_t* edge_index, int64_t num_edges_all, const float* edge_attr,
                int64_t num_edge_features, const float* y, float* x_out, int64_t* edge_index_out,
                int64_t num_edges_out, float* edge_attr_out, int64_t* batch_out, int64_t* ptr_out,
                float* y_out, void* stream);

/* Training loss (replaces torch.nn.MSELoss(reduction="sum") of train.py:120 as trainer.py:142-143
 * applies it; reduction_mean != 0 is MSELoss(reduction="mean")).  input, target: device [n] fp32.
 * forward: *loss (device scalar) = sum (input - target)^2 (/ n).  backward: grad_input =
 * 2 (input - target) grad_loss[0] (/ n), grad_target = -grad_input; either output may be NULL.
 * One launch each, deterministic. */
int cgr_mse_loss_forward(const float* input, const float* target, int64_t n,
                         int32_t reduction_mean, float* loss, void* stream);
int cgr_mse_loss_backward(const float* input, const float* target, const float* grad_loss,
                          int64_t n, int32_t reduction_mean, float* grad_input,
                          float* grad_target, void* stream);

/* Instrumentation (no reference counterpart): per-kernel-class device time measured with HIP
 * events recorded on the launch stream around every launch of cgr_gnn_forward/_backward.
 * Off by default; do not enable while capturing a graph.  cgr_profile_collect() waits for the
 * recorded events; cgr_profile_report() writes "name count total_ms" lines and returns the
 * buffer size needed. */
int cgr_profile_enable(int32_t on);
int cgr_profile_collect(void);
void cgr_profile_reset(void);
int64_t cgr_profile_report(char* buf, int64_t len);

/* Diagnostic builds only (-DCGR_STAMPS, tools/stamp_lab.py): every split-bf16 NT GEMM workgroup
 * appends one 16 x uint64 record of shader-clock phase stamps to `buffer` (device, zeroed by the
 * caller; its first 16 bytes are the record counter) for at most `records` workgroups; NULL stops
 * recording.  The product build returns CGR_ERR_UNSUPPORTED. */
int cgr_debug_stamps(void* buffer, int64_t records);

/* Process diagnostics (no reference counterpart): on != 0 installs a SIGABRT handler that prints
 * the aborting thread's id, name and native backtrace to stderr, then passes the signal to the
 * handler installed before it (e.g. Python's faulthandler) or the default action; 0 restores
 * that handler.  Used by the multi-process / RCCL tests and the distributed bench, so an abort in
 * a runtime thread without Python frames still names its origin. */
int cgr_debug_abort_backtrace(int32_t on);

#ifdef __cplusplus
}
#endif

#endif /* CGR_MPNN3D_H */
