// C ABI of libcgr_mpnn3d.so (include/cgr_mpnn3d.h): validation, arena/workspace layout, error
// reporting.  No entry point allocates or synchronises; all work is enqueued on `stream`.
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>

#include "dispatch.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"
#include "streams.hpp"

namespace cgr {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// `training` bits of the forward that last filled each arena (host side, so the check costs no
// device sync and holds under graph capture): the backward needs the W^T images that only a
// CGR_TRAIN_FOR_BACKWARD forward packs.  Keys are arena addresses; the caching allocator reuses
// them, so the table stays as small as the set of live arena blocks.
static std::mutex g_arena_mu;
static std::unordered_map<const void*, int> g_arena_flags;
// every forward into an arena starts a new generation of it; a backward enqueued on (arena,
// generation) records its workspace, and cgr_gnn_input_grads -- which reads dpre0 and the
// readout's operands from that workspace -- requires the record to name the same arena at its
// current generation (otherwise it silently returned garbage)
static std::unordered_map<const void*, uint64_t> g_arena_gen;
static std::unordered_map<const void*, std::pair<const void*, uint64_t>> g_ws_backward;
static void note_forward(const void* arena, int flags) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  g_arena_flags[arena] = flags;
  ++g_arena_gen[arena];
}
static int forward_flags(const void* arena) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  const auto it = g_arena_flags.find(arena);
  return it == g_arena_flags.end() ? -1 : it->second;
}
static void note_backward(const void* arena, const void* workspace) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  g_ws_backward[workspace] = {arena, g_arena_gen[arena]};
}
static bool backward_matches(const void* arena, const void* workspace) {
  std::lock_guard<std::mutex> lk(g_arena_mu);
  const auto it = g_ws_backward.find(workspace);
  if (it == g_ws_backward.end() || it->second.first != arena) return false;
  const auto g = g_arena_gen.find(arena);
  return g != g_arena_gen.end() && g->second == it->second.second;
}

int gnn_forward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, uint64_t* rng_counter, int training,
                     void* arena, float* y, hipStream_t st, const FwdMode& mode);
hipError_t pack_forward_images(const Dims& d, const float* const* params, const ImageLayout& IL,
                               void* images, hipStream_t st);
int gnn_backward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                      const float* dropout_p, uint64_t seed, int training, const void* arena,
                      const float* dy, float* const* grads, void* workspace,
                      hipEvent_t const* bucket_events, hipStream_t st);
int gnn_input_grads_impl(const Dims& d, const float* const* params, const void* arena,
                         const float* dy, void* workspace, float* dx, float* de, hipStream_t st);

Dims make_dims(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B) {
  Dims d;
  d.N = N;
  d.E = E;
  d.B = B;
  d.F = cfg->num_node_features;
  d.Fe = cfg->num_edge_features;
  d.Fep = (int)round_up(d.Fe, 4);
  d.Fp = (int)round_up(d.F, 4);
  d.H = cfg->hidden;
  d.Hp = (int)round_up(d.H, 4);
  d.D = cfg->depth;
  d.act = cfg->activation;
  d.learnable_skip = cfg->learnable_skip ? 1 : 0;
  d.aggr = cfg->aggregation;
  d.pool = cfg->pooling;
  return d;
}

int bwd_seg_tiles(const Dims& d);

namespace {
struct Bump {
  size_t off = 0;
  size_t take(size_t bytes) {
    const size_t o = off;
    off = (size_t)round_up((int64_t)(off + bytes), (int64_t)kAlign);
    return o;
  }
};
constexpr size_t kNone = (size_t)-1;
}  // namespace

// index bookkeeping, sorted edge features and the x-GEMM outputs: shared by both layouts
static void layout_prefix(const Dims& d, ArenaLayout& L, Bump& b) {
  const size_t N = (size_t)d.N, E = (size_t)d.E, B = (size_t)d.B, Hp = (size_t)d.Hp;
  // zero block: six int arrays back to back, padded to a multiple of 16 bytes
  L.zero_block = b.off;
  L.deg_dst = b.off;
  L.deg_src = L.deg_dst + 4 * N;
  L.cursor = L.deg_src + 4 * N;
  L.cursor2 = L.cursor + 4 * N;
  L.graph_cnt = L.cursor2 + 4 * N;
  L.status = L.graph_cnt + 4 * B;
  // + the ticket counters of the layer GEMMs' hub segments (EpLayerSeg: zero on entry, reset by
  // each completer)
  L.fcnt = L.status + 16;
  // the layer forward runs in layer_cols(d), or in b3_cols(H) over caller-packed images (predict)
  const B3Cols lc = layer_cols(d), dc = b3_cols(d.H);
  const size_t fcnt_n = N * (size_t)std::max(lc.tiles, dc.tiles);
  L.zero_bytes = (size_t)round_up((int64_t)(4 * (4 * N + B) + 16 + 4 * fcnt_n), 16);
  b.take(L.zero_bytes);
  L.rng = b.take(8);
  L.perm = b.take(4 * E);
  L.src_s = b.take(4 * E);
  L.dst_s = b.take(4 * E);
  L.rev_s = b.take(4 * E);
  L.src_list = b.take(4 * E);
  L.inv = b.take(4 * E);
  L.src_c = b.take(4 * E);
  L.dst_c = b.take(4 * E);
  L.dst_ptr = b.take(4 * (N + 1));
  L.src_ptr = b.take(4 * (N + 1));
  L.graph_ptr = b.take(4 * (B + 1));
  L.node_graph = b.take(4 * N);
  L.e_s = d.Fep ? b.take(4 * E * (size_t)d.Fep) : kNone;
  L.w0eT = d.Fe ? b.take(4 * (size_t)d.Fe * Hp) : kNone;
  L.P = b.take(4 * N * Hp);
  L.Q = b.take(4 * N * Hp);
  L.xp = (d.F % 4 != 0) ? b.take(4 * N * (size_t)d.Fp) : kNone;
  L.inv_deg = d.aggr == CGR_AGGR_MEAN ? b.take(4 * N) : kNone;
  L.inv_cnt = d.pool == CGR_POOL_MEAN ? b.take(4 * B) : kNone;
  L.pool_arg = d.pool == CGR_POOL_MAX ? b.take(4 * B * Hp) : kNone;
  // partial sums of the layer GEMMs' hub segments (over >= 3 row tiles), one slot pair per tile
  const size_t rt = (size_t)cdiv(d.E, b3nt_rows((int)d.E, d.H));
  L.fpart = b.take(4 * rt * 2 * 16 *
                   std::max((size_t)lc.tiles * lc.nf, (size_t)dc.tiles * dc.nf));
}

ArenaLayout arena_layout(const Dims& d) {
  ArenaLayout L;
  memset(&L, 0xff, sizeof(L));
  Bump b;
  const size_t N = (size_t)d.N, E = (size_t)d.E, B = (size_t)d.B, Hp = (size_t)d.Hp;
  layout_prefix(d, L, b);
  L.b3x = d.F > 0 ? b.take(16 * b3_img_u4(b3nt_cols((int)d.N, 2 * d.H), d.F)) : kNone;
  // the node-row readout GEMMs in their grid-filling column tiling (b3nt_cols)
  const B3Cols rc = b3nt_cols((int)d.N, d.H);
  L.b3rof = b.take(16 * b3_img_u4(rc, d.H));
  L.b3rob = b.take(16 * b3_img_u4(rc, d.H));
  for (int l = 0; l < d.D; ++l) {
    L.b3lf[l] = b.take(16 * b3_img_u4(layer_cols(d), d.H));
    L.b3lb[l] = b.take(16 * b3_img_u4(layer_cols(d), d.H));
  }
  for (int l = 0; l <= CGR_MAX_DEPTH; ++l) {
    L.h[l] = l <= d.D ? b.take(4 * E * Hp) : kNone;
    L.a[l] = l <= d.D ? b.take(4 * N * Hp) : kNone;
    L.pre[l] = (l <= d.D && d.act != CGR_ACT_RELU) ? b.take(4 * E * Hp) : kNone;
  }
  L.zn = d.act != CGR_ACT_RELU ? b.take(4 * N * Hp) : kNone;
  L.hn = b.take(4 * N * Hp);
  L.g = b.take(4 * B * Hp);
  L.bytes = b.off;
  L.off_index_begin = 0;
  return L;
}

ArenaLayout eval_arena_layout(const Dims& d) {
  ArenaLayout L;
  memset(&L, 0xff, sizeof(L));
  Bump b;
  const size_t N = (size_t)d.N, E = (size_t)d.E, B = (size_t)d.B, Hp = (size_t)d.Hp;
  layout_prefix(d, L, b);
  const size_t h0 = b.take(4 * E * Hp);
  const size_t hr[2] = {d.D >= 2 ? b.take(4 * E * Hp) : kNone, b.take(4 * E * Hp)};
  const size_t ar[3] = {b.take(4 * N * Hp), b.take(4 * N * Hp),
                        d.D >= 2 ? b.take(4 * N * Hp) : kNone};
  for (int l = 0; l <= CGR_MAX_DEPTH; ++l) {
    L.h[l] = l > d.D ? kNone : (l == 0 ? h0 : hr[l & 1]);
    L.a[l] = l > d.D ? kNone : ar[l % 3];
  }
  L.hn = b.take(4 * N * Hp);
  L.g = b.take(4 * B * Hp);
  // forward weight images, packed by every predict that is not handed pre-packed ones
  L.b3x = d.F > 0 ? b.take(16 * b3_img_u4(b3nt_cols((int)d.N, 2 * d.H), d.F)) : kNone;
  L.b3rof = b.take(16 * b3_img_u4(b3nt_cols((int)d.N, d.H), d.H));
  for (int l = 0; l < d.D; ++l) L.b3lf[l] = b.take(16 * b3_img_u4(layer_cols(d), d.H));
  L.bytes = b.off;
  L.off_index_begin = 0;
  return L;
}

ImageLayout image_layout(const Dims& d) {
  ImageLayout I;
  Bump b;
  I.b3x = d.F > 0 ? b.take(16 * b3_img_u4(2 * d.H, d.F)) : kNone;
  I.b3rof = b.take(16 * b3_img_u4(d.H, d.H));
  for (int l = 0; l < CGR_MAX_DEPTH; ++l) I.b3lf[l] = l < d.D ? b.take(16 * b3_img_u4(d.H, d.H)) : kNone;
  I.bytes = b.off;
  return I;
}

static inline void* at(void* base, size_t off) {
  return off == kNone ? nullptr : static_cast<char*>(base) + off;
}

IndexView index_view(void* arena, const ArenaLayout& L) {
  IndexView v;
  v.deg_dst = (int*)at(arena, L.deg_dst);
  v.deg_src = (int*)at(arena, L.deg_src);
  v.cursor = (int*)at(arena, L.cursor);
  v.cursor2 = (int*)at(arena, L.cursor2);
  v.graph_cnt = (int*)at(arena, L.graph_cnt);
  v.status = (int*)at(arena, L.status);
  v.fcnt = (int*)at(arena, L.fcnt);
  v.fpart = (float*)at(arena, L.fpart);
  v.rng = (uint64_t*)at(arena, L.rng);
  v.zero_block = at(arena, L.zero_block);
  v.zero_bytes = L.zero_bytes;
  v.perm = (int*)at(arena, L.perm);
  v.src_s = (int*)at(arena, L.src_s);
  v.dst_s = (int*)at(arena, L.dst_s);
  v.rev_s = (int*)at(arena, L.rev_s);
  v.src_list = (int*)at(arena, L.src_list);
  v.inv = (int*)at(arena, L.inv);
  v.src_c = (int*)at(arena, L.src_c);
  v.dst_c = (int*)at(arena, L.dst_c);
  v.dst_ptr = (int*)at(arena, L.dst_ptr);
  v.src_ptr = (int*)at(arena, L.src_ptr);
  v.graph_ptr = (int*)at(arena, L.graph_ptr);
  v.node_graph = (int*)at(arena, L.node_graph);
  return v;
}

FloatView float_view(void* arena, const ArenaLayout& L, const Dims& d) {
  FloatView f;
  f.e_s = (float*)at(arena, L.e_s);
  f.w0eT = (float*)at(arena, L.w0eT);
  f.P = (float*)at(arena, L.P);
  f.Q = (float*)at(arena, L.Q);
  f.xp = (float*)at(arena, L.xp);
  f.inv_deg = (float*)at(arena, L.inv_deg);
  f.inv_cnt = (float*)at(arena, L.inv_cnt);
  f.pool_arg = (int*)at(arena, L.pool_arg);
  for (int l = 0; l <= CGR_MAX_DEPTH; ++l) {
    f.h[l] = (float*)at(arena, L.h[l]);
    f.a[l] = (float*)at(arena, L.a[l]);
    f.pre[l] = (float*)at(arena, L.pre[l]);
  }
  f.zn = (float*)at(arena, L.zn);
  f.hn = (float*)at(arena, L.hn);
  f.g = (float*)at(arena, L.g);
  f.b3x = at(arena, L.b3x);
  f.b3rof = at(arena, L.b3rof);
  f.b3rob = at(arena, L.b3rob);
  for (int l = 0; l < CGR_MAX_DEPTH; ++l) {
    f.b3lf[l] = l < d.D ? at(arena, L.b3lf[l]) : nullptr;
    f.b3lb[l] = l < d.D ? at(arena, L.b3lb[l]) : nullptr;
  }
  return f;
}

// column tiling of the layer GEMMs (forward and fused backward) over this batch's E rows: b3_cols
// when that fills the chip, else the narrower tiles of b3nt_cols (small batches: train.py's 32
// reactions run 60 -> 210 workgroups per layer GEMM)
B3Cols layer_cols(const Dims& d) { return b3nt_cols((int)d.E, d.H); }

// row tiles x column tiles of the fused layer-backward GEMM (gnn_bwd.hip, ep_bwd.hpp)
int bwd_seg_tiles(const Dims& d) {
  return (int)cdiv(d.E, b3nt_rows((int)d.E, d.H)) * layer_cols(d).tiles;
}

// learnable-skip partial sums per layer: the top layer's activation kernel writes one per block,
// the fused layer-backward GEMM below it two per workgroup (its rows, the crossing segment that
// starts in its tile: ep_bwd.hpp)
int bwd_dsig_slots(const Dims& d) {
  return (int)std::max<int64_t>(2 * (int64_t)bwd_seg_tiles(d), layer_act_bwd_blocks(d.E, d.Hp));
}

WorkspaceLayout workspace_layout(const Dims& d) {
  WorkspaceLayout W;
  Bump b;
  const size_t N = (size_t)d.N, E = (size_t)d.E, Hp = (size_t)d.Hp;
  W.dpre = b.take(4 * E * Hp * (size_t)d.D);  // one per layer (gnn_bwd.hip)
  W.dm = b.take(4 * E * Hp);
  W.dh0 = b.take(4 * E * Hp);
  W.dzn = b.take(4 * N * Hp);
  W.ds = b.take(4 * N * Hp);
  W.Gs = b.take(4 * N * Hp);
  W.img_side = b.take(b3_eimg_bytes(std::max(d.E, d.N), d.H));
  W.img_main = b.take(b3_eimg_bytes(d.N, d.H));
  W.img_top = b.take(b3_eimg_bytes(d.E, d.H));
  // split-K slabs: every plan a call site may pick for its shape (gnn_bwd.hip), the largest wins.
  // The side-stream weight gradients (readout, layers, edge features) run one after another and
  // share `slab`; the node weight gradient runs beside them on the caller's stream: `slab2`.
  size_t slab = 0, bslab = 0;
  auto fit = [&](const TnPlan& p, int Nout, int Kout) {
    slab = std::max(slab, (size_t)p.splits * Nout * (size_t)((Kout + 3) & ~3));  // rows to 4
    bslab = std::max(bslab, (size_t)p.splits * Nout);
  };
  auto tnr = [&](const TnrPlan& q) { return TnPlan{q.tiles_n, q.tiles_k, q.splits, q.rows_per_split}; };
  const int Fx = d.F % 4 ? d.Fp : d.F;  // x columns the x-side GEMMs cover (pad columns zero)
  const int Kr = Fx + d.H;              // readout: [x | s]
  fit(tn_plan(d.H, Kr, (int)d.N), d.H, Kr);
  fit(tnr(plan_tnr<5, 4>(d.H, Kr, (int)d.N, kTnrReadoutTarget)), d.H, Kr);
  fit(b3tn_tnplan(d.H, Kr, (int)d.N, kB3TnReadoutTarget), d.H, Kr);
  fit(tn_plan(d.H, d.H, (int)d.E), d.H, d.H);
  fit(b3tn_tnplan(d.H, d.H, (int)d.E), d.H, d.H);
  {
    const int tf = tnr_layer_frags(d.H);
    if (tf == 5) fit(tnr(plan_tnr<5, 5>(d.H, d.H, (int)d.E, kTnrLayerTarget)), d.H, d.H);
    if (tf == 4) fit(tnr(plan_tnr<4, 4>(d.H, d.H, (int)d.E, kTnrLayerTarget)), d.H, d.H);
  }
  if (d.Fe > 0) fit(tn_plan(d.H, d.Fe, (int)d.E, kEdgeTnTargetWorkgroups), d.H, d.Fe);
  W.slab_elems = slab;
  W.bslab_elems = bslab;
  W.slab = b.take(4 * std::max<size_t>(slab, 1));
  W.bslab = b.take(4 * std::max<size_t>(bslab, 1));
  W.slab_b = b.take(4 * std::max<size_t>(slab, 1));  // alternating with slab (gnn_bwd.hip)
  W.bslab_b = b.take(4 * std::max<size_t>(bslab, 1));
  slab = bslab = 0;
  if (d.F > 0) {
    fit(tn_plan(d.H, d.F, (int)d.N), d.H, d.F);
    fit(tnr(plan_tnr<5, 4>(d.H, Fx, (int)d.N, kTnrNodeTarget)), d.H, Fx);
    fit(b3tn_tnplan(d.H, Fx, (int)d.N, kB3TnNodeTarget), d.H, Fx);
  }
  W.slab2 = b.take(4 * std::max<size_t>(slab, 1));
  W.bslab2 = b.take(4 * std::max<size_t>(bslab, 1));
  W.dag = b.take(2 * 4 * N * Hp);  // two, alternating by layer
  // segment tickets, then one unpaired grid counter per fused layer-backward launch
  W.cnt = b.take(4 * (N * (size_t)layer_cols(d).tiles + CGR_MAX_DEPTH));
  W.part = b.take(4 * (size_t)bwd_seg_tiles(d) * 2 * (size_t)layer_cols(d).nf * 16);
  W.wxT = b.take(4 * (size_t)d.F * (size_t)input_grad_ldw(d.H));
  W.dsig_blocks = bwd_dsig_slots(d);
  W.dsig_part = b.take(4 * (size_t)d.D * (size_t)W.dsig_blocks);
  W.bytes = b.off;
  return W;
}

static int validate_config(const cgr_gnn_config* c) {
  CGR_CHECK(c != nullptr, "cgr: config is NULL");
  CGR_CHECK(c->num_node_features >= 0, "cgr: num_node_features must be >= 0");
  CGR_CHECK(c->num_edge_features >= 0, "cgr: num_edge_features must be >= 0");
  CGR_CHECK(c->hidden >= 1, "cgr: hidden size must be >= 1");
  CGR_CHECK(c->depth >= 1 && c->depth <= CGR_MAX_DEPTH, "cgr: depth must be in [1, 32]");
  CGR_CHECK(c->activation >= 0 && c->activation < ACT_COUNT, "cgr: unknown activation code");
  CGR_CHECK(c->aggregation == CGR_AGGR_ADD || c->aggregation == CGR_AGGR_MEAN,
            "cgr: unknown aggregation (CGR_AGGR_ADD, CGR_AGGR_MEAN)");
  CGR_CHECK(c->pooling == CGR_POOL_ADD || c->pooling == CGR_POOL_MEAN ||
                c->pooling == CGR_POOL_MAX,
            "cgr: unknown pooling (CGR_POOL_ADD, CGR_POOL_MEAN, CGR_POOL_MAX)");
  return 0;
}

static int validate_batch(const cgr_gnn_config* c, const cgr_batch* b) {
  CGR_CHECK(b != nullptr, "cgr: batch is NULL");
  CGR_CHECK(b->num_nodes >= 1 && b->num_nodes < (1ll << 31), "cgr: num_nodes out of range");
  CGR_CHECK(b->num_edges >= 1 && b->num_edges < (1ll << 30),
            "cgr: num_edges must be >= 1 (the reference's flip/view needs edge pairs)");
  CGR_CHECK(b->num_edges % 2 == 0,
            "cgr: num_edges must be even: reverse edge of e is e^1 (GNN.py:136-138)");
  CGR_CHECK(b->num_graphs >= 1 && b->num_graphs <= b->num_nodes, "cgr: num_graphs out of range");
  CGR_CHECK(b->batch != nullptr || b->graph_ptr != nullptr || b->num_graphs == 1,
            "cgr: batch == NULL requires num_graphs == 1");
  CGR_CHECK(b->edge_index != nullptr, "cgr: edge_index is NULL");
  CGR_CHECK(c->num_node_features == 0 || b->x != nullptr, "cgr: x is NULL");
  CGR_CHECK(c->num_edge_features == 0 || b->edge_attr != nullptr, "cgr: edge_attr is NULL");
  return 0;
}

}  // namespace cgr

using namespace cgr;

extern "C" {

int cgr_abi_version(void) { return CGR_ABI_VERSION; }

const char* cgr_last_error(void) { return g_err.c_str(); }

int cgr_gnn_num_params(const cgr_gnn_config* cfg) {
  if (validate_config(cfg)) return -1;
  return 6 + 2 * cfg->depth + (cfg->learnable_skip ? cfg->depth : 0);
}

int64_t cgr_gnn_arena_bytes(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B) {
  if (validate_config(cfg)) return -1;
  return (int64_t)arena_layout(make_dims(cfg, N, E, B)).bytes;
}

int64_t cgr_gnn_workspace_bytes(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B) {
  if (validate_config(cfg)) return -1;
  return (int64_t)workspace_layout(make_dims(cfg, N, E, B)).bytes;
}

int64_t cgr_gnn_arena_offset(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B,
                             const char* name, int32_t index) {
  if (validate_config(cfg) || name == nullptr) return -1;
  const ArenaLayout L = arena_layout(make_dims(cfg, N, E, B));
  size_t o = (size_t)-1;
  const std::string n(name);
  const bool li = index >= 0 && index <= CGR_MAX_DEPTH;
  if (n == "status") o = L.status;
  if (n == "rng") o = L.rng;
  else if (n == "perm") o = L.perm;
  else if (n == "src_s") o = L.src_s;
  else if (n == "dst_s") o = L.dst_s;
  else if (n == "rev_s") o = L.rev_s;
  else if (n == "src_list") o = L.src_list;
  else if (n == "dst_ptr") o = L.dst_ptr;
  else if (n == "src_ptr") o = L.src_ptr;
  else if (n == "graph_ptr") o = L.graph_ptr;
  else if (n == "node_graph") o = L.node_graph;
  else if (n == "e_s") o = L.e_s;
  else if (n == "P") o = L.P;
  else if (n == "Q") o = L.Q;
  else if (n == "h" && li) o = L.h[index];
  else if (n == "a" && li) o = L.a[index];
  else if (n == "pre" && li) o = L.pre[index];
  else if (n == "zn") o = L.zn;
  else if (n == "hn") o = L.hn;
  else if (n == "g") o = L.g;
  return o == (size_t)-1 ? -1 : (int64_t)o;
}

int cgr_graph_prep(const cgr_gnn_config* cfg, const cgr_batch* b, void* arena, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(arena != nullptr, "cgr: arena is NULL");
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  const ArenaLayout L = arena_layout(d);
  const FloatView fv = float_view(arena, L, d);
  PrepArgs pa{b->edge_index, b->batch, b->graph_ptr, b->edge_attr, d.N, d.E, d.B,
              d.Fe,          d.Fep,   index_view(arena, L), fv.e_s};
  return cgr_graph_prep_impl(pa, (hipStream_t)stream);
}

int cgr_gnn_forward(const cgr_gnn_config* cfg, const float* const* params, const cgr_batch* b,
                    const float* dropout_p, uint64_t seed, uint64_t* rng_counter,
                    int32_t training, void* arena, float* y, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && arena != nullptr && y != nullptr,
            "cgr: params / arena / y must not be NULL");
  CGR_CHECK((training & ~(CGR_TRAIN_DROPOUT | CGR_TRAIN_FOR_BACKWARD)) == 0,
            "cgr: unknown `training` bits (CGR_TRAIN_DROPOUT | CGR_TRAIN_FOR_BACKWARD)");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  note_forward(arena, -1);  // not usable by a backward unless the forward below succeeds
  const int r = gnn_forward_impl(d, params, b, dropout_p, seed, rng_counter, training, arena, y,
                                 (hipStream_t)stream, FwdMode{});
  if (r == 0) note_forward(arena, training);
  return r;
}

int cgr_gnn_backward(const cgr_gnn_config* cfg, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, int32_t training, const void* arena,
                     const float* dy, float* const* grads, void* workspace,
                     void* const* bucket_events, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && arena != nullptr && dy != nullptr && grads != nullptr &&
                workspace != nullptr,
            "cgr: params / arena / dy / grads / workspace must not be NULL");
  CGR_CHECK((training & ~(CGR_TRAIN_DROPOUT | CGR_TRAIN_FOR_BACKWARD)) == 0,
            "cgr: unknown `training` bits (CGR_TRAIN_DROPOUT | CGR_TRAIN_FOR_BACKWARD)");
  const int ff = forward_flags(arena);
  CGR_CHECK(ff >= 0 && (ff & CGR_TRAIN_FOR_BACKWARD),
            "cgr_gnn_backward: `arena` was not filled by a successful cgr_gnn_forward with "
            "CGR_TRAIN_FOR_BACKWARD set");
  CGR_CHECK((ff & CGR_TRAIN_DROPOUT) == (training & CGR_TRAIN_DROPOUT),
            "cgr_gnn_backward: `training` dropout bit differs from the forward's");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) {
    CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
    CGR_CHECK(grads[i] != nullptr, "cgr: NULL gradient pointer");
  }
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  if (bucket_events)
    for (int i = 0; i < CGR_GRAD_BUCKETS(cfg->depth); ++i)
      CGR_CHECK(bucket_events[i] != nullptr, "cgr_gnn_backward: NULL bucket event");
  const int r = gnn_backward_impl(d, params, b, dropout_p, seed, training, arena, dy, grads,
                                  workspace, reinterpret_cast<hipEvent_t const*>(bucket_events),
                                  (hipStream_t)stream);
  if (r == 0) note_backward(arena, workspace);
  return r;
}

int cgr_gnn_input_grads(const cgr_gnn_config* cfg, const float* const* params,
                        const cgr_batch* b, const void* arena, const float* dy, void* workspace,
                        float* dx, float* dedge_attr, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && arena != nullptr && dy != nullptr && workspace != nullptr,
            "cgr: params / arena / dy / workspace must not be NULL");
  const int ff = forward_flags(arena);
  CGR_CHECK(ff >= 0 && (ff & CGR_TRAIN_FOR_BACKWARD),
            "cgr_gnn_input_grads: `arena` was not filled by a successful cgr_gnn_forward with "
            "CGR_TRAIN_FOR_BACKWARD set");
  CGR_CHECK(backward_matches(arena, workspace),
            "cgr_gnn_input_grads: `workspace` does not hold a cgr_gnn_backward of this `arena`'s "
            "latest forward (run the backward first, with the same arena and workspace)");
  CGR_CHECK(((uintptr_t)dx & 15) == 0 && ((uintptr_t)dedge_attr & 15) == 0,
            "cgr_gnn_input_grads: dx / dedge_attr must be 16-byte aligned (or NULL)");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  return gnn_input_grads_impl(d, params, arena, dy, workspace, dx, dedge_attr,
                              (hipStream_t)stream);
}

int64_t cgr_gnn_image_bytes(const cgr_gnn_config* cfg) {
  if (validate_config(cfg)) return -1;
  return (int64_t)image_layout(make_dims(cfg, 1, 2, 1)).bytes;
}

int cgr_gnn_pack_images(const cgr_gnn_config* cfg, const float* const* params, void* images,
                        void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && images != nullptr, "cgr: params / images must not be NULL");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
  const Dims d = make_dims(cfg, 1, 2, 1);
  HIP_RET(pack_forward_images(d, params, image_layout(d), images, (hipStream_t)stream));
  return 0;
}

int64_t cgr_gnn_predict_arena_bytes(const cgr_gnn_config* cfg, int64_t N, int64_t E, int64_t B) {
  if (validate_config(cfg)) return -1;
  return (int64_t)eval_arena_layout(make_dims(cfg, N, E, B)).bytes;
}

int cgr_gnn_predict(const cgr_gnn_config* cfg, const float* const* params, const cgr_batch* b,
                    const float* dropout_p, uint64_t seed, uint64_t* rng_counter,
                    int32_t training, const void* images, void* arena, float* y, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && arena != nullptr && y != nullptr,
            "cgr: params / arena / y must not be NULL");
  CGR_CHECK((training & ~CGR_TRAIN_DROPOUT) == 0,
            "cgr_gnn_predict: `training` may only hold CGR_TRAIN_DROPOUT (no backward follows)");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  FwdMode m;
  m.eval = true;
  m.images = images;
  note_forward(arena, -1);  // never a backward's arena
  return gnn_forward_impl(d, params, b, dropout_p, seed, rng_counter, training, arena, y,
                          (hipStream_t)stream, m);
}

int32_t cgr_device_errors(int32_t device, int32_t clear) {
  SideStreams* ss = side_streams_of(device);
  if (!ss || !ss->err_host) return 0;
  volatile int* w = ss->err_host;
  int32_t bits = 0;
  if (w[kDevErrUnpairedTimeout]) bits |= CGR_DEVERR_UNPAIRED_TIMEOUT;
  if (w[kDevErrUnpairedSeen]) bits |= CGR_DEVERR_UNPAIRED_SEEN;
  if (clear) {
    if (bits & CGR_DEVERR_UNPAIRED_TIMEOUT) w[kDevErrUnpairedTimeout] = 0;
    if (bits & CGR_DEVERR_UNPAIRED_SEEN) w[kDevErrUnpairedSeen] = 0;
  }
  return bits;
}

int cgr_segment_sum(const float* values, int64_t ld_values, const int32_t* index,
                    const int32_t* seg_ptr, int64_t num_segments, int64_t width, float* out,
                    int64_t ld_out, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(values != nullptr && seg_ptr != nullptr && out != nullptr,
            "cgr_segment_sum: NULL pointer");
  CGR_CHECK(num_segments >= 0 && width >= 0 && ld_values >= width && ld_out >= width,
            "cgr_segment_sum: bad sizes");
  HIP_RET(segment_sum(values, ld_values, index, seg_ptr, num_segments, width, out, ld_out,
                      (hipStream_t)stream));
  return 0;
}

}  // extern "C"
