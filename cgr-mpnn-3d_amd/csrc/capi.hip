// C ABI of libcgr_mpnn3d.so (include/cgr_mpnn3d.h): validation, arena/workspace layout, error
// reporting.  No entry point allocates or synchronises; all work is enqueued on `stream`.
#include <string.h>

#include <string>

#include "dispatch.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"

namespace cgr {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

int gnn_forward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, uint64_t* rng_counter, int training,
                     void* arena, float* y, hipStream_t st);
int gnn_backward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                      const float* dropout_p, uint64_t seed, int training, const void* arena,
                      const float* dy, float* const* grads, void* workspace, hipStream_t st);

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
  return d;
}

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

ArenaLayout arena_layout(const Dims& d) {
  ArenaLayout L;
  memset(&L, 0xff, sizeof(L));
  Bump b;
  const size_t N = (size_t)d.N, E = (size_t)d.E, B = (size_t)d.B, Hp = (size_t)d.Hp;
  // zero block: six int arrays back to back, padded to a multiple of 16 bytes
  L.zero_block = b.off;
  L.deg_dst = b.off;
  L.deg_src = L.deg_dst + 4 * N;
  L.cursor = L.deg_src + 4 * N;
  L.cursor2 = L.cursor + 4 * N;
  L.graph_cnt = L.cursor2 + 4 * N;
  L.status = L.graph_cnt + 4 * B;
  L.zero_bytes = (size_t)round_up((int64_t)(4 * (4 * N + B) + 16), 16);
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
  L.wT = CGR_B3 ? kNone : b.take(4 * (size_t)(d.D + 1) * d.H * Hp);
  if (CGR_B3) {
    // x-GEMM images: one of 2H rows, or (split x-GEMM) two of H rows back to back
    const size_t xi = std::max(b3_img_u4(2 * d.H, d.F), 2 * b3_img_u4(d.H, d.F));
    L.b3x = d.F > 0 ? b.take(16 * xi) : kNone;
    L.b3rof = b.take(16 * b3_img_u4(d.H, d.H));
    L.b3rob = b.take(16 * b3_img_u4(d.H, d.H));
    for (int l = 0; l < d.D; ++l) {
      L.b3lf[l] = b.take(16 * b3_img_u4(d.H, d.H));
      L.b3lb[l] = b.take(16 * b3_img_u4(d.H, d.H));
    }
    if (CGR_B3TP) {
      const size_t pb = 2 * (size_t)b3tp_rows(d.E) * (size_t)b3tp_layer_ld(d.H);
      for (int l = 0; l < d.D; ++l) {
        L.mhi[l] = b.take(pb);
        L.mlo[l] = b.take(pb);
      }
    }
  }
  for (int l = 0; l <= CGR_MAX_DEPTH; ++l) {
    L.h[l] = l <= d.D ? b.take(4 * E * Hp) : kNone;
    L.a[l] = l <= d.D ? b.take(4 * N * Hp) : kNone;
    L.pre[l] = (l <= d.D && d.act != CGR_ACT_RELU) ? b.take(4 * E * Hp) : kNone;
    // h_0's mask comes from the fused edge init (Hp <= 512), every layer's from its epilogue
    L.hb[l] = (CGR_HBITS && l <= d.D && d.act == CGR_ACT_RELU && (l > 0 || Hp <= 512))
                  ? b.take(E * (Hp / 4)) : kNone;
  }
  L.zn = d.act != CGR_ACT_RELU ? b.take(4 * N * Hp) : kNone;
  L.hn = b.take(4 * N * Hp);
  L.g = b.take(4 * B * Hp);
  L.bytes = b.off;
  L.off_index_begin = 0;
  return L;
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
  f.wT = (float*)at(arena, L.wT);
  for (int l = 0; l <= CGR_MAX_DEPTH; ++l) {
    f.h[l] = (float*)at(arena, L.h[l]);
    f.a[l] = (float*)at(arena, L.a[l]);
    f.pre[l] = (float*)at(arena, L.pre[l]);
    f.hb[l] = (uint8_t*)at(arena, L.hb[l]);
  }
  f.zn = (float*)at(arena, L.zn);
  f.hn = (float*)at(arena, L.hn);
  f.g = (float*)at(arena, L.g);
  f.b3x = f.b3rof = f.b3rob = nullptr;
  for (int l = 0; l < CGR_MAX_DEPTH; ++l) f.b3lf[l] = f.b3lb[l] = nullptr;
  for (int l = 0; l < CGR_MAX_DEPTH; ++l) f.mhi[l] = f.mlo[l] = nullptr;
  f.mld = b3tp_layer_ld(d.H);
  if (CGR_B3) {
    f.b3x = at(arena, L.b3x);
    f.b3rof = at(arena, L.b3rof);
    f.b3rob = at(arena, L.b3rob);
    for (int l = 0; l < d.D; ++l) {
      f.b3lf[l] = at(arena, L.b3lf[l]);
      f.b3lb[l] = at(arena, L.b3lb[l]);
      if (CGR_B3TP) {
        f.mhi[l] = static_cast<uint16_t*>(at(arena, L.mhi[l]));
        f.mlo[l] = static_cast<uint16_t*>(at(arena, L.mlo[l]));
      }
    }
  }
  return f;
}

WorkspaceLayout workspace_layout(const Dims& d) {
  WorkspaceLayout W;
  Bump b;
  const size_t N = (size_t)d.N, E = (size_t)d.E, B = (size_t)d.B, Hp = (size_t)d.Hp;
  for (int l = 0; l < (CGR_DPRE_RING ? 2 : d.D); ++l) W.dpre[l] = b.take(4 * E * Hp);
  for (int l = 0; l < CGR_MAX_DEPTH; ++l) W.dphi[l] = W.dplo[l] = (size_t)-1;
  if (CGR_B3 && CGR_B3TP) {
    const size_t pb = 2 * (size_t)b3tp_rows(d.E) * (size_t)b3tp_layer_ld(d.H);
    for (int l = 0; l < (CGR_DPRE_RING ? 2 : d.D); ++l) {
      W.dphi[l] = b.take(pb);
      W.dplo[l] = b.take(pb);
    }
  }
  W.dm = b.take(4 * E * Hp);
  W.dh0 = b.take(4 * E * Hp);
  W.dzn = b.take(4 * N * Hp);
  W.ds = b.take(4 * N * Hp);
  W.Gs = b.take(4 * N * Hp);
  W.dg = b.take(4 * B * Hp);
  size_t slab = 0, bslab = 0;
  auto acc = [&](int Nout, int Kout, int64_t R) {
    const TnPlan p = tn_plan(Nout, Kout, (int)R);
    const size_t s = (size_t)p.splits * Nout * (size_t)((Kout + 3) & ~3);  // rows padded to 4
    const size_t bs = (size_t)p.splits * Nout;
    slab = s > slab ? s : slab;
    bslab = bs > bslab ? bs : bslab;
  };
  // side-stream TN GEMMs (readout, layers, edge features): with batched reduction each gets its
  // own slab (reduced together in one launch at the end of the side stream), otherwise they share
  // one; the main-stream TN (x-part of edge init) runs beside them and always gets its own
  auto side = [&](int Nout, int Kout, int64_t R) {
    if (!CGR_BATCH_REDUCE) return acc(Nout, Kout, R);
    const TnPlan p = tn_plan(Nout, Kout, (int)R);
    slab += (size_t)p.splits * Nout * (size_t)((Kout + 3) & ~3);
    bslab += (size_t)p.splits * Nout;
  };
  side(d.H, (d.F % 4 ? d.Fp : d.F) + d.H, d.N);  // readout TN runs over [xp | s] when padded
  if (!CGR_BATCH_REDUCE) {  // register-direct readout TN: its own split count
    const int Kr = (d.F % 4 ? d.Fp : d.F) + d.H;
    const TnrPlan q = plan_tnr<5, 4>(d.H, Kr, (int)d.N, CGR_TNR_RO_TARGET);
    const size_t s2 = (size_t)q.splits * d.H * (size_t)((Kr + 3) & ~3), bs2 = (size_t)q.splits * d.H;
    slab = s2 > slab ? s2 : slab;
    bslab = bs2 > bslab ? bs2 : bslab;
  }
  auto b3acc = [&](int Nout, int Kout, int64_t R, int copies,
                   int target = CGR_B3TN_TARGET) {  // split-bf16 TN plans
    if (!CGR_B3TN) return;
    const TnPlan q = b3tn_tnplan(Nout, Kout, (int)R, target);
    const size_t s = (size_t)q.splits * Nout * (size_t)((Kout + 3) & ~3);
    const size_t bs = (size_t)q.splits * Nout;
    if (CGR_BATCH_REDUCE) {
      slab += (size_t)copies * s;  // (over-allocates, as below)
      bslab += (size_t)copies * bs;
    } else {
      slab = s > slab ? s : slab;
      bslab = bs > bslab ? bs : bslab;
    }
  };
  b3acc(d.H, (d.F % 4 ? d.Fp : d.F) + d.H, d.N, 1, CGR_B3TN_RO_TARGET);
  b3acc(d.H, d.H, d.E, d.D);
  if (CGR_B3 && CGR_B3TP) {  // plane TN plans of the layer weight gradients
    const B3TpPlan q = b3tp_plan(d.H, d.H, (int)d.E);
    const size_t s = (size_t)q.splits * d.H * (size_t)((d.H + 3) & ~3), bs = (size_t)q.splits * d.H;
    if (CGR_BATCH_REDUCE) {
      slab += (size_t)d.D * s;
      bslab += (size_t)d.D * bs;
    } else {
      slab = s > slab ? s : slab;
      bslab = bs > bslab ? bs : bslab;
    }
  }
  for (int l = 0; l < (CGR_BATCH_REDUCE ? d.D : 1); ++l) side(d.H, d.H, d.E);
  {  // the layer weight gradient may run on the register-direct kernel with its own split count
    const int tf = tnr_layer_frags(d.H);
    const TnrPlan q = tf == 5   ? plan_tnr<5, 5>(d.H, d.H, (int)d.E, CGR_TNR_TARGET_WGS)
                      : tf == 4 ? plan_tnr<4, 4>(d.H, d.H, (int)d.E, CGR_TNR_TARGET_WGS)
                                : TnrPlan{0, 0, 0, 0};
    const size_t s = (size_t)q.splits * d.H * (size_t)((d.H + 3) & ~3);
    const size_t bs = (size_t)q.splits * d.H;
    if (CGR_BATCH_REDUCE) {
      slab += (size_t)d.D * s;  // (over-allocates: both sizes counted; batching is an A/B option)
      bslab += (size_t)d.D * bs;
    } else {
      slab = s > slab ? s : slab;
      bslab = bs > bslab ? bs : bslab;
    }
  }
  if (d.Fe > 0) side(d.H, d.Fe, d.E);
  W.slab_elems = slab;
  W.bslab_elems = bslab;
  W.slab = b.take(4 * slab);
  W.bslab = b.take(4 * bslab);
  slab = 0;
  bslab = 0;
  if (d.F > 0) {
    acc(d.H, d.F, d.N);
    const int Fx = d.F % 4 ? d.Fp : d.F;  // register-direct node TN covers the padded columns
    const TnrPlan q = plan_tnr<5, 4>(d.H, Fx, (int)d.N, CGR_TNR_NODE_TARGET);
    const size_t s2 = (size_t)q.splits * d.H * (size_t)((Fx + 3) & ~3), bs2 = (size_t)q.splits * d.H;
    slab = s2 > slab ? s2 : slab;
    bslab = bs2 > bslab ? bs2 : bslab;
    if (CGR_B3TN) {
      const TnPlan b3 = b3tn_tnplan(d.H, Fx, (int)d.N, CGR_B3TN_NODE_TARGET);
      const size_t s3 = (size_t)b3.splits * d.H * (size_t)((Fx + 3) & ~3), bs3 = (size_t)b3.splits * d.H;
      slab = s3 > slab ? s3 : slab;
      bslab = bs3 > bslab ? bs3 : bslab;
    }
  }
  if (d.Fe > 0) acc(d.H, d.Fe, d.E);  // the edge-feature TN may use slab2 (CGR_EDGE_TN_MAIN)
  W.slab2 = b.take(4 * (slab > 0 ? slab : 1));
  W.bslab2 = b.take(4 * (bslab > 0 ? bslab : 1));
  W.dsig_blocks = segsum_act_bwd_blocks(d.E, d.N, d.Hp);
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
  CGR_CHECK(c->activation >= 0 && c->activation <= 2, "cgr: unknown activation code");
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
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  return gnn_forward_impl(d, params, b, dropout_p, seed, rng_counter, training, arena, y,
                          (hipStream_t)stream);
}

int cgr_gnn_backward(const cgr_gnn_config* cfg, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, int32_t training, const void* arena,
                     const float* dy, float* const* grads, void* workspace, void* stream) {
  clear_stale_hip_error();
  int rc = validate_config(cfg);
  if (rc) return rc;
  rc = validate_batch(cfg, b);
  if (rc) return rc;
  CGR_CHECK(params != nullptr && arena != nullptr && dy != nullptr && grads != nullptr &&
                workspace != nullptr,
            "cgr: params / arena / dy / grads / workspace must not be NULL");
  const int np = cgr_gnn_num_params(cfg);
  for (int i = 0; i < np; ++i) {
    CGR_CHECK(params[i] != nullptr, "cgr: NULL parameter pointer");
    CGR_CHECK(grads[i] != nullptr, "cgr: NULL gradient pointer");
  }
  const Dims d = make_dims(cfg, b->num_nodes, b->num_edges, b->num_graphs);
  return gnn_backward_impl(d, params, b, dropout_p, seed, training, arena, dy, grads, workspace,
                           (hipStream_t)stream);
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
