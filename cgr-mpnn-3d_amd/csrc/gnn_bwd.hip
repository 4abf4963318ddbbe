// Reverse mode of gnn_fwd.hip (the math is restated and pinned in
// oracle/dmpnn_numpy.py::backward).  Same gather -> MFMA GEMM -> segmented-reduce pattern as the
// forward with src and dst swapped; weight gradients are split-K TN GEMMs over the edge / node
// dimension reduced deterministically; the only atomics add the two partial sums of a segment
// that crosses a row tile onto zero (order-independent), so gradients are bitwise stable.
//
//   dwf = dy^T g ; dbf = sum dy ; dzn = dy[graph(v)] wf * act'(zn)        (ffn, pool, edge_to_node)
//   dW_n = dzn^T [x | s], db_n = colsum(dzn), ds = dzn W_n[:, F:]
//   dh_D = ds[dst]
//   for l = D-1 .. 0:
//     dpre_l = dh_{l+1} * mask * act'(pre_l) ; ds_l = sum dpre_l*h0
//     dW_l = dpre^T (a_l[src] - h_l[rev])  (message recomputed, never stored) ; db_l = colsum
//     dm = dpre W_l ; da = segsum_src(dm) ; dh_l = da[dst] - dm[rev] -> the next lower layer's
//     dpre, all in the dm GEMM's epilogue (EpLayerBwdSeg, ep_bwd.hpp: rows gathered through rev
//     so each dst segment's rows are the dm rows its node sums; dm and da never stored; segments
//     that cross a row tile completed in the same launch by their last contributor)
//   dh0 = sum_l s_l dpre_l (every layer's skip term) ; dpre0 = (dh0 + dh_0) * act'(pre0)
//   dW0[:, F:] = dpre0^T e ; db0 = colsum(dpre0) ; dW0[:, :F] = (segsum_src dpre0)^T x
//
// Streams: the critical path is act_bwd -> the fused dm GEMM per layer.
// Every weight-gradient TN GEMM (+ its slab reduction) only feeds the gradient outputs, so it runs on the side stream,
// forked right after its input is produced; every layer's dpre has a buffer of its own (the
// edge-init backward sums them into dh0), so the main stream waits for the side stream only at
// the very end.
#include <string>

#include "dispatch.hpp"
#include "ep_bwd.hpp"
#include "epilogues.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"
#include "profiling.hpp"
#include "streams.hpp"

namespace cgr {

void dropout_params(const float* dropout_p, int training, int l, uint32_t* thresh, float* scale);

template <class AL, class BL>
static hipError_t tn_gemm(const char* name, const AL& al, const BL& bl, int Nout, int Kout, int R,
                          float* slab, float* bslab, bool want_bias, TnPlan* plan, hipStream_t st,
                          int target = kTnTargetWorkgroups) {
  *plan = tn_plan(Nout, Kout, R, target);
  const TnPlan p = *plan;
  // profile class "<name>[f32]": the fallback family is visible in the per-class report (tests
  // assert which family ran for a width, bench.py keys its roofline on the plain names)
  const std::string cls = std::string(name) + "[f32]";
  ProfScope _p(cls.c_str(), st);
  return with_tn_shape(Nout, Kout, [&](auto W, auto RN) {
    return launch_tn<decltype(W)::value, decltype(RN)::value>(al, bl, p, slab, bslab,
                                                                         Nout, Kout, R, want_bias,
                                                                         st);
  });
}

// register-direct strided-fragment TN (gemm_tnr.hpp); same slab layout as tn_gemm
template <int FA, int FB, class SA, class SB>
static hipError_t tnr_gemm(const char* name, const SA& sa, const SB& sb, int Nout, int Kout,
                           int R, float* slab, float* bslab, bool want_bias, TnPlan* plan,
                           hipStream_t st, int target = kTnrLayerTarget) {
  const TnrPlan q = plan_tnr<FA, FB>(Nout, Kout, R, target);
  *plan = TnPlan{q.tiles_n, q.tiles_k, q.splits, q.rows_per_split};
  const std::string cls = std::string(name) + "[tnr]";  // "<name>[tnr]", as tn_gemm's "[f32]"
  ProfScope _p(cls.c_str(), st);
  return launch_gemm_tnr<FA, FB>(sa, sb, q, slab, bslab, Nout, Kout, R, want_bias, st);
}

// split-bf16 TN with the n-side operand A [R, Nout] as an e-image (gemm_b3.hpp): A was split
// once into `img` (by its producer -- the dzn and top-layer dpre kernels, the Gs segmented sum --
// or by b3_eimage), then every k-tile of the GEMM reads it pre-split
// prev: a previous weight gradient's slab reduction folded into this launch (gemm_b3.hpp)
template <class BL>
static hipError_t b3tni_run(const char* name, const void* img, const BL& bl, int Nout, int Kout,
                            int R, float* slab, float* bslab, bool want_bias, TnPlan* plan,
                            hipStream_t st, int target = kB3TnTarget,
                            const RedJob& prev = RedJob{}) {
  const B3TnPlan q = b3tn_plan(Nout, Kout, R, target);
  *plan = TnPlan{1, q.tiles_k, q.splits, q.rows_per_split};
  ProfScope _p(name, st);
  return launch_b3tni(B3EImg{static_cast<const b3_u4*>(img), b3_eimg_cols(Nout)}, bl, q, slab,
                      bslab, Nout, Kout, R, want_bias, st, prev);
}

// a split-K reduction waiting for its launch: folded into the next side-stream split-bf16 TN
// (the launch-boundary reduce), or launched on its own (flush) before anything that would
// overwrite its slabs; its gradient bucket's event is recorded once it has run
struct PendingReduce {
  RedJob job{};  // job.slab == nullptr: none
  int bucket = -1;
};
static RedJob make_red_job(const TnPlan& p, const float* slab, const float* bslab, int Nout,
                           int Kout, float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                           int gap_at = 0, int gap_len = 0) {
  RedJobs js{};
  add_reduce_job(js, slab, bslab, p.splits, Nout, Kout, dst, ld_dst, col_off, bias_dst, gap_at,
                 gap_len);
  return js.n ? js.j[0] : RedJob{};
}

static hipError_t tn_reduce(const TnPlan& p, const float* slab, const float* bslab, int Nout,
                            int Kout, float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                            hipStream_t st, int gap_at = 0, int gap_len = 0, bool flat = false) {
  ProfScope _p("splitk_reduce", st);
  return reduce_slabs(slab, bslab, p.splits, Nout, Kout, dst, ld_dst, col_off, bias_dst, st,
                      gap_at, gap_len, flat);
}

int gnn_backward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                      const float* dropout_p, uint64_t seed, int training, const void* arena,
                      const float* dy, float* const* grads, void* workspace,
                      hipEvent_t const* bucket_events, hipStream_t st) {
  const ArenaLayout L = arena_layout(d);
  const IndexView iv = index_view(const_cast<void*>(arena), L);
  const FloatView fv = float_view(const_cast<void*>(arena), L, d);
  const WorkspaceLayout WL = workspace_layout(d);
  char* ws = static_cast<char*>(workspace);
  float* dm = reinterpret_cast<float*>(ws + WL.dm);
  float* dh0 = reinterpret_cast<float*>(ws + WL.dh0);
  float* dzn = reinterpret_cast<float*>(ws + WL.dzn);
  float* ds = reinterpret_cast<float*>(ws + WL.ds);
  float* Gs = reinterpret_cast<float*>(ws + WL.Gs);
  // side-stream slab buffers, alternating: a TN writes one while the previous weight gradient's
  // slabs in the other are reduced in its prologue
  float* slabs[2] = {reinterpret_cast<float*>(ws + WL.slab),
                     reinterpret_cast<float*>(ws + WL.slab_b)};
  float* bslabs[2] = {reinterpret_cast<float*>(ws + WL.bslab),
                      reinterpret_cast<float*>(ws + WL.bslab_b)};
  int sb = 0;  // buffer of the next side-stream TN
  float* slab2 = reinterpret_cast<float*>(ws + WL.slab2);
  float* bslab2 = reinterpret_cast<float*>(ws + WL.bslab2);
  float* dsig_part = reinterpret_cast<float*>(ws + WL.dsig_part);
  void* img_side = ws + WL.img_side;
  void* img_main = ws + WL.img_main;
  void* img_top = ws + WL.img_top;
  // partial sums of tile-crossing segments, accumulated by layer l's fused backward GEMM: two
  // buffers, alternating by layer (a segment's completer zeroes its entries of the next one)
  auto dag_of = [&](int l) {
    return reinterpret_cast<float*>(ws + WL.dag) + (l & 1) * (int64_t)d.N * d.Hp;
  };

  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  // dpre of layer l: a buffer per layer, so that writing dpre_{l-1} never waits for the side
  // stream's weight gradient of layer l+1 (a cross-queue edge on the critical chain of a
  // captured step: ~5 us each)
  auto dpre = [&](int l) {
    return reinterpret_cast<float*>(ws + WL.dpre) + (int64_t)l * E * Hp;
  };

  SideStreams* ss = side_streams(st);
  if (!ss) return CGR_ERR_HIP;
  std::lock_guard<std::mutex> ss_lock(ss->mu);
  // instrumented (profiling) runs stay serial so per-kernel event times are isolated durations
  hipStream_t side = (prof_enabled() || single_stream()) ? st : ss->side;

  PendingReduce pend;
  auto retire = [&]() -> int {  // pend has run (folded into a TN, or launched)
    if (pend.job.slab && bucket_events && pend.bucket >= 0)
      HIP_RET(hipEventRecord(bucket_events[pend.bucket], side));
    pend = PendingReduce{};
    return 0;
  };
  // launch pend on its own (with `extra`, a job that runs in the same launch, if any)
  // max_blocks: the grid bound of the grouped reduce (kReduceMaxBlocks while the main chain runs
  // beside it; the backward's last one runs after the main chain has finished: unbounded)
  auto flush = [&](const RedJob* extra = nullptr, int max_blocks = kReduceMaxBlocks) -> int {
    RedJobs js{};
    if (pend.job.slab) js.j[js.n++] = pend.job;
    if (extra && extra->slab) js.j[js.n++] = *extra;
    if (js.n == 0) return 0;
    for (int i = 0; i < js.n; ++i) js.total += js.j[i].nblk;
    {
      ProfScope _p("splitk_reduce", side);
      HIP_RET(reduce_slabs_batched(js, max_blocks, side));
    }
    return retire();
  };
  // the side TN writing slabs[sb] took pend's job as its prologue; its own becomes pending
  auto fold = [&](const RedJob& mine, int bucket) -> int {
    const int rc = retire();
    if (rc) return rc;
    pend.job = mine;
    pend.bucket = bucket;
    sb ^= 1;
    return 0;
  };
  // a TN that cannot fold (fp32 families, the edge-feature TN): pend and its own reduction in one
  // launch after it
  auto unfolded = [&](const RedJob& mine, int bucket,
                      int max_blocks = kReduceMaxBlocks) -> int {
    const int rc = flush(&mine, max_blocks);
    if (rc) return rc;
    if (bucket_events && bucket >= 0) HIP_RET(hipEventRecord(bucket_events[bucket], side));
    sb ^= 1;
    return 0;
  };


  // side: dwf, dbf; dzn; dW_n = dzn^T [x | s], db_n (forked before the main stream's readout NT:
  // deferring it behind a layer, or enqueuing the NT first, A/B -4..-14 %).  dzn is materialised
  // for the weight gradient only: the main stream's NT forms it inside the GEMM (LdActGrad).
  // the split-bf16 e-image TN takes dzn as the e-image the dzn kernel writes (dzn itself is
  // then never stored); the fp32 families read dzn
  const bool ro_b3 =
      fv.xp ? (b3tni_ok(LdConcat<4>{fv.xp, d.Fp, fv.a[D], Hp, d.Fp}, H, N) &&
               ((uintptr_t)fv.xp & 15) == 0)
            : (F % 4 == 0 && ((uintptr_t)b->x & 15) == 0 &&
               b3tni_ok(LdConcat<4>{b->x, F, fv.a[D], Hp, F}, H, N));
  const bool max_pool = fv.pool_arg != nullptr;  // global_max_pool (CGR_POOL_MAX)
  auto side_readout = [&]() -> int {
    {  // dwf = dy^T g, dbf: off the main chain (step A/B +0.8 %)
      ProfScope _p("head_bwd", side);
      HIP_RET(head_bwd(dy, fv.g, params[CGR_PARAM_FFN_W(D)], d.B, H, Hp, nullptr,
                       grads[CGR_PARAM_FFN_W(D)], grads[CGR_PARAM_FFN_B(D)], side));
    }
    if (!max_pool) {  // (max pooling: dzn and its image came from the main stream, below)
      ProfScope _p("readout_act_bwd", side);
      HIP_RET(readout_act_bwd(dy, params[CGR_PARAM_FFN_W(D)], iv.node_graph, fv.hn, fv.zn, N, H,
                              Hp, d.act, ro_b3 ? nullptr : dzn, ro_b3 ? img_side : nullptr,
                              side, fv.inv_cnt));
    }
    TnPlan p;
    float* sl = slabs[sb];
    float* bsl = bslabs[sb];
    float* gW = grads[CGR_PARAM_E2N_W(D)];
    float* gb = grads[CGR_PARAM_E2N_B(D)];
    // bucket 0 (edge_to_node, ffn): complete once this reduction has run
    if (fv.xp) {  // [xp | s] with x padded to Fp: the pad columns are skipped by the reduce
      const int Fp = d.Fp;
      LdPlain<4> al{dzn, Hp};
      LdConcat<4> bl{fv.xp, Fp, fv.a[D], Hp, Fp};
      const RedJob mine = make_red_job(TnPlan{}, sl, bsl, H, Fp + H, gW, F + H, 0, gb, F, Fp - F);
      if (ro_b3) {
        HIP_RET(b3tni_run("gemm_tn_wgrad_readout", img_side, bl, H, Fp + H, N, sl, bsl, true, &p,
                          side, kB3TnReadoutTarget, pend.job));
        RedJob j = mine;
        red_job_set_splits(j, p.splits);
        if (const int rc = fold(j, 0)) return rc;
      } else {
        if (tnr_x_ok(H, Fp + H, Fp, fv.xp)) {
          HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_readout", TnrRows{dzn, Hp},
                                  TnrConcat{fv.xp, Fp, fv.a[D], Hp, Fp}, H, Fp + H, N, sl, bsl,
                                  true, &p, side, kTnrReadoutTarget)));
        } else {
          HIP_RET(tn_gemm("gemm_tn_wgrad_readout", al, bl, H, Fp + H, N, sl, bsl, true, &p,
                          side));
        }
        RedJob j = mine;
        red_job_set_splits(j, p.splits);
        if (const int rc = unfolded(j, 0)) return rc;
      }
    } else {
      const LdConcat<4> bl4{b->x, F, fv.a[D], Hp, F};
      const RedJob mine = make_red_job(TnPlan{}, sl, bsl, H, F + H, gW, F + H, 0, gb);
      if (ro_b3) {
        HIP_RET(b3tni_run("gemm_tn_wgrad_readout", img_side, bl4, H, F + H, N, sl, bsl, true, &p,
                          side, kB3TnReadoutTarget, pend.job));
        RedJob j = mine;
        red_job_set_splits(j, p.splits);
        if (const int rc = fold(j, 0)) return rc;
      } else {
        if (F % 4 == 0 && tnr_x_ok(H, F + H, F, b->x)) {
          HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_readout", TnrRows{dzn, Hp},
                                  TnrConcat{b->x, F, fv.a[D], Hp, F}, H, F + H, N, sl, bsl, true,
                                  &p, side, kTnrReadoutTarget)));
        } else {
          hipError_t e = with_vec(vec_for(b->x, F, F), [&](auto VX) {
            LdPlain<4> al{dzn, Hp};
            LdConcat<decltype(VX)::value> bl{b->x, F, fv.a[D], Hp, F};
            return tn_gemm("gemm_tn_wgrad_readout", al, bl, H, F + H, N, sl, bsl, true, &p,
                           side);
          });
          HIP_RET(e);
        }
        RedJob j = mine;
        red_job_set_splits(j, p.splits);
        if (const int rc = unfolded(j, 0)) return rc;
      }
    }
    return 0;
  };
  // main: ds = dzn W_n[:, F:] = diag(dy[graph]) act'(zn) (diag(wf) W_n[:, F:]) -- the row factor in
  // the epilogue, the column factor in the weight image (gnn_fwd.hip), act' in the A loader
  auto readout_nt = [&]() -> int {
    ProfScope _p("gemm_nt_readout_bwd", st);
    const float* m = d.act == ACT_RELU ? fv.hn : fv.zn;
    const b3_u4* img = static_cast<const b3_u4*>(fv.b3rob);
    if (max_pool) {  // ds = dzn W_n[:, F:] with dzn materialised (its per-element arg-max mask is
                     // no row / column factor); the image is unscaled (gnn_fwd.hip)
      const EpStoreRowScale ep{ds, Hp, N, H, nullptr, iv.node_graph, nullptr, fv.inv_deg};
      HIP_RET(launch_b3nt(LdPlain<4>{dzn, Hp}, img, b3nt_cols(N, H), ep, N, H, H, st));
      return 0;
    }
    // (mean pooling: dy / graph count; mean aggregation: ds / in-degree, for dh_D = ds[dst])
    const EpStoreRowScale ep{ds, Hp, N, H, dy, iv.node_graph, fv.inv_cnt, fv.inv_deg};
    const B3Cols rc = b3nt_cols(N, H);  // the image's tiling (gnn_fwd.hip)
    // the activation derivative in the A loader, specialised per activation (main-loop code)
    if (d.act == ACT_RELU)
      HIP_RET(launch_b3nt(LdActGradT<ACT_RELU>{m, Hp, d.act}, img, rc, ep, N, H, H, st));
    else if (d.act == ACT_SILU)
      HIP_RET(launch_b3nt(LdActGradT<ACT_SILU>{m, Hp, d.act}, img, rc, ep, N, H, H, st));
    else
      HIP_RET(launch_b3nt(LdActGradT<-1>{m, Hp, d.act}, img, rc, ep, N, H, H, st));
    return 0;
  };
  // capture order: fork, side work, then the main NT.  Enqueuing the NT first (the fork point
  // recorded before it, the side work after -- same dependencies) moves the NT onto the forward's
  // hardware queue in a captured graph but puts the first layer NT beside the readout TN: r05
  // same-box A/B 344.0k -> 341.0k reactions/s (3 runs each, profiles/r05_ro_first_ab.txt)
  if (max_pool) {  // dzn (fp32 for the NT, and the TN's e-image) before the fork
    ProfScope _p("readout_act_bwd", st);
    HIP_RET(readout_act_bwd(dy, params[CGR_PARAM_FFN_W(D)], iv.node_graph, fv.hn, fv.zn, N, H, Hp,
                            d.act, dzn, ro_b3 ? img_side : nullptr, st, nullptr, fv.pool_arg, fv.g));
  }
  if (side != st) HIP_RET(fork_to(ss, st, side));
  if (const int rc = side_readout()) return rc;
  if (const int rc = readout_nt()) return rc;

  // learnable-skip partial-sum slots per layer (bwd_dsig_slots)
  const int nb = WL.dsig_blocks;
  // row tile of the fused layer-backward GEMMs: crossing segments accumulate in dag
  const int seg_rows = b3nt_rows(E, H);
  const B3Cols lcols = layer_cols(d);  // the layer images' tiling (gnn_fwd.hip)
  const int seg_cols = lcols.tiles;
  const int seg_tiles = bwd_seg_tiles(d);
  int* cnt = reinterpret_cast<int*>(ws + WL.cnt);
  const int spin = unpaired_spin_limit();  // CGR_UNPAIRED_SPIN_LIMIT (debug knob), per call
  float* part = reinterpret_cast<float*>(ws + WL.part);
  auto layer_args = [&](int l) {
    uint32_t thresh;
    float scale;
    dropout_params(dropout_p, training, l, &thresh, &scale);
    LayerBwdArgs la{};
    la.ds = ds;
    la.dm = dm;
    la.dst_s = iv.dst_s;
    la.rev_s = iv.rev_s;
    la.hnext = fv.h[l + 1];
    la.pre = fv.pre[l + 1];
    la.h0 = fv.h[0];
    la.sigma = d.learnable_skip ? params[CGR_PARAM_SKIP(D, l)] : nullptr;
    la.seed = iv.rng;  // the key the forward used (arena)
    la.thresh = thresh;
    la.scale = scale;
    la.layer = l;
    la.act = d.act;
    la.E = E;
    la.H = H;
    la.Hp = Hp;
    la.dpre = dpre(l);
    la.dsig_part = d.learnable_skip ? dsig_part + (int64_t)l * nb : nullptr;
    return la;
  };
  // the top layer's weight gradient on the split-bf16 e-image TN takes dpre_{D-1}'s e-image from
  // the activation kernel that writes dpre_{D-1} (no e-image pass over it).  (The layers below
  // keep the e-image pass: written by the fused layer-backward GEMM's epilogue it cost each such
  // launch 10 us, step 0.755 -> 0.769 ms, profiles/r05_rejected_epilogue_eimage_*.  Against
  // the top layer's pass on the side stream: same-box A/B 341.6k vs 341.1k reactions/s,
  // profiles/r05_ab2_top_eimage_fused_vs_side.txt.)
  const bool top_b3 =
      D > 0 && b3tni_ok(LdGatherDiff<false>{fv.a[D - 1], fv.h[D - 1], iv.src_s, iv.rev_s, Hp}, H, E);
  if (D > 0) {  // top layer: dh_D = ds[dst]
    ProfScope _p("layer_act_bwd", st);
    LayerBwdArgs la = layer_args(D - 1);
    la.dag = dag_of(D - 1);
    la.cnt = cnt;
    la.cnt_nodes = N;
    la.cnt_tiles = seg_cols;
    la.tile_rows = seg_rows;
    HIP_RET(layer_act_bwd(la, nb, top_b3 ? img_top : nullptr, st));
  }
  auto edge_args = [&]() {
    LayerBwdArgs le{};
    le.dm = dm;
    le.rev_s = iv.rev_s;
    le.h0 = fv.h[0];
    le.pre = fv.pre[0];
    le.act = d.act;
    le.E = E;
    le.H = H;
    le.Hp = Hp;
    le.dh0 = dh0;
    le.dpre = dh0;  // dpre0 is written in place of dh0 (the buffer it names)
    le.dpre_all = dpre(0);
    le.dpre_stride = (int64_t)E * Hp;
    le.nlayers = D;
    for (int k = 0; k < D; ++k) le.sig[k] = d.learnable_skip ? params[CGR_PARAM_SKIP(D, k)] : nullptr;
    return le;
  };
  // edge init: dpre0 = (dh0 + dh_0) * act'(pre0), dh0 summed from the layers' dpre buffers,
  // written to the dh0 buffer
  float* dpre0 = dh0;
  for (int l = D - 1; l >= 0; --l) {
    float* dp = dpre(l);  // written by the previous iteration's fused kernel (or just above)
    // main: dm = dpre W_l.  The fork point is recorded before the NT is enqueued and the side
    // work after it: same dependencies, but a captured graph then keeps the main chain on one
    // hardware queue (A/B 1.283 -> 1.263 ms; DESIGN.md §9 "Stream order")
    hipEvent_t fork_ev = nullptr;
    if (side != st) HIP_RET(record_point(ss, st, &fork_ev));
    // dm = dpre_l W_l with the layer below's activation backward (or the edge init's) in the
    // epilogue: rows gathered through rev, dst segments summed in the tile (ep_bwd.hpp)
    const LayerBwdArgs lb = l > 0 ? layer_args(l - 1) : edge_args();
    {
      ProfScope _p("gemm_nt_layer_bwd_seg", st);
      const LdGatherRows al{dp, iv.rev_s, Hp};
      const b3_u4* img = static_cast<const b3_u4*>(fv.b3lb[l]);
      float* dg = dag_of(l);
      float* dgn = l > 0 ? dag_of(l - 1) : nullptr;
      int* gcnt = cnt + (int64_t)N * seg_cols + l;  // this launch's unpaired grid counter
      if (l > 0)
        HIP_RET(launch_b3nt(al, img, lcols,
                            EpLayerBwdSeg<false>{lb, dm, iv.dst_s, iv.dst_ptr, iv.src_list,
                                                 iv.src_ptr, dg, dgn, part, cnt, iv.status, E, H, N,
                                                 seg_cols, gcnt, ss->dev_err, spin, fv.inv_deg},
                            E, H, H, st));
      else
        HIP_RET(launch_b3nt(al, img, lcols,
                            EpLayerBwdSeg<true>{lb, dm, iv.dst_s, iv.dst_ptr, iv.src_list,
                                                iv.src_ptr, dg, dgn, part, cnt, iv.status, E, H, N,
                                                seg_cols, gcnt, ss->dev_err, spin, fv.inv_deg},
                            E, H, H, st));
    }
    if (fork_ev) HIP_RET(hipStreamWaitEvent(side, fork_ev, 0));
    {  // side: dW_l = dpre^T m_l, db_l = colsum(dpre); the previous weight gradient's slabs are
       // reduced in the TN's prologue, this one's by the next TN (bucket D - l complete then)
      LdPlain<4> al{dp, Hp};
      LdGatherDiff<false> bl{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp};
      TnPlan p;
      float* sl = slabs[sb];
      float* bsl = bslabs[sb];
      RedJob mine = make_red_job(TnPlan{}, sl, bsl, H, H, grads[CGR_PARAM_CONV_W(l)], H, 0,
                                 grads[CGR_PARAM_CONV_B(l)]);
      const int tf = tnr_layer_frags(H);
      if (l == D - 1 && top_b3) {
        HIP_RET(b3tni_run("gemm_tn_wgrad_layer", img_top, bl, H, H, E, sl, bsl, true, &p, side,
                          kB3TnTarget, pend.job));
        red_job_set_splits(mine, p.splits);
        if (const int rc = fold(mine, D - l)) return rc;
      } else if (b3tni_ok(bl, H, E)) {
        {
          ProfScope _p("eimage", side);
          HIP_RET(b3_eimage(dp, Hp, E, H, static_cast<b3_u4*>(img_side), side));
        }
        HIP_RET(b3tni_run("gemm_tn_wgrad_layer", img_side, bl, H, H, E, sl, bsl, true, &p, side,
                          kB3TnTarget, pend.job));
        red_job_set_splits(mine, p.splits);
        if (const int rc = fold(mine, D - l)) return rc;
      } else {
        if (tf == 5) {
          HIP_RET((tnr_gemm<5, 5>("gemm_tn_wgrad_layer", TnrRows{dp, Hp},
                                  TnrDiff{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp}, H, H, E, sl,
                                  bsl, true, &p, side)));
        } else if (tf == 4) {
          HIP_RET((tnr_gemm<4, 4>("gemm_tn_wgrad_layer", TnrRows{dp, Hp},
                                  TnrDiff{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp}, H, H, E, sl,
                                  bsl, true, &p, side)));
        } else {
          HIP_RET(tn_gemm("gemm_tn_wgrad_layer", al, bl, H, H, E, sl, bsl, true, &p, side));
        }
        red_job_set_splits(mine, p.splits);
        if (const int rc = unfolded(mine, D - l)) return rc;
      }
    }
  }
  float* gW0 = grads[CGR_PARAM_EDGE_INIT_W];
  float* gb0 = grads[CGR_PARAM_EDGE_INIT_B];
  // tail: the fork point is recorded here and the side work (edge-feature TN) enqueued after the
  // main tail, as in the layer loop (A/B -0.8 %)
  hipEvent_t tail_ev = nullptr;
  if (side != st) HIP_RET(record_point(ss, st, &tail_ev));
  auto edge_tn = [&]() -> int {
    if (Fe > 0) {  // dW0[:, F:] = dpre0^T e, db0
      if (tail_ev) HIP_RET(hipStreamWaitEvent(side, tail_ev, 0));
      LdPlain<4> al{dpre0, Hp};
      LdPlain<4> bl{fv.e_s, d.Fep};
      TnPlan p;
      float* sl = slabs[sb];
      float* bsl = bslabs[sb];
      HIP_RET(tn_gemm("gemm_tn_wgrad_edge", al, bl, H, Fe, E, sl, bsl, true, &p, side,
                      kEdgeTnTargetWorkgroups));
      // with the last layer's pending reduction, in one launch (bucket D + 1 is recorded at the
      // join below)
      // the last side-stream reduction: by the time it runs the main chain has ended (r05 trace:
      // 13.5 us on 256 blocks for 1,300 logical ones, the step's tail), so it takes the GPU
      return unfolded(make_red_job(p, sl, bsl, H, Fe, gW0, F + Fe, F, gb0), -1, 1 << 20);
    }
    return flush();
  };
  if (!tail_ev) {
    const int rc = edge_tn();
    if (rc) return rc;
  }
  if (F > 0) {  // main: dW0[:, :F] = Gs^T x, Gs = segsum_src(dpre0) (own slab: beside the side
                // stream's work)
    const float* xb = fv.xp ? fv.xp : b->x;
    const int64_t ldx = fv.xp ? d.Fp : F;
    TnPlan p;
    const int Fx = fv.xp ? d.Fp : F;  // x columns the GEMM covers (pad columns are zero)
    const LdPlain<4> gbl{xb, ldx};
    const bool b3 = ldx % 4 == 0 && ((uintptr_t)xb & 15) == 0 && b3tni_ok(gbl, H, N);
    if (b3) {  // Gs straight into the TN's e-image (never stored in fp32)
      ProfScope _p("segsum_src_bwd", st);
      HIP_RET(b3_segsum_eimage(dpre0, Hp, iv.src_list, iv.src_ptr, N, H,
                               static_cast<b3_u4*>(img_main), st));
    } else {
      ProfScope _p("segsum_src_bwd", st);
      HIP_RET(segment_sum(dpre0, Hp, iv.src_list, iv.src_ptr, N, Hp, Gs, Hp, st));
    }
    if (b3) {
      HIP_RET(b3tni_run("gemm_tn_wgrad_node", img_main, gbl, H, Fx, N, slab2, bslab2, Fe == 0, &p,
                        st, kB3TnNodeTarget));
      // the flat reduce: this one ends the backward's main chain
      HIP_RET(tn_reduce(p, slab2, bslab2, H, Fx, gW0, F + Fe, 0, Fe > 0 ? nullptr : gb0, st, F,
                        Fx - F, true));
    } else if (tnr_x_ok(H, Fx, ldx, xb)) {
      HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_node", TnrRows{Gs, Hp}, TnrRows{xb, ldx}, H, Fx, N,
                              slab2, bslab2, Fe == 0, &p, st, kTnrNodeTarget)));
      HIP_RET(tn_reduce(p, slab2, bslab2, H, Fx, gW0, F + Fe, 0, Fe > 0 ? nullptr : gb0, st, F,
                        Fx - F));
    } else {
      hipError_t e = with_vec(vec_for(xb, ldx, F), [&](auto VX) {
        LdPlain<4> al{Gs, Hp};
        LdPlain<decltype(VX)::value> bl{xb, ldx};
        return tn_gemm("gemm_tn_wgrad_node", al, bl, H, F, N, slab2, bslab2, Fe == 0, &p, st);
      });
      HIP_RET(e);
      HIP_RET(tn_reduce(p, slab2, bslab2, H, F, gW0, F + Fe, 0, Fe > 0 ? nullptr : gb0, st));
    }
  } else if (Fe == 0) {
    HIP_RET(hipMemsetAsync(gb0, 0, sizeof(float) * H, st));
  }
  if (tail_ev) {
    const int rc = edge_tn();
    if (rc) return rc;
  }

  if (d.learnable_skip) {
    ScalarReduceJobs sj{};
    for (int l = 0; l < D; ++l) {
      sj.out[l] = grads[CGR_PARAM_SKIP(D, l)];
      // the top layer's activation kernel fills all nb slots, the fused GEMMs two per workgroup
      sj.count[l] = l == D - 1 ? nb : 2 * seg_tiles;
    }
    sj.n = D;
    ProfScope _p("skip_grad_reduce", st);
    HIP_RET(reduce_partials(dsig_part, nb, sj, st));
  }
  if (const int rc = flush()) return rc;  // (nothing left unless an edge TN was not run)
  // join: every gradient is complete when the main stream reaches here
  HIP_RET(depend(ss, side, st));
  if (bucket_events) HIP_RET(hipEventRecord(bucket_events[D + 1], st));
  return 0;
}

// Input gradients (autograd's x.grad / edge_attr.grad for the reference, GNN.py:85-86,105-106):
// x enters edge_init through x[src] and edge_to_node through [x | s], edge_attr edge_init only:
//   dq0 = dpre0 W0                     (q0 = [x[src] | e], GNN.py:86)
//   dx  = segsum_src(dpre0) W0[:, :F] + dzn W_n[:, :F]  = [Gs | dzn] [W0x ; W_nx]
//   de  = dpre0 W0[:, F:]              (rows back to the caller's edge order through perm)
// dpre0 is what gnn_backward_impl left in the workspace's dh0 buffer; Gs and dzn are re-formed
// in fp32 (the backward keeps them as e-images only) and the stacked weight slices transposed
// into wxT, so both products are one fp32 MFMA NT launch each (gemm.hpp), exact-fp32 products.
int gnn_input_grads_impl(const Dims& d, const float* const* params, const void* arena,
                         const float* dy, void* workspace, float* dx, float* de, hipStream_t st) {
  const ArenaLayout L = arena_layout(d);
  const IndexView iv = index_view(const_cast<void*>(arena), L);
  const FloatView fv = float_view(const_cast<void*>(arena), L, d);
  const WorkspaceLayout WL = workspace_layout(d);
  char* ws = static_cast<char*>(workspace);
  const float* dpre0 = reinterpret_cast<const float*>(ws + WL.dh0);
  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  if (de && Fe > 0) {  // de = dpre0 W0e: B = W0[:, F:]^T, the forward's w0eT [Fe, Hp]
    ProfScope _p("input_grad_edge", st);
    const LdPlain<4> al{dpre0, Hp};
    const LdPlain<4> bl{fv.w0eT, Hp};
    const EpStorePermRows ep{de, Fe, E, Fe, iv.perm};
    HIP_RET(with_nt_rn(Fe, [&](auto RN) {
      return launch_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, E, Fe, H, st);
    }));
  }
  if (dx && F > 0) {
    float* Gs = reinterpret_cast<float*>(ws + WL.Gs);
    float* dzn = reinterpret_cast<float*>(ws + WL.dzn);
    float* wxT = reinterpret_cast<float*>(ws + WL.wxT);
    const int ldw = input_grad_ldw(H);
    {
      ProfScope _p("input_grad_prep", st);
      HIP_RET(segment_sum(dpre0, Hp, iv.src_list, iv.src_ptr, N, H, Gs, Hp, st));
      HIP_RET(readout_act_bwd(dy, params[CGR_PARAM_FFN_W(D)], iv.node_graph, fv.hn, fv.zn, N, H,
                              Hp, d.act, dzn, nullptr, st, fv.inv_cnt, fv.pool_arg, fv.g));
      TransposeJobs tj{};  // wxT [F, ldw] = [W0[:, :F]^T | W_n[:, :F]^T]
      tj.job[0] = TransposeJob{params[CGR_PARAM_EDGE_INIT_W], F + Fe, 0, wxT, ldw, H, F};
      tj.job[1] = TransposeJob{params[CGR_PARAM_E2N_W(D)], F + H, 0, wxT + H, ldw, H, F};
      tj.n = 2;
      HIP_RET(transpose_batch(tj, st));
    }
    ProfScope _p("input_grad_node", st);
    const LdPlain<4> bl{wxT, ldw};
    const EpStore ep{dx, F, N, F, nullptr};
    // [Gs | dzn] rows: the concat boundary H must not split a VEC-wide chunk
    HIP_RET(with_vec(H % 4 == 0 ? 4 : (H % 2 == 0 ? 2 : 1), [&](auto V) {
      const LdConcat<decltype(V)::value> al{Gs, Hp, dzn, Hp, H};
      return with_nt_rn(F, [&](auto RN) {
        return launch_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, N, F, 2 * H, st);
      });
    }));
  }
  return 0;
}

}  // namespace cgr
