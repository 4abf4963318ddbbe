// GNN.forward (GNN.py:76-110) as HIP launches on the caller's stream plus one side stream.
//
//   side:  [P | Q] = x [W0[:, :F]; W_n[:, :F]]^T   one GEMM reads x once; P = node-level half of
//          edge init (N*F*H instead of E*F*H FLOPs), Q = x-part of the readout; runs while the
//          main stream does the graph bookkeeping (it needs neither)
//   main:  graph prep ; join
//          h0  = act(P[src] + e W0e^T + b0)                                     (GNN.py:85-87)
//          a0  = segsum_dst(h0)                                                 (GNN.py:134)
//          for l: h_{l+1} = drop(act((a_l[src] - h_l[rev]) W_l^T + b_l + s_l h0))
//                 a_{l+1} = segsum_dst(h_{l+1})                            (GNN.py:90-102, 134)
//          hn  = act(a_D W_n[:, F:]^T + Q + b_n)   (a_D IS the readout aggregate s, GNN.py:105-107)
//          y   = (sum_{v in graph} hn[v]) . wf + bf                             (GNN.py:110)
// The reference's discarded readout GEMM (GNN.py:105 -> lin(...) at :141) is not executed.
#include "dispatch.hpp"
#include "epilogues.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"
#include "profiling.hpp"
#include "streams.hpp"

namespace cgr {

static void dropout_consts(const float* dropout_p, int training, int l, uint32_t* thresh,
                           float* scale) {
  *thresh = 0;
  *scale = 1.f;
  if (!(training & CGR_TRAIN_DROPOUT) || dropout_p == nullptr) return;
  const double p = dropout_p[l];
  if (p <= 0.0) return;
  if (p >= 1.0) {
    *thresh = 0xFFFFFFFFu;
    *scale = 0.f;
    return;
  }
  double t = p * 4294967296.0;
  if (t > 4294967295.0) t = 4294967295.0;
  *thresh = (uint32_t)t;
  if (*thresh == 0) *thresh = 1;
  *scale = (float)(1.0 / (1.0 - p));
}

void dropout_params(const float* dropout_p, int training, int l, uint32_t* thresh, float* scale) {
  dropout_consts(dropout_p, training, l, thresh, scale);
}

// every forward weight image (x-GEMM, readout, layers) into `images` (ImageLayout), one launch
hipError_t pack_forward_images(const Dims& d, const float* const* params, const ImageLayout& IL,
                               void* images, hipStream_t st) {
  const int H = d.H, F = d.F, Fe = d.Fe, D = d.D;
  const float* W0 = params[CGR_PARAM_EDGE_INIT_W];
  const float* Wn = params[CGR_PARAM_E2N_W(D)];
  char* base = static_cast<char*>(images);
  B3PackJobs pj{};
  hipError_t e;
  if (F > 0) {
    b3_u4* ximg = reinterpret_cast<b3_u4*>(base + IL.b3x);
    const B3Cols cx = b3_cols(2 * H);
    if ((e = b3_pack_add(pj, B3PackJob{W0, F + Fe, 1, ximg, 0, H, H, F, cx.nimg, b3_nk(F)}, st)))
      return e;
    if ((e = b3_pack_add(pj, B3PackJob{Wn, F + H, 1, ximg, H, cx.nimg - H, H, F, cx.nimg,
                                       b3_nk(F)}, st)))
      return e;
  }
  if ((e = b3_pack_add(pj, b3_job(Wn + F, F + H, 1, H, H, base + IL.b3rof), st))) return e;
  for (int l = 0; l < D; ++l)
    if ((e = b3_pack_add(pj, b3_job(params[CGR_PARAM_CONV_W(l)], H, 1, H, H, base + IL.b3lf[l]),
                         st)))
      return e;
  return b3_pack(pj, st);
}

int gnn_forward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, uint64_t* rng_counter, int training,
                     void* arena, float* y, hipStream_t st, const FwdMode& mode) {
  const ArenaLayout L = mode.eval ? eval_arena_layout(d) : arena_layout(d);
  const IndexView iv = index_view(arena, L);
  FloatView fv = float_view(arena, L, d);
  // forward weight images pre-packed by the caller (cgr_gnn_pack_images), or packed below into
  // the arena by this call
  const bool caller_images = mode.eval && mode.images != nullptr;
  if (caller_images) {
    const ImageLayout IL = image_layout(d);
    char* im = static_cast<char*>(const_cast<void*>(mode.images));
    fv.b3x = d.F > 0 ? im + IL.b3x : nullptr;
    fv.b3rof = im + IL.b3rof;
    for (int l = 0; l < d.D; ++l) fv.b3lf[l] = im + IL.b3lf[l];
  }
  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  const float* W0 = params[CGR_PARAM_EDGE_INIT_W];
  const float* b0 = params[CGR_PARAM_EDGE_INIT_B];
  const float* Wn = params[CGR_PARAM_E2N_W(D)];
  const float* bn = params[CGR_PARAM_E2N_B(D)];

  // dropout key of this forward -> arena (the backward and every epilogue read it from there;
  // computed by the first graph-prep kernel, see PrepArgs)
  bool any_dropout = false;
  for (int l = 0; l < D; ++l) {
    uint32_t t;
    float s;
    dropout_consts(dropout_p, training, l, &t, &s);
    any_dropout = any_dropout || t != 0;
  }

  SideStreams* ss = side_streams(st);
  if (!ss) return CGR_ERR_HIP;
  std::lock_guard<std::mutex> ss_lock(ss->mu);
  const bool packs = !caller_images;
  // column tilings: the x-GEMM's and the readout GEMMs' grid-filling over this batch's N rows
  // (b3nt_cols) for the images packed here, b3_cols for batch-independent caller images
  // (cgr_gnn_pack_images); the layer GEMMs' layer_cols
  const B3Cols xcols = caller_images ? b3_cols(2 * H) : b3nt_cols(N, 2 * H);
  const B3Cols rcols = caller_images ? b3_cols(H) : b3nt_cols(N, H);
  const B3Cols lcols = caller_images ? b3_cols(H) : layer_cols(d);
  // small batches: the graph bookkeeping as the x-GEMM launch's extra workgroup (prep_one.hpp)
  // on a CU no tile takes -- the whole forward start on one queue, no fork / join (each costs
  // ~5-10 us in a captured graph); else graph_prep.hip's launches on the caller's stream beside
  // the x chain on the side stream
  const bool one_prep =
      F > 0 && packs && !prep_split() && prep_one_fits(N, E, d.Fep) &&
      b3nt_side_fits(N, 2 * H, xcols, (size_t)prep_one_lds_ints(N, E, d.B) * 4);
  // instrumented (profiling) runs stay serial so per-kernel event times are isolated durations
  hipStream_t side = (one_prep || prof_enabled() || single_stream()) ? st : ss->side;
  if (side != st) HIP_RET(fork_to(ss, st, side));

  // x rows padded to 16 bytes (F % 4 != 0): the x-GEMM and both x-part weight gradients read xp
  // with 16-byte loads; the padding, W0[:, F:]^T (edge init) and the zeroing of the bookkeeping's
  // counters ride in the pack launches when this forward packs its own images
  const float* xa = b->x;
  int64_t ldx = F;
  B3PackRiders rx{}, rm{};
  if (fv.xp) {
    if (packs && F > 0) {
      rx.p_src = b->x;
      rx.p_dst = fv.xp;
      rx.p_rows = N;
      rx.p_F = F;
      rx.p_ld = (int)d.Fp;
    } else {
      ProfScope _p("pad_x", side);
      HIP_RET(pad_rows(b->x, N, F, fv.xp, d.Fp, side));
    }
    xa = fv.xp;
    ldx = d.Fp;
  }
  if (Fe > 0 && packs) {
    rm.t_src = W0 + F;
    rm.t_ld_src = F + Fe;
    rm.t_dst = fv.w0eT;
    rm.t_ld_dst = Hp;
    rm.t_rows = H;
    rm.t_cols = Fe;
  } else if (Fe > 0) {
    ProfScope _p("weight_transpose", st);
    TransposeJobs tj{};
    tj.job[0] = TransposeJob{W0, F + Fe, F, fv.w0eT, Hp, H, Fe};
    tj.n = 1;
    HIP_RET(transpose_batch(tj, st));
  }
  // split-bf16 weight images of every NT GEMM of this step: the x-GEMM's on the x chain's
  // stream, the layer / readout images (forward, and backward unless this is an eval forward) on
  // the caller's stream ahead of graph prep (one launch when both are the same stream)
  if (packs) {
    ProfScope _p("weight_pack", st);
    B3PackJobs pj{}, pm{};
    if (F > 0) {
      HIP_RET(b3_pack_add(pj, B3PackJob{W0, F + Fe, 1, static_cast<b3_u4*>(fv.b3x), 0, H, H, F,
                                        xcols.nimg, b3_nk(F)}, side));
      HIP_RET(b3_pack_add(pj, B3PackJob{Wn, F + H, 1, static_cast<b3_u4*>(fv.b3x), H,
                                        xcols.nimg - H, H, F, xcols.nimg, b3_nk(F)}, side));
    }
    HIP_RET(b3_pack_add(pm, b3_job(Wn + F, F + H, 1, H, H, fv.b3rof, rcols), st));
    for (int l = 0; l < D; ++l)
      HIP_RET(b3_pack_add(pm, b3_job(params[CGR_PARAM_CONV_W(l)], H, 1, H, H, fv.b3lf[l], lcols),
                          st));
    if (!mode.eval && (training & CGR_TRAIN_FOR_BACKWARD)) {  // the backward NT GEMMs' W^T images
      B3PackJob rob = b3_job(Wn + F, 1, F + H, H, H, fv.b3rob, rcols);  // scaled by wf: LdActGrad
      // (max pooling: the readout backward NT reads the materialised dzn, wf already in it)
      if (d.pool != CGR_POOL_MAX) rob.kscale = params[CGR_PARAM_FFN_W(D)];
      HIP_RET(b3_pack_add(pm, rob, st));
      for (int l = 0; l < D; ++l)
        HIP_RET(b3_pack_add(pm, b3_job(params[CGR_PARAM_CONV_W(l)], 1, H, H, H, fv.b3lb[l], lcols),
                            st));
    }
    rm.z_dst = iv.zero_block;
    rm.z_u4 = (int64_t)(iv.zero_bytes / 16);
    if (side == st) {
      for (int j = 0; j < pj.n; ++j) HIP_RET(b3_pack_add(pm, pj.job[j], st));
      rm.p_src = rx.p_src;
      rm.p_dst = rx.p_dst;
      rm.p_rows = rx.p_rows;
      rm.p_F = rx.p_F;
      rm.p_ld = rx.p_ld;
    } else {
      HIP_RET(b3_pack(pj, side, &rx));
    }
    HIP_RET(b3_pack(pm, st, &rm));
  }
  if (F > 0) {
    ProfScope _p("gemm_nt_x", side);
    // over padded x the GEMM runs to K = Fp (zero columns against the image's zero rows), the
    // unmasked form, when that adds no k step to the image
    const int Kx = (xa == fv.xp && fv.xp && b3_nk(d.Fp) == b3_nk(F)) ? (int)d.Fp : F;
    EpSplit2 ep{fv.P, fv.Q, Hp, N, H};
    if (one_prep) {
      ep.side_on = 1;
      PrepOne& po = ep.prep;
      po.ei = b->edge_index;
      po.batch = b->batch;
      po.gptr64 = b->graph_ptr;
      po.ea = b->edge_attr;
      po.E = E;
      po.N = N;
      po.B = (int)d.B;
      po.Fe = Fe;
      po.Fep = (int)d.Fep;
      po.src_c = iv.src_c;
      po.dst_c = iv.dst_c;
      po.perm = iv.perm;
      po.inv = iv.inv;
      po.src_s = iv.src_s;
      po.dst_s = iv.dst_s;
      po.rev_s = iv.rev_s;
      po.src_list = iv.src_list;
      po.dst_ptr = iv.dst_ptr;
      po.src_ptr = iv.src_ptr;
      po.graph_ptr = iv.graph_ptr;
      po.node_graph = iv.node_graph;
      po.status = iv.status;
      po.e_s = fv.e_s;
      po.want_key = any_dropout ? 1 : 0;
      po.seed = seed;
      po.counter = rng_counter;
      po.key_out = iv.rng;
    }
    hipError_t e = with_vec(vec_for(xa, ldx, F), [&](auto VX) {
      LdPlain<decltype(VX)::value> al{xa, ldx};
      return launch_b3nt(al, static_cast<const b3_u4*>(fv.b3x), xcols, ep, N, 2 * H, Kx, side);
    });
    HIP_RET(e);
  } else {
    HIP_RET(hipMemsetAsync(fv.P, 0, sizeof(float) * (size_t)N * Hp, side));
    HIP_RET(hipMemsetAsync(fv.Q, 0, sizeof(float) * (size_t)N * Hp, side));
  }
  if (!one_prep) {
    hipEvent_t p_ready = nullptr;  // P and Q written
    if (side != st) HIP_RET(record_point(ss, side, &p_ready));
    // main stream: graph bookkeeping, then join
    {
      ProfScope _p("graph_prep", st);
      PrepArgs pa{b->edge_index, b->batch, b->graph_ptr, b->edge_attr, d.N, d.E, d.B,
                  d.Fe,          d.Fep,   iv,           fv.e_s};
      pa.want_key = any_dropout;
      pa.zeroed = packs;
      pa.seed = seed;
      pa.rng_counter = rng_counter;
      int rc = cgr_graph_prep_impl(pa, st);
      if (rc) return rc;
    }
    if (p_ready) HIP_RET(hipStreamWaitEvent(st, p_ready, 0));
  }

  // mean aggregation / pooling (DMPNNConv(aggr="mean"), global_mean_pool): the per-node and
  // per-graph factors once the CSRs exist; every a_l is formed as the sum and scaled in place
  // right after the launch that completes it (scale_rows), before anything reads it
  if (fv.inv_deg || fv.inv_cnt) {
    ProfScope _p("mean_scales", st);
    HIP_RET(mean_scales(iv.dst_ptr, N, iv.graph_ptr, d.B, fv.inv_deg, fv.inv_cnt, st));
  }
  auto mean_of = [&](float* a) -> int {
    if (!fv.inv_deg) return 0;
    ProfScope _p("mean_aggr", st);
    HIP_RET(scale_rows(a, Hp, N, fv.inv_deg, st));
    return 0;
  };

  // the layer GEMMs sum their dst segments in the epilogue (EpLayerSeg: one gather -> MLP ->
  // segmented-reduce launch per layer) when the fused edge init zeroes what they accumulate
  const bool fused_seg = Hp <= 512;
  if (Hp <= 512) {  // edge init + a_0 in one pass
    ProfScope _p("edge_init_seg_fwd", st);
    // the entries the layer epilogues accumulate: every a_l (training), or the first two
    // buffers of the eval ring (each layer l >= 1 re-zeroes a_{l+2}'s, see below)
    SegZero z{};
    z.n = mode.eval ? (D < 2 ? D : 2) : D;
    z.tile_rows = b3nt_rows(E, H);
    for (int l = 0; l < z.n; ++l) z.a[l] = fv.a[l + 1];
    HIP_RET(edge_init_segsum_fwd(fv.P, iv.src_s, fv.e_s, Fe, d.Fep, fv.w0eT, b0, iv.dst_ptr, N,
                                 H, Hp, d.act, fv.h[0], fv.pre[0], fv.a[0], st, &z));
  } else {
    {
      ProfScope _p("edge_init_fwd", st);
      HIP_RET(edge_init_fwd(fv.P, iv.src_s, fv.e_s, Fe, d.Fep, fv.w0eT, b0, E, H, Hp, d.act,
                            fv.h[0], fv.pre[0], st));
    }
    ProfScope _p("segsum_dst_fwd", st);
    HIP_RET(segment_sum(fv.h[0], Hp, nullptr, iv.dst_ptr, N, Hp, fv.a[0], Hp, st));
  }
  if (const int rc = mean_of(fv.a[0])) return rc;

  for (int l = 0; l < D; ++l) {
    uint32_t thresh;
    float scale;
    dropout_consts(dropout_p, training, l, &thresh, &scale);
    EpLayer ep{params[CGR_PARAM_CONV_B(l)],
               d.learnable_skip ? params[CGR_PARAM_SKIP(D, l)] : nullptr,
               fv.h[0],  fv.h[l + 1],
               fv.pre[l + 1], Hp,
               E,        H,
               d.act,    thresh,
               scale,    iv.rng,
               l};
    LdGatherDiff<false> al{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp};
    const b3_u4* img = static_cast<const b3_u4*>(fv.b3lf[l]);
    if (fused_seg) {  // h_{l+1} and a_{l+1} = segsum_dst(h_{l+1}) from one launch
      ProfScope _p("gemm_nt_layer_seg_fwd", st);
      // eval ring: a_{l+2} reuses a_{l-1}'s buffer, free once layer l-1 read it; this layer
      // zeroes the entries layer l+1 will accumulate there
      float* znext = (mode.eval && l >= 1 && l + 2 <= D) ? fv.a[l + 2] : nullptr;
      HIP_RET(launch_b3nt(al, img, lcols,
                          EpLayerSeg{ep, iv.dst_s, fv.a[l + 1], Hp, znext, iv.dst_ptr, iv.fpart,
                                     iv.fcnt, lcols.tiles},
                          E, H, H, st));
    } else {
      {
        ProfScope _p("gemm_nt_layer_fwd", st);
        HIP_RET(launch_b3nt(al, img, lcols, ep, E, H, H, st));
      }
      ProfScope _p2("segsum_dst_fwd", st);
      HIP_RET(segment_sum(fv.h[l + 1], Hp, nullptr, iv.dst_ptr, N, Hp, fv.a[l + 1], Hp, st));
    }
    if (const int rc = mean_of(fv.a[l + 1])) return rc;
  }

  // readout: hn = act(s W_n[:, F:]^T + Q + b_n), s = a_D
  {
    ProfScope _p("gemm_nt_readout_fwd", st);
    EpReadoutQ ep{bn, fv.Q, fv.hn, fv.zn, Hp, N, H, d.act};
    HIP_RET(launch_b3nt(LdPlain<4>{fv.a[D], Hp}, static_cast<const b3_u4*>(fv.b3rof), rcols, ep,
                        N, H, H, st));
  }
  ProfScope _p("pool_head_fwd", st);
  HIP_RET(pool_head_fwd(fv.hn, Hp, iv.graph_ptr, d.B, H, params[CGR_PARAM_FFN_W(D)],
                        params[CGR_PARAM_FFN_B(D)], fv.g, y, st, fv.inv_cnt, fv.pool_arg,
                        b->batch == nullptr));
  return 0;
}

}  // namespace cgr
