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

#ifndef CGR_FUSED_SEGSUM
#define CGR_FUSED_SEGSUM 0  // layer scatter-add in the layer GEMM's epilogue + a boundary fixup
                            // (bitwise the unfused sums; the forward 5 us slower in the step:
                            // the epilogue's segment pass costs more than the launch it saves)
#endif
#ifndef CGR_B3_PACK_MAIN
#define CGR_B3_PACK_MAIN 1  // layer / readout weight images packed on the caller's stream
#endif
#ifndef CGR_B3_SPLIT_X
#define CGR_B3_SPLIT_X 0  // A/B: split 1.5 % slower (the Q half and the backward images packed beside the
                          // layers slow them and the edge init more than the 30 us it takes off)
#endif
#ifndef CGR_SPLIT_XGEMM
#define CGR_SPLIT_XGEMM 0
#endif
#ifndef CGR_PAD_ON_MAIN
#define CGR_PAD_ON_MAIN 0
#endif
#ifndef CGR_PAD_WITH_PACK
#define CGR_PAD_WITH_PACK 0  // 1: x padding in the same launch as the x-GEMM image pack: A/B -5.5 %
                             // (21.6 us for the merged launch vs 12.7 + 7.3, and a queue reshuffle)
#endif
#ifndef CGR_B3_XCOPY
#define CGR_B3_XCOPY 0  // 1: x-GEMM on unpadded x (8-byte loads) writes the padded copy xp itself
                        // (no padding pass); A/B 270.3k -> 251.7k rxn/s (-7 %), off
#endif

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

int gnn_forward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                     const float* dropout_p, uint64_t seed, uint64_t* rng_counter, int training,
                     void* arena, float* y, hipStream_t st) {
  const ArenaLayout L = arena_layout(d);
  const IndexView iv = index_view(arena, L);
  const FloatView fv = float_view(arena, L, d);
  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  const float* W0 = params[CGR_PARAM_EDGE_INIT_W];
  const float* b0 = params[CGR_PARAM_EDGE_INIT_B];
  const float* Wn = params[CGR_PARAM_E2N_W(D)];
  const float* bn = params[CGR_PARAM_E2N_B(D)];

  // dropout key of this forward -> arena (the backward and every epilogue read it from there)
  bool any_dropout = false;
  for (int l = 0; l < D; ++l) {
    uint32_t t;
    float s;
    dropout_consts(dropout_p, training, l, &t, &s);
    any_dropout = any_dropout || t != 0;
  }
  // (the key is computed by the first graph-prep kernel, see PrepArgs)

#ifndef CGR_WT_ON_MAIN
#define CGR_WT_ON_MAIN 1  // A/B: -0.6 % (the readout no longer joins the side stream)
#endif
#ifndef CGR_W0E_ON_MAIN
#define CGR_W0E_ON_MAIN 1  // r02 (split-bf16): 1 258.0k vs 0 256.6k rxn/s (A/B, 3 rounds, within noise); r01: 0 (x-GEMM stream) 1.2234 ms, 1 1.2278, 2 1.2305
#endif
  SideStreams* ss = side_streams(st);
  if (!ss) return CGR_ERR_HIP;
  std::lock_guard<std::mutex> ss_lock(ss->mu);
  // instrumented (profiling) runs stay serial so per-kernel event times are isolated durations
  hipStream_t side = (prof_enabled() || single_stream()) ? st : ss->side;
  HIP_RET(fork_to(ss, st, side));

  // ---- side stream: x padding, edge-feature weight slice, x-GEMM(s), backward transposes ----
  // x rows padded to 16 bytes (F % 4 != 0): the x-GEMM here and both x-part weight gradients
  // read xp with 16-byte loads
  const float* xa = b->x;
  int64_t ldx = F;
  // CGR_B3_XCOPY: no padding pass; the x-GEMM reads x with 8-byte loads and writes xp itself
  const bool xcopy = CGR_B3 && CGR_B3_XCOPY && !CGR_B3_SPLIT_X && !CGR_SPLIT_XGEMM && fv.xp &&
                     vec_for(b->x, F, F) >= 2;
  // CGR_PAD_WITH_PACK: the padding pass rides in the x-image pack launch below
  const bool pad_with_pack = CGR_PAD_WITH_PACK && CGR_B3 && !prof_enabled();
  bool pad_pending = false;
#if !CGR_PAD_ON_MAIN
  if (fv.xp && !xcopy) {
    if (pad_with_pack) {
      pad_pending = true;
    } else {
      ProfScope _p("pad_x", side);
      HIP_RET(pad_rows(b->x, N, F, fv.xp, d.Fp, side));
    }
    xa = fv.xp;
    ldx = d.Fp;
  }
#endif
  // W0[:, F:]^T for the edge init: on the x-GEMM's stream (0), ahead of graph prep on the
  // caller's stream (1), or on the caller's stream after graph prep (2)
  auto w0e_transpose = [&](hipStream_t s) -> hipError_t {
    if (Fe <= 0) return hipSuccess;
    ProfScope _p("weight_transpose", s);
    TransposeJobs tj{};
    tj.job[0] = TransposeJob{W0, F + Fe, F, fv.w0eT, Hp, H, Fe};
    tj.n = 1;
    return transpose_batch(tj, s);
  };
  if (CGR_W0E_ON_MAIN != 2) HIP_RET(w0e_transpose(CGR_W0E_ON_MAIN ? st : side));
  // split x-GEMM (CGR_B3_SPLIT_X): P = x W0[:, :F]^T first (the edge init waits for it), then
  // Q = x W_n[:, :F]^T beside the layers (only the readout reads it), from two images in b3x
  const bool split_x = CGR_B3 && CGR_B3_SPLIT_X && F > 0;
  b3_u4* ximg = static_cast<b3_u4*>(fv.b3x);
  b3_u4* ximg_q = split_x ? ximg + b3_img_u4(H, F) : nullptr;
  B3PackJobs pack_main{};
  if (CGR_B3) {  // split-bf16 weight images of every NT GEMM of this step (forward and backward)
    ProfScope _p("weight_pack", side);
    B3PackJobs pj{};
    if (split_x) {
      HIP_RET(b3_pack_add(pj, b3_job(W0, F + Fe, 1, H, F, ximg), side));
      HIP_RET(b3_pack_add(pj, b3_job(Wn, F + H, 1, H, F, ximg_q), side));
    } else if (F > 0) {
      const B3Cols cx = b3_cols(2 * H);
      HIP_RET(b3_pack_add(pj, B3PackJob{W0, F + Fe, 1, ximg, 0, H, H, F, cx.nimg, b3_nk(F)}, side));
      HIP_RET(b3_pack_add(
          pj, B3PackJob{Wn, F + H, 1, ximg, H, cx.nimg - H, H, F, cx.nimg, b3_nk(F)}, side));
    }
    // the layer / readout images: on the caller's stream ahead of graph prep (that chain has
    // slack beside the x-GEMM chain, and the layers that read them run there), or here
    B3PackJobs pm{};
    hipStream_t ms = CGR_B3_PACK_MAIN ? st : side;
    B3PackJobs& pl = CGR_B3_PACK_MAIN ? pm : pj;
    HIP_RET(b3_pack_add(pl, b3_job(Wn + F, F + H, 1, H, H, fv.b3rof), ms));
    for (int l = 0; l < D; ++l)
      HIP_RET(b3_pack_add(pl, b3_job(params[CGR_PARAM_CONV_W(l)], H, 1, H, H, fv.b3lf[l]), ms));
    if (!split_x) {  // backward images in the same launch
      HIP_RET(b3_pack_add(pl, b3_job(Wn + F, 1, F + H, H, H, fv.b3rob), ms));
      for (int l = 0; l < D; ++l)
        HIP_RET(b3_pack_add(pl, b3_job(params[CGR_PARAM_CONV_W(l)], 1, H, H, H, fv.b3lb[l]), ms));
    }
    if (pad_pending)
      HIP_RET(b3_pack_pad(pj, B3PadJob{b->x, N, F, (int)d.Fp, fv.xp}, side));
    else
      HIP_RET(b3_pack(pj, side));
    pack_main = pm;
  }
  if (CGR_B3 && CGR_B3_PACK_MAIN) {  // (own scope: in instrumented runs both are the same stream)
    ProfScope _p("weight_pack", st);
    HIP_RET(b3_pack(pack_main, st));
  }
  hipEvent_t p_ready = nullptr;  // P (and, unless split, Q) written
  hipEvent_t q_ready = nullptr;  // split x-GEMM: Q and the backward images written
  if (split_x) {
    const int vx = vec_for(xa, ldx, F);
    for (int part = 0; part < 2; ++part) {
      ProfScope _p("gemm_nt_x", side);
      hipError_t e = with_vec(vx, [&](auto VX) {
        LdPlain<decltype(VX)::value> al{xa, ldx};
        EpStore ep{part == 0 ? fv.P : fv.Q, Hp, (int)N, H, nullptr};
        return launch_b3nt(al, part == 0 ? ximg : ximg_q, ep, N, H, F, side);
      });
      HIP_RET(e);
      if (part == 0) HIP_RET(record_point(ss, side, &p_ready));
    }
    {
      ProfScope _p("weight_pack", side);
      B3PackJobs pj{};
      HIP_RET(b3_pack_add(pj, b3_job(Wn + F, 1, F + H, H, H, fv.b3rob), side));
      for (int l = 0; l < D; ++l)
        HIP_RET(b3_pack_add(pj, b3_job(params[CGR_PARAM_CONV_W(l)], 1, H, H, H, fv.b3lb[l]), side));
      HIP_RET(b3_pack(pj, side));
    }
    HIP_RET(record_point(ss, side, &q_ready));
  } else if (F > 0) {
    int vb = vec_for(W0, F + Fe, F);
    const int vb2 = vec_for(Wn, F + H, F);
    vb = vb < vb2 ? vb : vb2;
    const int vx = vec_for(xa, ldx, F);
#if CGR_SPLIT_XGEMM
    // P first (edge init waits for it), Q = x W_n[:, :F]^T afterwards beside the layers
    for (int part = 0; part < 2; ++part) {
      ProfScope _p("gemm_nt_x", side);
      const float* Wb = part == 0 ? W0 : Wn;
      const int64_t ldw = part == 0 ? F + Fe : F + H;
      const int vw = vec_for(Wb, ldw, F);
      hipError_t e = with_vec(vx, [&](auto VX) {
        return with_vec(vw, [&](auto VW) {
          return with_nt_rn(H, [&](auto RN) {
            LdPlain<decltype(VX)::value> al{xa, ldx};
            LdPlain<decltype(VW)::value> bl{Wb, ldw};
            EpStore ep{part == 0 ? fv.P : fv.Q, Hp, N, H, nullptr};
            return launch_nt<4, 1, decltype(RN)::value, CGR_XGEMM_KT>(al, bl, ep, N, H, F, side);
          });
        });
      });
      HIP_RET(e);
      if (part == 0) HIP_RET(record_point(ss, side, &p_ready));
    }
    (void)vb;
#else
    if (CGR_B3) {
      ProfScope _p("gemm_nt_x", side);
      // over padded x the GEMM runs to K = Fp (zero columns against the image's zero rows),
      // the unmasked form, when that adds no k step to the image
      const int Kx = (xa == fv.xp && fv.xp && b3_nk(d.Fp) == b3_nk(F)) ? (int)d.Fp : F;
      hipError_t e = with_vec(vx, [&](auto VX) {
        LdPlain<decltype(VX)::value> al{xa, ldx};
        EpSplit2 ep{fv.P, fv.Q, Hp, N, H};
        if (xcopy)
          return launch_b3nt(al, static_cast<const b3_u4*>(fv.b3x), ep, N, 2 * H, Kx, side,
                             B3RowCopy{fv.xp, d.Fp, (int)d.Fp});
        return launch_b3nt(al, static_cast<const b3_u4*>(fv.b3x), ep, N, 2 * H, Kx, side);
      });
      HIP_RET(e);
    } else {
      ProfScope _p("gemm_nt_x", side);
      hipError_t e = with_vec(vx, [&](auto VX) {
        return with_vec(vb, [&](auto VB) {
          return with_nt_rn(2 * H, [&](auto RN) {
            LdPlain<decltype(VX)::value> al{xa, ldx};
            LdTwoRows<decltype(VB)::value> bl{W0, F + Fe, Wn, F + H, H};
            EpSplit2 ep{fv.P, fv.Q, Hp, N, H};
            return launch_nt<4, 1, decltype(RN)::value, CGR_XGEMM_KT>(al, bl, ep, N, 2 * H, F,
                                                                      side);
          });
        });
      });
      HIP_RET(e);
    }
    HIP_RET(record_point(ss, side, &p_ready));
#endif
  } else {
    HIP_RET(hipMemsetAsync(fv.P, 0, sizeof(float) * (size_t)N * Hp, side));
    HIP_RET(hipMemsetAsync(fv.Q, 0, sizeof(float) * (size_t)N * Hp, side));
    HIP_RET(record_point(ss, side, &p_ready));
  }
  // W_l^T and W_n[:, F:]^T for the backward's NT GEMMs (arena), off the critical path: on the
  // side stream after the x-GEMM (joined before the readout), or (CGR_WT_ON_MAIN, merged x-GEMM)
  // on the caller's stream after graph prep, so that the side stream's last node is the x-GEMM
  // the edge init waits for anyway and the forward has no second join (every cross-queue
  // dependency in the captured graph costs 5-12 us)
  constexpr bool wt_main = CGR_WT_ON_MAIN && !CGR_SPLIT_XGEMM;  // (unused with CGR_B3: images)
  auto weight_transposes = [&](hipStream_t s) -> hipError_t {
    ProfScope _p("weight_transpose", s);
    const int64_t HHp = (int64_t)H * Hp;
    TransposeJobs tj{};
    for (int l = 0; l < D; ++l)
      tj.job[l] = TransposeJob{params[CGR_PARAM_CONV_W(l)], H, 0, fv.wT + l * HHp, Hp, H, H};
    tj.job[D] = TransposeJob{Wn, F + H, F, fv.wT + D * HHp, Hp, H, H};
    tj.n = D + 1;
    return transpose_batch(tj, s);
  };
  hipEvent_t side_done = nullptr;
  if (!wt_main && !CGR_B3) {
    HIP_RET(weight_transposes(side));
    HIP_RET(record_point(ss, side, &side_done));
  }

  // ---- main stream: graph bookkeeping, then join ----
  {
    ProfScope _p("graph_prep", st);
    PrepArgs pa{b->edge_index, b->batch, b->graph_ptr, b->edge_attr, d.N, d.E, d.B,
                d.Fe,          d.Fep,   iv,           fv.e_s};
    pa.want_key = any_dropout;
    pa.seed = seed;
    pa.rng_counter = rng_counter;
    int rc = cgr_graph_prep_impl(pa, st);
    if (rc) return rc;
  }
#if CGR_PAD_ON_MAIN
  // the main stream waits for the x-GEMM anyway: pad x for the backward's TN GEMMs here (the
  // forward x-GEMM reads x in place)
  if (fv.xp) {
    ProfScope _p("pad_x", st);
    HIP_RET(pad_rows(b->x, N, F, fv.xp, d.Fp, st));
  }
#endif
  if (CGR_W0E_ON_MAIN == 2) HIP_RET(w0e_transpose(st));
  if (wt_main && !CGR_B3) HIP_RET(weight_transposes(st));
  HIP_RET(hipStreamWaitEvent(st, p_ready, 0));

  if (Hp <= 512) {  // edge init + a_0 in one pass
    ProfScope _p("edge_init_seg_fwd", st);
    HIP_RET(edge_init_segsum_fwd(fv.P, iv.src_s, fv.e_s, Fe, d.Fep, fv.w0eT, b0, iv.dst_ptr, N,
                                 H, Hp, d.act, fv.h[0], fv.pre[0], fv.a[0], st, fv.hb[0]));
  } else {
    {
      ProfScope _p("edge_init_fwd", st);
      HIP_RET(edge_init_fwd(fv.P, iv.src_s, fv.e_s, Fe, d.Fep, fv.w0eT, b0, E, H, Hp, d.act,
                            fv.h[0], fv.pre[0], st));
    }
    ProfScope _p("segsum_dst_fwd", st);
    HIP_RET(segment_sum(fv.h[0], Hp, nullptr, iv.dst_ptr, N, Hp, fv.a[0], Hp, st));
  }

  // the layer GEMM also sums the dst segments inside its row tiles (EpLayerSeg)
  const bool fused_seg = CGR_B3 && CGR_FUSED_SEGSUM && Hp % 4 == 0;
  for (int l = 0; l < D; ++l) {
    const float* Wl = params[CGR_PARAM_CONV_W(l)];
    const float* bl_ = params[CGR_PARAM_CONV_B(l)];
    uint32_t thresh;
    float scale;
    dropout_consts(dropout_p, training, l, &thresh, &scale);
    EpLayer ep{bl_,      d.learnable_skip ? params[CGR_PARAM_SKIP(D, l)] : nullptr,
               fv.h[0],  fv.h[l + 1],
               fv.pre[l + 1], Hp,
               E,        H,
               d.act,    thresh,
               scale,    iv.rng,
               l,        fv.hb[l + 1]};
    LdGatherDiff<false> al{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp};
    {
      ProfScope _p("gemm_nt_layer_fwd", st);
      const int vw = vec_for(Wl, H, H);
      const bool planes = CGR_B3 && CGR_B3TP && (training & CGR_TRAIN_FOR_BACKWARD) && fv.mhi[l];
      const b3_u4* img = static_cast<const b3_u4*>(fv.b3lf[l]);
      const EpLayerSeg eps{ep, iv.dst_s, fv.a[l + 1], Hp};
      hipError_t e = (fused_seg && planes)
                         ? launch_b3nt(al, img, eps, E, H, H, st,
                                       B3PlaneOut{fv.mhi[l], fv.mlo[l], fv.mld})
                   : fused_seg ? launch_b3nt(al, img, eps, E, H, H, st)
                   : planes ? launch_b3nt(al, img, ep, E, H, H, st,
                                          B3PlaneOut{fv.mhi[l], fv.mlo[l], fv.mld})
                   : CGR_B3 ? launch_b3nt(al, img, ep, E, H, H, st)
                   : use_rs(H, H, H, Wl) ? with_rs_fmax(H, [&](auto FM) {
        return launch_gemm_rs<CGR_RS_RM, decltype(FM)::value>(al, Wl, H, ep, E, H, H, st);
      }) : with_vec(vw, [&](auto VW) {
        return with_nt_layer(H, [&](auto WV, auto RN) {
          LdPlain<decltype(VW)::value> blw{Wl, H};
          return launch_nt<decltype(WV)::value, 1, decltype(RN)::value, 1>(al, blw, ep, E,
                                                                              H, H, st);
        });
      });
      HIP_RET(e);
    }
    ProfScope _p2("segsum_dst_fwd", st);
    if (fused_seg)  // the GEMM summed the segments inside its row tiles
      HIP_RET(segsum_fixup(fv.h[l + 1], Hp, iv.dst_ptr, N, Hp, b3nt_rows(E, H), fv.a[l + 1], Hp,
                           st));
    else
      HIP_RET(segment_sum(fv.h[l + 1], Hp, nullptr, iv.dst_ptr, N, Hp, fv.a[l + 1], Hp, st));
  }

  // join: Q (split x-GEMM) and the backward transposes / images; the side stream is idle after this
  if (side_done) HIP_RET(hipStreamWaitEvent(st, side_done, 0));
  if (q_ready) HIP_RET(hipStreamWaitEvent(st, q_ready, 0));

  // readout: hn = act(s W_n[:, F:]^T + Q + b_n), s = a_D
  {
    ProfScope _p("gemm_nt_readout_fwd", st);
    const int vw = vec_for(Wn + F, F + H, H);
    EpReadoutQ ep{bn, fv.Q, fv.hn, fv.zn, Hp, N, H, d.act};
    hipError_t e = CGR_B3 ? launch_b3nt(LdPlain<4>{fv.a[D], Hp}, static_cast<const b3_u4*>(fv.b3rof),
                                        ep, N, H, H, st)
                          : with_vec(vw, [&](auto VW) {
      return with_nt_rn(H, [&](auto RN) {
        LdPlain<4> al{fv.a[D], Hp};
        LdPlain<decltype(VW)::value> blw{Wn + F, F + H};
        return launch_nt<CGR_NODE_NT_WAVES, 1, decltype(RN)::value, 1>(al, blw, ep, N, H, H, st);
      });
    });
    HIP_RET(e);
  }
  ProfScope _p("pool_head_fwd", st);
  HIP_RET(pool_head_fwd(fv.hn, Hp, iv.graph_ptr, d.B, H, params[CGR_PARAM_FFN_W(D)],
                        params[CGR_PARAM_FFN_B(D)], fv.g, y, st));
  return 0;
}

}  // namespace cgr
