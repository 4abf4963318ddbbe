// Reverse mode of gnn_fwd.hip (the math is restated and pinned in
// oracle/dmpnn_numpy.py::backward).  Same gather -> MFMA GEMM -> segmented-reduce pattern as the
// forward with src and dst swapped; weight gradients are split-K TN GEMMs over the edge / node
// dimension reduced deterministically; no atomics anywhere, so gradients are bitwise stable.
//
//   dwf = dy^T g ; dbf = sum dy ; dzn = dy[graph(v)] wf * act'(zn)        (ffn, pool, edge_to_node)
//   dW_n = dzn^T [x | s], db_n = colsum(dzn), ds = dzn W_n[:, F:]
//   dh_D = ds[dst]
//   for l = D-1 .. 0:
//     dpre = dh_{l+1} * mask * act'(pre_l) ; dh0 += s_l dpre ; ds_l = sum dpre*h0
//     dW_l = dpre^T (a_l[src] - h_l[rev])  (message recomputed, never stored) ; db_l = colsum
//     dm = dpre W_l ; da = segsum_src(dm) ; dh_l = da[dst] - dm[rev]  (one fused kernel with the
//     next lower layer's dpre, da never stored: k_segsum_act_bwd)
//   dpre0 = (dh0 + dh_0) * act'(pre0)
//   dW0[:, F:] = dpre0^T e ; db0 = colsum(dpre0) ; dW0[:, :F] = (segsum_src dpre0)^T x
//
// Streams: the critical path is act_bwd -> dm GEMM -> segsum per layer.  Every weight-gradient
// TN GEMM (+ its slab reduction) only feeds the gradient outputs, so it runs on the side stream,
// forked right after its input is produced; dpre is double-buffered so the next layer's act_bwd
// can proceed, and the main stream waits for the side stream only before re-using a dpre buffer
// and at the very end.
#include "dispatch.hpp"
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
  ProfScope _p(name, st);
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
                           hipStream_t st, int target = CGR_TNR_TARGET_WGS) {
  const TnrPlan q = plan_tnr<FA, FB>(Nout, Kout, R, target);
  *plan = TnPlan{q.tiles_n, q.tiles_k, q.splits, q.rows_per_split};
  ProfScope _p(name, st);
  return launch_gemm_tnr<FA, FB>(sa, sb, q, slab, bslab, Nout, Kout, R, want_bias, st);
}

// split-bf16 TN (gemm_b3.hpp); same slab layout as tn_gemm
template <class AL, class BL>
static hipError_t b3tn_gemm(const char* name, const AL& al, const BL& bl, int Nout, int Kout, int R,
                            float* slab, float* bslab, bool want_bias, TnPlan* plan,
                            hipStream_t st, int target = CGR_B3TN_TARGET) {
  const B3TnPlan q = b3tn_plan(Nout, Kout, R, target);
  *plan = TnPlan{1, q.tiles_k, q.splits, q.rows_per_split};
  ProfScope _p(name, st);
  return launch_b3tn(al, bl, q, slab, bslab, Nout, Kout, R, want_bias, st);
}

// jobs != nullptr: queue the reduction for one batched launch (CGR_BATCH_REDUCE) instead
#ifndef CGR_RO_TN_AT
#define CGR_RO_TN_AT -1
#endif

#ifndef CGR_NODE_REDUCE_FLAT
#define CGR_NODE_REDUCE_FLAT 1  // the node weight gradient's reduce ends the backward's main chain
#endif
#ifndef CGR_EDGE_TN_MAIN
#define CGR_EDGE_TN_MAIN 0
#endif
#ifndef CGR_EDGE_TN_TARGET
#define CGR_EDGE_TN_TARGET 256  // fewer splits, fewer CUs taken from the node TN beside it: A/B 1024 -> 256 -0.3 %, 128 +0.4 %, 64 +2 %
#endif
#ifndef CGR_MAIN_FIRST
#define CGR_MAIN_FIRST 1  // A/B: 1.283 -> 1.263 ms (the captured graph keeps the main chain on one queue)
#endif
#ifndef CGR_MAIN_FIRST_TAIL
#define CGR_MAIN_FIRST_TAIL 1  // A/B: -0.8 % (1.220 -> 1.211 ms)
#endif
#ifndef CGR_MAIN_FIRST_RO
#define CGR_MAIN_FIRST_RO 0  // A/B: +10 % (readout NT and TN both on the critical path)
#endif

static hipError_t tn_reduce(const TnPlan& p, const float* slab, const float* bslab, int Nout,
                            int Kout, float* dst, int64_t ld_dst, int64_t col_off, float* bias_dst,
                            hipStream_t st, int gap_at = 0, int gap_len = 0,
                            RedJobs* jobs = nullptr, bool flat = false) {
  if (jobs)
    return add_reduce_job(*jobs, slab, bslab, p.splits, Nout, Kout, dst, ld_dst, col_off,
                          bias_dst, gap_at, gap_len)
               ? hipSuccess
               : hipErrorInvalidValue;
  ProfScope _p("splitk_reduce", st);
  return reduce_slabs(slab, bslab, p.splits, Nout, Kout, dst, ld_dst, col_off, bias_dst, st,
                      gap_at, gap_len, flat);
}

int gnn_backward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                      const float* dropout_p, uint64_t seed, int training, const void* arena,
                      const float* dy, float* const* grads, void* workspace, hipStream_t st) {
  const ArenaLayout L = arena_layout(d);
  const IndexView iv = index_view(const_cast<void*>(arena), L);
  const FloatView fv = float_view(const_cast<void*>(arena), L, d);
  const WorkspaceLayout WL = workspace_layout(d);
  char* ws = static_cast<char*>(workspace);
  // dpre of layer l: buffer l (CGR_DPRE_RING: l & 1)
  auto dpre = [&](int l) { return reinterpret_cast<float*>(ws + WL.dpre[CGR_DPRE_RING ? l & 1 : l]); };
  // weight-gradient operands as bf16 planes: the forward wrote the messages' (arena), the
  // activation backward writes dpre's (same ring as dpre)
  const bool planes = CGR_B3 && CGR_B3TP && (training & CGR_TRAIN_FOR_BACKWARD) && d.D > 0 &&
                      fv.mhi[0] != nullptr;
  auto dphi = [&](int l) {
    return reinterpret_cast<uint16_t*>(ws + WL.dphi[CGR_DPRE_RING ? l & 1 : l]);
  };
  auto dplo = [&](int l) {
    return reinterpret_cast<uint16_t*>(ws + WL.dplo[CGR_DPRE_RING ? l & 1 : l]);
  };
  float* dm = reinterpret_cast<float*>(ws + WL.dm);
  float* dh0 = reinterpret_cast<float*>(ws + WL.dh0);
  float* dzn = reinterpret_cast<float*>(ws + WL.dzn);
  float* ds = reinterpret_cast<float*>(ws + WL.ds);
  float* Gs = reinterpret_cast<float*>(ws + WL.Gs);
  const float* wT = fv.wT;  // W_l^T, W_n[:, F:]^T, transposed by the forward (side stream)
  float* slab = reinterpret_cast<float*>(ws + WL.slab);
  float* bslab = reinterpret_cast<float*>(ws + WL.bslab);
  float* slab2 = reinterpret_cast<float*>(ws + WL.slab2);
  float* bslab2 = reinterpret_cast<float*>(ws + WL.bslab2);
  float* dsig_part = reinterpret_cast<float*>(ws + WL.dsig_part);

  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  const int64_t HHp = (int64_t)H * Hp;

  SideStreams* ss = side_streams(st);
  if (!ss) return CGR_ERR_HIP;
  std::lock_guard<std::mutex> ss_lock(ss->mu);
  // side-stream slabs: consecutive regions when batched (workspace_layout sizes them in the same
  // order: readout, layers D-1 .. 0, edge), else all at the start of the shared region
  RedJobs side_jobs{};
  float* slab_next = slab;
  float* bslab_next = bslab;
  auto side_slab = [&](int Nout, int Kout, int64_t R, float** sp, float** bp) {
    *sp = slab_next;
    *bp = bslab_next;
    if (CGR_BATCH_REDUCE) {
      const TnPlan q = tn_plan(Nout, Kout, (int)R);
      slab_next += (size_t)q.splits * Nout * (size_t)((Kout + 3) & ~3);
      bslab_next += (size_t)q.splits * Nout;
    }
  };
  RedJobs* sj = CGR_BATCH_REDUCE ? &side_jobs : nullptr;
  // instrumented (profiling) runs stay serial so per-kernel event times are isolated durations
  hipStream_t side = (prof_enabled() || single_stream()) ? st : ss->side;

  // rows [E, round_up(E, 32)) of the dpre planes are zero (the plane TN reads whole 32-row steps)
  if (planes && b3tp_rows(E) > E) {
    const size_t pad = (size_t)(b3tp_rows(E) - E) * (size_t)fv.mld * 2;
    for (int r = 0; r < (CGR_DPRE_RING ? (D < 2 ? D : 2) : D); ++r) {
      HIP_RET(hipMemsetAsync(dphi(r) + (int64_t)E * fv.mld, 0, pad, st));
      HIP_RET(hipMemsetAsync(dplo(r) + (int64_t)E * fv.mld, 0, pad, st));
    }
  }
  // head + readout
  {
    ProfScope _p("head_readout_bwd", st);
#ifndef CGR_HEAD_MERGE
#define CGR_HEAD_MERGE 0  // 1: dwf / dbf column sums as extra blocks of the dzn launch (one launch
                          // less on the critical chain, 15 -> 9.5 us, but the step A/B -1.4 %)
#endif
    if (CGR_HEAD_MERGE) {
      HIP_RET(head_readout_bwd(dy, fv.g, d.B, grads[CGR_PARAM_FFN_W(D)],
                               grads[CGR_PARAM_FFN_B(D)], params[CGR_PARAM_FFN_W(D)],
                               iv.node_graph, fv.hn, fv.zn, N, H, Hp, d.act, dzn, st));
    } else {
      HIP_RET(head_bwd(dy, fv.g, params[CGR_PARAM_FFN_W(D)], d.B, H, Hp, nullptr,
                       grads[CGR_PARAM_FFN_W(D)], grads[CGR_PARAM_FFN_B(D)], st));
      HIP_RET(readout_act_bwd(dy, params[CGR_PARAM_FFN_W(D)], iv.node_graph, fv.hn, fv.zn, N, H,
                              Hp, d.act, dzn, st));
    }
  }
  // side: dW_n = dzn^T [x | s], db_n.  Enqueued here (CGR_RO_TN_AT < 0) or after the layer
  // weight gradient of layer CGR_RO_TN_AT, so that it does not run beside the main stream's
  // readout/top-layer GEMMs, which sit on the critical path
  auto readout_tn = [&](hipEvent_t fork_ev) -> int {
    if (fork_ev) HIP_RET(hipStreamWaitEvent(side, fork_ev, 0));
    else HIP_RET(fork_to(ss, st, side));
    if (fv.xp) {  // [xp | s] with x padded to Fp: the pad columns are skipped by the reduce
      const int Fp = d.Fp;
      TnPlan p;
      float *rsl, *rbs;
      side_slab(H, Fp + H, N, &rsl, &rbs);
      LdPlain<4> al{dzn, Hp};
      LdConcat<4> bl{fv.xp, Fp, fv.a[D], Hp, Fp};
      if (CGR_B3TN && b3tn_ok(al, bl, H, N) && ((uintptr_t)fv.xp & 15) == 0) {
        HIP_RET(b3tn_gemm("gemm_tn_wgrad_readout", al, bl, H, Fp + H, N, rsl, rbs, true, &p, side,
                          CGR_B3TN_RO_TARGET));
      } else if (CGR_TNR_RO && tnr_x_ok(H, Fp + H, Fp, fv.xp)) {
        HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_readout", TnrRows{dzn, Hp},
                                TnrConcat{fv.xp, Fp, fv.a[D], Hp, Fp}, H, Fp + H, N, rsl, rbs,
                                true, &p, side, CGR_TNR_RO_TARGET)));
      } else {
        HIP_RET(tn_gemm("gemm_tn_wgrad_readout", al, bl, H, Fp + H, N, rsl, rbs, true, &p, side));
      }
      HIP_RET(tn_reduce(p, rsl, rbs, H, Fp + H, grads[CGR_PARAM_E2N_W(D)], F + H, 0,
                        grads[CGR_PARAM_E2N_B(D)], side, F, Fp - F, sj));
    } else {
      const int vx = vec_for(b->x, F, F);
      TnPlan p;
      float *rsl, *rbs;
      side_slab(H, F + H, N, &rsl, &rbs);
      const LdPlain<4> al4{dzn, Hp};
      const LdConcat<4> bl4{b->x, F, fv.a[D], Hp, F};
      if (CGR_B3TN && F % 4 == 0 && ((uintptr_t)b->x & 15) == 0 && b3tn_ok(al4, bl4, H, N)) {
        HIP_RET(b3tn_gemm("gemm_tn_wgrad_readout", al4, bl4, H, F + H, N, rsl, rbs, true, &p, side,
                          CGR_B3TN_RO_TARGET));
      } else if (CGR_TNR_RO && F % 4 == 0 && tnr_x_ok(H, F + H, F, b->x)) {
        HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_readout", TnrRows{dzn, Hp},
                                TnrConcat{b->x, F, fv.a[D], Hp, F}, H, F + H, N, rsl, rbs, true,
                                &p, side, CGR_TNR_RO_TARGET)));
      } else {
        hipError_t e = with_vec(vx, [&](auto VX) {
          LdPlain<4> al{dzn, Hp};
          LdConcat<decltype(VX)::value> bl{b->x, F, fv.a[D], Hp, F};
          return tn_gemm("gemm_tn_wgrad_readout", al, bl, H, F + H, N, rsl, rbs, true, &p, side);
        });
        HIP_RET(e);
      }
      HIP_RET(tn_reduce(p, rsl, rbs, H, F + H, grads[CGR_PARAM_E2N_W(D)], F + H, 0,
                        grads[CGR_PARAM_E2N_B(D)], side, 0, 0, sj));
    }
    return 0;
  };
  const int ro_at = (CGR_RO_TN_AT >= 0 && CGR_RO_TN_AT < D) ? CGR_RO_TN_AT : -1;
  // main: ds = dzn W_n[:, F:]
  auto readout_nt = [&]() -> int {
    ProfScope _p("gemm_nt_readout_bwd", st);
    if (CGR_B3) {
      HIP_RET(launch_b3nt(LdPlain<4>{dzn, Hp}, static_cast<const b3_u4*>(fv.b3rob),
                          EpStore{ds, Hp, N, H, nullptr}, N, H, H, st));
      return 0;
    }
    hipError_t e = with_nt_rn(H, [&](auto RN) {
      LdPlain<4> al{dzn, Hp};
      LdPlain<4> bl{wT + D * HHp, Hp};
      EpStore ep{ds, Hp, N, H, nullptr};
      return launch_nt<CGR_NODE_NT_WAVES, 1, decltype(RN)::value, 1>(al, bl, ep, N, H, H, st);
    });
    HIP_RET(e);
    return 0;
  };
  // CGR_MAIN_FIRST (see the layer loop): the main stream's NT is enqueued before the side work
  // that forks from the same point
  if (ro_at < 0 && CGR_MAIN_FIRST_RO && side != st) {
    hipEvent_t fork_ev = nullptr;
    HIP_RET(record_point(ss, st, &fork_ev));
    int rc = readout_nt();
    if (rc) return rc;
    rc = readout_tn(fork_ev);
    if (rc) return rc;
  } else {
    if (ro_at < 0) {
      const int rc = readout_tn(nullptr);
      if (rc) return rc;
    }
    const int rc = readout_nt();
    if (rc) return rc;
  }

  // learnable-skip partial-sum slots per layer (same count for the fused and unfused kernels)
  const int nb = segsum_act_bwd_blocks(E, N, Hp);
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
    la.hbits = fv.hb[l + 1];
    la.pre = fv.pre[l + 1];
    la.h0 = fv.h[0];
    la.sigma = d.learnable_skip ? params[CGR_PARAM_SKIP(D, l)] : nullptr;
    la.seed = iv.rng;  // the key the forward used (arena)
    la.thresh = thresh;
    la.scale = scale;
    la.layer = l;
    la.act = d.act;
    la.first = (l == D - 1);
    la.E = E;
    la.H = H;
    la.Hp = Hp;
    la.dpre = dpre(l);
    la.dphi = planes ? dphi(l) : nullptr;
    la.dplo = planes ? dplo(l) : nullptr;
    la.dpld = fv.mld;
    la.dh0 = CGR_DH0_DEFER ? nullptr : dh0;
    la.dsig_part = d.learnable_skip ? dsig_part + (int64_t)l * nb : nullptr;
    return la;
  };
  hipEvent_t tn_done[CGR_MAX_DEPTH];
  if (D > 0) {  // top layer: dh_D = ds[dst]
    ProfScope _p("layer_act_bwd", st);
    HIP_RET(layer_act_bwd(layer_args(D - 1), nb, st));
  }
  // edge init: dpre0 overwrites dh0 in place (each element read then written by one thread)
  float* dpre0 = dh0;
  for (int l = D - 1; l >= 0; --l) {
    float* dp = dpre(l);  // written by the previous iteration's fused kernel (or just above)
    // main: dm = dpre W_l
    auto layer_nt = [&]() -> int {
      ProfScope _p("gemm_nt_layer_bwd", st);
      if (CGR_B3) {
        HIP_RET(launch_b3nt(LdPlain<4>{dp, Hp}, static_cast<const b3_u4*>(fv.b3lb[l]),
                            EpStore{dm, Hp, E, H, nullptr}, E, H, H, st));
        return 0;
      }
      hipError_t e = CGR_RS_BWD && use_rs(H, H, Hp, wT + l * HHp) ? with_rs_fmax(H, [&](auto FM) {
        LdPlain<4> al{dp, Hp};
        EpStore ep{dm, Hp, E, H, nullptr};
        return launch_gemm_rs<CGR_RS_RM, decltype(FM)::value>(al, wT + l * HHp, Hp, ep, E, H, H, st);
      }) : with_nt_layer(H, [&](auto WV, auto RN) {
        LdPlain<4> al{dp, Hp};
        LdPlain<4> bl{wT + l * HHp, Hp};
        EpStore ep{dm, Hp, E, H, nullptr};
        return launch_nt<decltype(WV)::value, 1, decltype(RN)::value, 1>(al, bl, ep, E, H, H,
                                                                            st);
      });
      HIP_RET(e);
      return 0;
    };
    // side: dW_l = dpre^T m_l, db_l = colsum(dpre).  CGR_MAIN_FIRST: the fork point is recorded
    // before the main stream's NT is enqueued and the side work after it (same dependencies;
    // only the order in which a captured graph sees the two children differs)
    hipEvent_t fork_ev = nullptr;
    if (CGR_MAIN_FIRST && side != st) {
      HIP_RET(record_point(ss, st, &fork_ev));
      const int rc = layer_nt();
      if (rc) return rc;
      HIP_RET(hipStreamWaitEvent(side, fork_ev, 0));
    } else {
      HIP_RET(fork_to(ss, st, side));
    }
    {
      LdPlain<4> al{dp, Hp};
      LdGatherDiff<false> bl{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp};
      TnPlan p;
      float *lsl, *lbs;
      side_slab(H, H, E, &lsl, &lbs);
      const int tf = tnr_layer_frags(H);
      const B3TpPlan tq = b3tp_plan(H, H, E);
      const B3Planes pa{planes ? dphi(l) : nullptr, planes ? dplo(l) : nullptr, fv.mld};
      const B3Planes pm{fv.mhi[l], fv.mlo[l], fv.mld};
      if (planes && b3tp_ok(pa, pm, Hp, tq)) {
        ProfScope _pt("gemm_tn_wgrad_layer", side);
        p = TnPlan{tq.tiles_n, tq.tiles_k, tq.splits, tq.rows_per_split};
        HIP_RET(launch_b3tp(pa, pm, dp, Hp, tq, lsl, lbs, H, H, E, true, side));
      } else if (CGR_B3TN && b3tn_ok(al, bl, H, E)) {
        HIP_RET(b3tn_gemm("gemm_tn_wgrad_layer", al, bl, H, H, E, lsl, lbs, true, &p, side));
      } else if (tf == 5) {
        HIP_RET((tnr_gemm<5, 5>("gemm_tn_wgrad_layer", TnrRows{dp, Hp},
                                TnrDiff{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp}, H, H, E, lsl,
                                lbs, true, &p, side)));
      } else if (tf == 4) {
        HIP_RET((tnr_gemm<4, 4>("gemm_tn_wgrad_layer", TnrRows{dp, Hp},
                                TnrDiff{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp}, H, H, E, lsl,
                                lbs, true, &p, side)));
      } else {
        HIP_RET(tn_gemm("gemm_tn_wgrad_layer", al, bl, H, H, E, lsl, lbs, true, &p, side));
      }
      if (CGR_DPRE_RING) HIP_RET(record_point(ss, side, &tn_done[l]));
      HIP_RET(tn_reduce(p, lsl, lbs, H, H, grads[CGR_PARAM_CONV_W(l)], H, 0,
                        grads[CGR_PARAM_CONV_B(l)], side, 0, 0, sj));
    }
    if (l == ro_at) {
      const int rc = readout_tn(nullptr);
      if (rc) return rc;
    }
    if (!(CGR_MAIN_FIRST && side != st)) {
      const int rc = layer_nt();
      if (rc) return rc;
    }
    // main: da[v] = sum_{src(e) = v} dm[e], consumed in place by the layer below:
    // dh_l = da[dst] - dm[rev] -> dpre_{l-1} (or dpre0 of the edge init when l == 0)
    ProfScope _p("segsum_act_bwd", st);
    if (l > 0) {
      // ring: dpre buffer (l-1) & 1 was last read by the weight gradient of layer l+1
      if (CGR_DPRE_RING && l + 1 <= D - 1) HIP_RET(hipStreamWaitEvent(st, tn_done[l + 1], 0));
      HIP_RET(segsum_act_bwd(layer_args(l - 1), iv.src_list, iv.src_ptr, iv.dst_ptr, N, false,
                             iv.status, st));
    } else {
      LayerBwdArgs le{};
      le.dm = dm;
      le.rev_s = iv.rev_s;
      le.h0 = fv.h[0];
      le.hbits = fv.hb[0];
      le.pre = fv.pre[0];
      le.act = d.act;
      le.E = E;
      le.H = H;
      le.Hp = Hp;
      le.dh0 = CGR_DH0_DEFER ? nullptr : dh0;
      if (CGR_DH0_DEFER) {
        le.nl = D;
        for (int q = 0; q < D; ++q) {
          le.dpre_l[q] = dpre(q);
          le.sigma_l[q] = d.learnable_skip ? params[CGR_PARAM_SKIP(D, q)] : nullptr;
        }
      }
      le.dpre = dpre0;
      HIP_RET(segsum_act_bwd(le, iv.src_list, iv.src_ptr, iv.dst_ptr, N, true, iv.status, st));
    }
  }
  float* gW0 = grads[CGR_PARAM_EDGE_INIT_W];
  float* gb0 = grads[CGR_PARAM_EDGE_INIT_B];
  // CGR_MAIN_FIRST_TAIL: fork point recorded here, the side work enqueued after the main tail
  hipEvent_t tail_ev = nullptr;
  if (CGR_MAIN_FIRST_TAIL && !CGR_BATCH_REDUCE && side != st) HIP_RET(record_point(ss, st, &tail_ev));
  // CGR_EDGE_TN_MAIN: the edge-feature TN follows the node TN on the caller's stream (own slab:
  // slab2, free once the node reduce has run) instead of running beside it on the side stream
  const bool edge_main = CGR_EDGE_TN_MAIN && side != st;
  auto edge_tn = [&]() -> int {
    if (Fe > 0) {  // dW0[:, F:] = dpre0^T e, db0
      hipStream_t es = edge_main ? st : side;
      if (!edge_main) {
        if (tail_ev) HIP_RET(hipStreamWaitEvent(side, tail_ev, 0));
        else HIP_RET(fork_to(ss, st, side));
      }
      LdPlain<4> al{dpre0, Hp};
      LdPlain<4> bl{fv.e_s, d.Fep};
      TnPlan p;
      float *esl, *ebs;
      if (edge_main) {
        esl = slab2;
        ebs = bslab2;
      } else {
        side_slab(H, Fe, E, &esl, &ebs);
      }
      HIP_RET(tn_gemm("gemm_tn_wgrad_edge", al, bl, H, Fe, E, esl, ebs, true, &p, es,
                      CGR_EDGE_TN_TARGET));
      HIP_RET(tn_reduce(p, esl, ebs, H, Fe, gW0, F + Fe, F, gb0, es, 0, 0, edge_main ? nullptr : sj));
    }
    return 0;
  };
  if (!tail_ev && !edge_main) {
    const int rc = edge_tn();
    if (rc) return rc;
  }
  if (sj) {  // every side-stream weight gradient, one launch, at the end of the side stream
    ProfScope _p("splitk_reduce", side);
    HIP_RET(reduce_slabs_batched(side_jobs, CGR_BATCH_REDUCE_BLOCKS, side));
  }
  {
    ProfScope _p("segsum_src_bwd", st);
    HIP_RET(segment_sum(dpre0, Hp, iv.src_list, iv.src_ptr, N, Hp, Gs, Hp, st));
  }
  if (F > 0) {  // main: dW0[:, :F] = Gs^T x (own slab: runs beside the side stream's work)
    const float* xb = fv.xp ? fv.xp : b->x;
    const int64_t ldx = fv.xp ? d.Fp : F;
    const int vx = vec_for(xb, ldx, F);
    TnPlan p;
    const int Fx = fv.xp ? d.Fp : F;  // x columns the GEMM covers (pad columns are zero)
    const LdPlain<4> gal{Gs, Hp}, gbl{xb, ldx};
    if (CGR_B3TN && ldx % 4 == 0 && ((uintptr_t)xb & 15) == 0 && b3tn_ok(gal, gbl, H, N)) {
      HIP_RET(b3tn_gemm("gemm_tn_wgrad_node", gal, gbl, H, Fx, N, slab2, bslab2, Fe == 0, &p, st,
                        CGR_B3TN_NODE_TARGET));
      HIP_RET(tn_reduce(p, slab2, bslab2, H, Fx, gW0, F + Fe, 0, Fe > 0 ? nullptr : gb0, st, F,
                        Fx - F, nullptr, CGR_NODE_REDUCE_FLAT));
    } else if (CGR_TNR_NODE && tnr_x_ok(H, Fx, ldx, xb)) {
      HIP_RET((tnr_gemm<5, 4>("gemm_tn_wgrad_node", TnrRows{Gs, Hp}, TnrRows{xb, ldx}, H, Fx, N,
                              slab2, bslab2, Fe == 0, &p, st, CGR_TNR_NODE_TARGET)));
      HIP_RET(tn_reduce(p, slab2, bslab2, H, Fx, gW0, F + Fe, 0, Fe > 0 ? nullptr : gb0, st, F,
                        Fx - F));
    } else {
      hipError_t e = with_vec(vx, [&](auto VX) {
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
  if (tail_ev || edge_main) {
    const int rc = edge_tn();
    if (rc) return rc;
  }

  if (d.learnable_skip) {
    ScalarReduceJobs sj{};
    for (int l = 0; l < D; ++l) sj.out[l] = grads[CGR_PARAM_SKIP(D, l)];
    sj.n = D;
    ProfScope _p("skip_grad_reduce", st);
    HIP_RET(reduce_partials(dsig_part, nb, sj, st));
  }
  // join: every gradient is complete when the main stream reaches here
  HIP_RET(depend(ss, side, st));
  return 0;
}

}  // namespace cgr
