// Reverse mode of gnn_fwd.hip (the math is restated and pinned in
// oracle/dmpnn_numpy.py::backward).  Same gather -> MFMA GEMM -> segmented-reduce pattern as the
// forward with src and dst swapped; weight gradients are split-K TN GEMMs over the edge / node
// dimension reduced deterministically; no atomics anywhere, so gradients are bitwise stable.
//
//   dg = dy wf ; dwf = dy^T g ; dbf = sum dy                          (ffn + add-pool)
//   dzn = dg[graph(v)] * act'(zn)                                     (edge_to_node act)
//   dW_n = dzn^T [x | s], db_n = colsum(dzn), ds = dzn W_n[:, F:]
//   dh_D = ds[dst]
//   for l = D-1 .. 0:
//     dpre = dh_{l+1} * mask * act'(pre_l) ; dh0 += s_l dpre ; ds_l = sum dpre*h0
//     dW_l = dpre^T (a_l[src] - h_l[rev])  (message recomputed, never stored) ; db_l = colsum
//     dm = dpre W_l ; da = segsum_src(dm) ; dh_l = da[dst] - dm[rev]
//   dpre0 = (dh0 + dh_0) * act'(pre0)
//   dW0[:, F:] = dpre0^T e ; db0 = colsum(dpre0) ; dW0[:, :F] = (segsum_src dpre0)^T x
#include "dispatch.hpp"
#include "epilogues.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"
#include "profiling.hpp"

namespace cgr {

void dropout_params(const float* dropout_p, int training, int l, uint32_t* thresh, float* scale);

template <class AL, class BL>
static hipError_t tn_and_reduce(const AL& al, const BL& bl, int Nout, int Kout, int R,
                                float* slab, float* bslab, float* dst, int64_t ld_dst,
                                int64_t col_off, float* bias_dst, hipStream_t st) {
  const TnPlan p = tn_plan(Nout, Kout, R);
  ProfScope _p1("gemm_tn_wgrad", st);
  hipError_t e = with_tn_shape(Nout, Kout, [&](auto W, auto RN) {
    return launch_gemm_tn<decltype(W)::value, 1, decltype(RN)::value, 1>(al, bl, p, slab, bslab, Nout,
                                                                   Kout, R, bias_dst != nullptr,
                                                                   st);
  });
  if (e != hipSuccess) return e;
  _p1.end();
  ProfScope _p2("splitk_reduce", st);
  return reduce_slabs(slab, bslab, p.splits, Nout, Kout, dst, ld_dst, col_off, bias_dst, st);
}

int gnn_backward_impl(const Dims& d, const float* const* params, const cgr_batch* b,
                      const float* dropout_p, uint64_t seed, int training, const void* arena,
                      const float* dy, float* const* grads, void* workspace, hipStream_t st) {
  const ArenaLayout L = arena_layout(d);
  const IndexView iv = index_view(const_cast<void*>(arena), L);
  const FloatView fv = float_view(const_cast<void*>(arena), L, d);
  const WorkspaceLayout WL = workspace_layout(d);
  char* ws = static_cast<char*>(workspace);
  float* dpre = reinterpret_cast<float*>(ws + WL.dpre);
  float* dm = reinterpret_cast<float*>(ws + WL.dm);
  float* dh0 = reinterpret_cast<float*>(ws + WL.dh0);
  float* da = reinterpret_cast<float*>(ws + WL.da);
  float* dzn = reinterpret_cast<float*>(ws + WL.dzn);
  float* ds = reinterpret_cast<float*>(ws + WL.ds);
  float* Gs = reinterpret_cast<float*>(ws + WL.Gs);
  float* dg = reinterpret_cast<float*>(ws + WL.dg);
  float* wT = reinterpret_cast<float*>(ws + WL.wT);
  float* slab = reinterpret_cast<float*>(ws + WL.slab);
  float* bslab = reinterpret_cast<float*>(ws + WL.bslab);
  float* dsig_part = reinterpret_cast<float*>(ws + WL.dsig_part);

  const int N = (int)d.N, E = (int)d.E, H = d.H, Hp = d.Hp, F = d.F, Fe = d.Fe, D = d.D;
  const int64_t HHp = (int64_t)H * Hp;

  // transposed weights: wT[l] = W_l^T (l < D), wT[D] = W_n[:, F:]^T, all [H, Hp]
  {
    ProfScope _p("weight_transpose", st);
    TransposeJobs tj{};
    for (int l = 0; l < D; ++l)
      tj.job[l] = TransposeJob{params[CGR_PARAM_CONV_W(l)], H, 0, wT + l * HHp, Hp, H, H};
    tj.job[D] = TransposeJob{params[CGR_PARAM_E2N_W(D)], F + H, F, wT + D * HHp, Hp, H, H};
    tj.n = D + 1;
    HIP_RET(transpose_batch(tj, st));
  }

  // head + readout
  {
    ProfScope _p("head_readout_bwd", st);
    HIP_RET(head_bwd(dy, fv.g, params[CGR_PARAM_FFN_W(D)], d.B, H, Hp, dg,
                     grads[CGR_PARAM_FFN_W(D)], grads[CGR_PARAM_FFN_B(D)], st));
    HIP_RET(readout_act_bwd(dy, params[CGR_PARAM_FFN_W(D)], iv.node_graph, fv.hn, fv.zn, N, H, Hp,
                            d.act, dzn, st));
  }
  {
    const int vx = vec_for(b->x, F, F);
    hipError_t e = with_vec(vx, [&](auto VX) {
      LdPlain<4> al{dzn, Hp};
      LdConcat<decltype(VX)::value> bl{b->x, F, fv.a[D], Hp, F};
      return tn_and_reduce(al, bl, H, F + H, N, slab, bslab, grads[CGR_PARAM_E2N_W(D)], F + H, 0,
                           grads[CGR_PARAM_E2N_B(D)], st);
    });
    HIP_RET(e);
  }
  {
    ProfScope _p("gemm_nt_bwd", st);
    hipError_t e = with_nt_rn(H, [&](auto RN) {
      LdPlain<4> al{dzn, Hp};
      LdPlain<4> bl{wT + D * HHp, Hp};
      EpStore ep{ds, Hp, N, H, nullptr};
      return launch_gemm_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, N, H, H, st);
    });
    HIP_RET(e);
  }

  int nb = layer_act_bwd_blocks(E, Hp);
  for (int l = D - 1; l >= 0; --l) {
    uint32_t thresh;
    float scale;
    dropout_params(dropout_p, training, l, &thresh, &scale);
    LayerBwdArgs la{};
    la.ds = ds;
    la.da = da;
    la.dm = dm;
    la.dst_s = iv.dst_s;
    la.rev_s = iv.rev_s;
    la.hnext = fv.h[l + 1];
    la.pre = fv.pre[l + 1];
    la.h0 = fv.h[0];
    la.sigma = d.learnable_skip ? params[CGR_PARAM_SKIP(D, l)] : nullptr;
    la.seed = seed;
    la.thresh = thresh;
    la.scale = scale;
    la.layer = l;
    la.act = d.act;
    la.first = (l == D - 1);
    la.E = E;
    la.H = H;
    la.Hp = Hp;
    la.dpre = dpre;
    la.dh0 = dh0;
    la.dsig_part = d.learnable_skip ? dsig_part + (int64_t)l * nb : nullptr;
    {
      ProfScope _p("layer_act_bwd", st);
      HIP_RET(layer_act_bwd(la, nullptr, st));
    }

    // dW_l = dpre^T m_l, db_l = colsum(dpre)
    {
      LdPlain<4> al{dpre, Hp};
      LdGatherDiff<false> bl{fv.a[l], fv.h[l], iv.src_s, iv.rev_s, Hp};
      HIP_RET(tn_and_reduce(al, bl, H, H, E, slab, bslab, grads[CGR_PARAM_CONV_W(l)], H, 0,
                            grads[CGR_PARAM_CONV_B(l)], st));
    }
    // dm = dpre W_l
    {
      ProfScope _p("gemm_nt_bwd", st);
      hipError_t e = with_nt_rn(H, [&](auto RN) {
        LdPlain<4> al{dpre, Hp};
        LdPlain<4> bl{wT + l * HHp, Hp};
        EpStore ep{dm, Hp, E, H, nullptr};
        return launch_gemm_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, E, H, H, st);
      });
      HIP_RET(e);
    }
    // da[v] = sum_{src(e) = v} dm[e]
    {
      ProfScope _p("segsum_src_bwd", st);
      HIP_RET(segment_sum(dm, Hp, iv.src_list, iv.src_ptr, N, Hp, da, Hp, st));
    }
  }

  // edge init
  {
    ProfScope _p("edge_init_bwd", st);
    HIP_RET(edge_init_bwd(dh0, da, dm, iv.dst_s, iv.rev_s, fv.h[0], fv.pre[0], E, H, Hp, d.act,
                          dpre, st));
  }
  float* gW0 = grads[CGR_PARAM_EDGE_INIT_W];
  float* gb0 = grads[CGR_PARAM_EDGE_INIT_B];
  if (Fe > 0) {
    LdPlain<4> al{dpre, Hp};
    LdPlain<4> bl{fv.e_s, d.Fep};
    HIP_RET(tn_and_reduce(al, bl, H, Fe, E, slab, bslab, gW0, F + Fe, F, gb0, st));
  }
  {
    ProfScope _p("segsum_src_bwd", st);
    HIP_RET(segment_sum(dpre, Hp, iv.src_list, iv.src_ptr, N, Hp, Gs, Hp, st));
  }
  {
    const int vx = vec_for(b->x, F, F);
    hipError_t e = with_vec(vx, [&](auto VX) {
      LdPlain<4> al{Gs, Hp};
      LdPlain<decltype(VX)::value> bl{b->x, F};
      return tn_and_reduce(al, bl, H, F, N, slab, bslab, gW0, F + Fe, 0,
                           Fe > 0 ? nullptr : gb0, st);
    });
    HIP_RET(e);
  }

  if (d.learnable_skip) {
    ScalarReduceJobs sj{};
    for (int l = 0; l < D; ++l) sj.out[l] = grads[CGR_PARAM_SKIP(D, l)];
    sj.n = D;
    ProfScope _p("skip_grad_reduce", st);
    HIP_RET(reduce_partials(dsig_part, nb, sj, st));
  }
  return 0;
}

}  // namespace cgr
