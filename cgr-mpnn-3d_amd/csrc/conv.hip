// Standalone DMPNNConv (GNN.py:113-145) on the native kernels, in the caller's edge order:
//   a[v]  = sum_{dst(e) = v} h[e]                    (propagate, aggr="add", dim_size = N;
//                                                     aggr="mean": / max(in-degree, 1))
//   h'[e] = (a[src(e)] - h[e ^ 1]) W^T + b           (GNN.py:136-141)
// and its reverse mode.  GNN.forward never calls this (the fused path inlines the layer); it keeps
// the reference's public DMPNNConv usable on its own.
#include "dispatch.hpp"
#include "epilogues.hpp"
#include "gnn_internal.hpp"
#include "kernels.hpp"

namespace cgr {

int split_edges(const int64_t* ei, int E, int N, int* src_c, int* dst_c, hipStream_t st);
int csr_from_keys(const int* key, int n, int nb, int* deg, int* cursor, int* ptr, int* list,
                  hipStream_t st);

namespace {

struct ConvLayout {
  size_t src_c, dst_c, perm, dst_ptr, src_perm, src_ptr, deg, cursor;  // ints
  size_t h_p, a_p, dout_p, dm, da, wT, slab, bslab, inv_deg;           // floats
  size_t bytes;
};

ConvLayout conv_layout(int64_t N, int64_t E, int64_t H) {
  ConvLayout L;
  size_t off = 0;
  auto take = [&](size_t b) {
    const size_t o = off;
    off = (size_t)round_up((int64_t)(off + b), (int64_t)kAlign);
    return o;
  };
  const size_t Hp = (size_t)round_up(H, 4);
  L.src_c = take(4 * E);
  L.dst_c = take(4 * E);
  L.perm = take(4 * E);
  L.dst_ptr = take(4 * (N + 1));
  L.src_perm = take(4 * E);
  L.src_ptr = take(4 * (N + 1));
  L.deg = take(4 * N);
  L.cursor = take(4 * N);
  L.h_p = take(4 * E * Hp);
  L.a_p = take(4 * N * Hp);
  L.dout_p = take(4 * E * Hp);
  L.dm = take(4 * E * Hp);
  L.da = take(4 * N * Hp);
  L.wT = take(4 * H * Hp);
  const TnPlan p = tn_plan((int)H, (int)H, (int)E);
  L.slab = take(4 * (size_t)p.splits * H * (size_t)((H + 3) & ~3));  // slab rows padded to 4
  L.bslab = take(4 * (size_t)p.splits * H);
  L.inv_deg = take(4 * N);
  L.bytes = off;
  return L;
}

template <class T>
T* P(void* base, size_t off) {
  return reinterpret_cast<T*>(static_cast<char*>(base) + off);
}

// da[v, :] += g[v, :H]  (g unpadded [N, H])
__global__ void k_add_rows(float* __restrict__ da, int64_t N, int H, int Hp,
                           const float* __restrict__ g) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  const int64_t v = t / H;
  const int c = (int)(t - v * H);
  da[v * Hp + c] += g[t];
}

// dh[e, :H] = da[dst(e)] (* inv_deg[dst(e)]: mean) - dm[e ^ 1]
__global__ void k_conv_dh(const float* __restrict__ da, const float* __restrict__ dm,
                          const int* __restrict__ dst_c, int64_t E, int H, int Hp,
                          float* __restrict__ dh, const float* __restrict__ inv_deg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * H) return;
  const int64_t e = t / H;
  const int c = (int)(t - e * H);
  const int v = dst_c[e];
  const float s = inv_deg ? inv_deg[v] : 1.f;
  dh[t] = da[(int64_t)v * Hp + c] * s - dm[(e ^ 1) * Hp + c];
}

}  // namespace
}  // namespace cgr

using namespace cgr;

extern "C" {

int64_t cgr_dmpnn_conv_scratch_bytes(int64_t num_nodes, int64_t num_edges, int64_t hidden) {
  if (num_nodes < 1 || num_edges < 0 || hidden < 1) return -1;
  return (int64_t)conv_layout(num_nodes, num_edges, hidden).bytes;
}

int cgr_dmpnn_conv_forward(const int64_t* edge_index, int64_t N, int64_t E, const float* h,
                           int64_t H, const float* weight, const float* bias, float* a_out,
                           float* h_out, void* scratch, int32_t aggregation, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(edge_index && h && weight && bias && a_out && h_out && scratch,
            "cgr_dmpnn_conv_forward: NULL pointer");
  CGR_CHECK(aggregation == CGR_AGGR_ADD || aggregation == CGR_AGGR_MEAN,
            "cgr_dmpnn_conv_forward: unknown aggregation");
  CGR_CHECK(N >= 1 && E >= 2 && E % 2 == 0 && H >= 1 && E < (1ll << 30) && N < (1ll << 31),
            "cgr_dmpnn_conv_forward: bad sizes (E must be even and > 0)");
  hipStream_t st = (hipStream_t)stream;
  const ConvLayout L = conv_layout(N, E, H);
  const int Hp = (int)round_up(H, 4);
  int* src_c = P<int>(scratch, L.src_c);
  int* dst_c = P<int>(scratch, L.dst_c);
  int rc = split_edges(edge_index, (int)E, (int)N, src_c, dst_c, st);
  if (rc) return rc;
  rc = csr_from_keys(dst_c, (int)E, (int)N, P<int>(scratch, L.deg), P<int>(scratch, L.cursor),
                     P<int>(scratch, L.dst_ptr), P<int>(scratch, L.perm), st);
  if (rc) return rc;
  rc = csr_from_keys(src_c, (int)E, (int)N, P<int>(scratch, L.deg), P<int>(scratch, L.cursor),
                     P<int>(scratch, L.src_ptr), P<int>(scratch, L.src_perm), st);
  if (rc) return rc;
  float* h_p = P<float>(scratch, L.h_p);
  float* a_p = P<float>(scratch, L.a_p);
  HIP_RET(hipMemcpy2DAsync(h_p, Hp * 4, h, H * 4, H * 4, E, hipMemcpyDeviceToDevice, st));
  HIP_RET(segment_sum(h_p, Hp, P<int>(scratch, L.perm), P<int>(scratch, L.dst_ptr), N, Hp, a_p,
                      Hp, st));
  if (aggregation == CGR_AGGR_MEAN) {  // the mean: a / max(in-degree, 1), kept for the backward
    float* inv = P<float>(scratch, L.inv_deg);
    HIP_RET(mean_scales(P<int>(scratch, L.dst_ptr), N, nullptr, 0, inv, nullptr, st));
    HIP_RET(scale_rows(a_p, Hp, N, inv, st));
  }
  HIP_RET(hipMemcpy2DAsync(a_out, H * 4, a_p, Hp * 4, H * 4, N, hipMemcpyDeviceToDevice, st));
  const int vw = vec_for(weight, H, H);
  hipError_t e = with_vec(vw, [&](auto VW) {
    return with_nt_rn((int)H, [&](auto RN) {
      LdGatherDiff<true> al{a_p, h_p, src_c, nullptr, Hp};
      LdPlain<decltype(VW)::value> bl{weight, H};
      EpStore ep{h_out, H, (int)E, (int)H, bias};
      return launch_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, (int)E, (int)H, (int)H, st);
    });
  });
  HIP_RET(e);
  return 0;
}

int cgr_dmpnn_conv_backward(const int64_t* edge_index, int64_t N, int64_t E, const float* h,
                            int64_t H, const float* weight, const float* grad_a,
                            const float* grad_h_out, float* grad_h, float* grad_weight,
                            float* grad_bias, void* scratch, int32_t aggregation, void* stream) {
  clear_stale_hip_error();
  (void)edge_index;
  (void)h;
  CGR_CHECK(weight && grad_h && grad_weight && grad_bias && scratch,
            "cgr_dmpnn_conv_backward: NULL pointer");
  CGR_CHECK(aggregation == CGR_AGGR_ADD || aggregation == CGR_AGGR_MEAN,
            "cgr_dmpnn_conv_backward: unknown aggregation");
  CGR_CHECK(N >= 1 && E >= 2 && E % 2 == 0 && H >= 1, "cgr_dmpnn_conv_backward: bad sizes");
  hipStream_t st = (hipStream_t)stream;
  const ConvLayout L = conv_layout(N, E, H);
  const int Hp = (int)round_up(H, 4);
  float* h_p = P<float>(scratch, L.h_p);
  float* a_p = P<float>(scratch, L.a_p);
  float* dout_p = P<float>(scratch, L.dout_p);
  float* dm = P<float>(scratch, L.dm);
  float* da = P<float>(scratch, L.da);
  float* wT = P<float>(scratch, L.wT);
  const int* src_c = P<int>(scratch, L.src_c);
  const int* dst_c = P<int>(scratch, L.dst_c);
  if (grad_h_out) {
    HIP_RET(hipMemcpy2DAsync(dout_p, Hp * 4, grad_h_out, H * 4, H * 4, E, hipMemcpyDeviceToDevice,
                             st));
    // dW = dout^T m, db = colsum(dout)
    {
      LdPlain<4> al{dout_p, Hp};
      LdGatherDiff<true> bl{a_p, h_p, src_c, nullptr, Hp};
      const TnPlan p = tn_plan((int)H, (int)H, (int)E);
      hipError_t e = with_tn_shape((int)H, (int)H, [&](auto W, auto RN) {
        return launch_tn<decltype(W)::value, decltype(RN)::value>(
            al, bl, p, P<float>(scratch, L.slab), P<float>(scratch, L.bslab), (int)H, (int)H,
            (int)E, true, st);
      });
      HIP_RET(e);
      HIP_RET(reduce_slabs(P<float>(scratch, L.slab), P<float>(scratch, L.bslab), p.splits,
                           (int)H, (int)H, grad_weight, H, 0, grad_bias, st));
    }
    TransposeJobs tj{};
    tj.job[0] = TransposeJob{weight, H, 0, wT, Hp, (int)H, (int)H};
    tj.n = 1;
    HIP_RET(transpose_batch(tj, st));
    hipError_t e = with_nt_rn((int)H, [&](auto RN) {
      LdPlain<4> al{dout_p, Hp};
      LdPlain<4> bl{wT, Hp};
      EpStore ep{dm, Hp, (int)E, (int)H, nullptr};
      return launch_nt<4, 1, decltype(RN)::value, 1>(al, bl, ep, (int)E, (int)H, (int)H, st);
    });
    HIP_RET(e);
    HIP_RET(segment_sum(dm, Hp, P<int>(scratch, L.src_perm), P<int>(scratch, L.src_ptr), N, Hp, da,
                        Hp, st));
  } else {
    HIP_RET(hipMemsetAsync(grad_weight, 0, sizeof(float) * H * H, st));
    HIP_RET(hipMemsetAsync(grad_bias, 0, sizeof(float) * H, st));
    HIP_RET(hipMemsetAsync(dm, 0, sizeof(float) * E * Hp, st));
    HIP_RET(hipMemsetAsync(da, 0, sizeof(float) * N * Hp, st));
  }
  if (grad_a) {
    hipLaunchKernelGGL(k_add_rows, dim3(cdiv(N * H, 256)), dim3(256), 0, st, da, N, (int)H, Hp,
                       grad_a);
    HIP_RET(hipGetLastError());
  }
  hipLaunchKernelGGL(k_conv_dh, dim3(cdiv(E * H, 256)), dim3(256), 0, st, da, dm, dst_c, E, (int)H,
                     Hp, grad_h,
                     aggregation == CGR_AGGR_MEAN ? P<float>(scratch, L.inv_deg) : nullptr);
  HIP_RET(hipGetLastError());
  return 0;
}

}  // extern "C"
