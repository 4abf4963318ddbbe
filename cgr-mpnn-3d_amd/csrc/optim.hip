// Fused Adam / AMSGrad step (torch.optim.Adam as train.py:117-119 builds it) -- see cgr_adam_step
// in include/cgr_mpnn3d.h.  Memory-bound streaming: 5 reads + 4 writes of fp32 per element
// (amsgrad), float4 when every pointer of a tensor is 16-byte aligned, scalar otherwise.
#include <math.h>

#include "common.hpp"
#include "gnn_internal.hpp"
#include "streams.hpp"

namespace cgr {

struct AdamGroup {
  float* p[CGR_ADAM_GROUP];
  const float* g[CGR_ADAM_GROUP];
  float* m[CGR_ADAM_GROUP];
  float* v[CGR_ADAM_GROUP];
  float* vmax[CGR_ADAM_GROUP];
  float* step[CGR_ADAM_GROUP];
  int64_t numel[CGR_ADAM_GROUP];
  int32_t vec4[CGR_ADAM_GROUP];
  int32_t first_block[CGR_ADAM_GROUP + 1];
  int32_t n;
  // the timeout gate (streams.hpp adam_gate): `err` = the host-mapped error words, `gate` = the
  // device word the step-count kernel sets from them; both null = ungated
  const int* err;
  int* gate;
};

struct AdamHyper {
  double lr, b1, b2;
  float w1, b2f, w2, eps, wd;  // (float)(1 - b1), (float)b2, (float)(1 - b2), ... as torch casts
  int amsgrad, maximize;
};

constexpr int kAdamThreads = 256;
// one float4 per thread: 1.49 M parameters at cfg2 make ~1,460 blocks, every element's five loads
// in flight at once (r04's 16 elements per thread gave 91 blocks on 256 CUs: 15.4 us in the
// replayed step for 54 MB)
constexpr int kAdamElemsPerBlock = kAdamThreads * 4;

// t <- t + 1 for every tensor of the group (before k_adam reads it, same stream) -- unless an
// unpaired backward's completion timed out (its gradients are NaN): then the gate word tells
// k_adam to skip the step, and the parameters stay finite until the model's next forward raises
__global__ void k_adam_step_count(AdamGroup G) {
  __shared__ int poisoned;
  if (threadIdx.x == 0) {
    poisoned = G.err ? __hip_atomic_load(G.err + kDevErrUnpairedTimeout, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) != 0
                     : 0;
    if (G.gate) G.gate[0] = poisoned;
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i < G.n && !poisoned) G.step[i][0] = G.step[i][0] + 1.f;
}

// torch _multi_tensor_adam order: lerp_ (weight < 0.5: m + w (g - m)), mul_(b2), addcmul_,
// maximum_, sqrt, div_(bc2_sqrt), add_(eps), addcdiv_(m, denom, -step_size)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float& vm,
                                          const AdamHyper& h, float neg_step_size,
                                          float bc2_sqrt) {
  if (h.maximize) g = -g;
  if (h.wd != 0.f) g = fmaf(p, h.wd, g);          // grad.add(param, alpha=wd)
  m = fmaf(h.w1, g - m, m);
  v = fmaf(h.w2 * g, g, v * h.b2f);
  float vv = v;
  if (h.amsgrad) {
    vm = fmaxf(vm, v);
    vv = vm;
  }
  const float denom = sqrtf(vv) / bc2_sqrt + h.eps;
  p = fmaf(neg_step_size, m / denom, p);
}

__global__ __launch_bounds__(kAdamThreads) void k_adam(AdamGroup G, AdamHyper h) {
  if (G.gate && G.gate[0]) return;  // the gradients are NaN-poisoned: no update (above)
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < G.n && G.first_block[t + 1] <= b) ++t;
  // the bias corrections once per block (double pow), broadcast through LDS
  __shared__ float sc[2];
  if (threadIdx.x == 0) {
    const double step = (double)G.step[t][0];
    const double bc1 = 1.0 - pow(h.b1, step);
    const double bc2 = 1.0 - pow(h.b2, step);
    sc[0] = (float)(-(h.lr / bc1));
    sc[1] = (float)sqrt(bc2);
  }
  __syncthreads();
  const float neg_step_size = sc[0], bc2_sqrt = sc[1];
  const int64_t base = (int64_t)(b - G.first_block[t]) * kAdamElemsPerBlock;
  const int64_t n = G.numel[t];
  float* P = G.p[t];
  const float* Gr = G.g[t];
  float* M = G.m[t];
  float* V = G.v[t];
  float* VM = G.vmax[t];
  const int64_t e = base + 4 * (int64_t)threadIdx.x;
  if (G.vec4[t] && e + 4 <= n) {
    float4 p4 = *reinterpret_cast<const float4*>(P + e);
    const float4 g4 = *reinterpret_cast<const float4*>(Gr + e);
    float4 m4 = *reinterpret_cast<const float4*>(M + e);
    float4 v4 = *reinterpret_cast<const float4*>(V + e);
    float4 x4 = h.amsgrad ? *reinterpret_cast<const float4*>(VM + e) : v4;
    adam_elem(p4.x, g4.x, m4.x, v4.x, x4.x, h, neg_step_size, bc2_sqrt);
    adam_elem(p4.y, g4.y, m4.y, v4.y, x4.y, h, neg_step_size, bc2_sqrt);
    adam_elem(p4.z, g4.z, m4.z, v4.z, x4.z, h, neg_step_size, bc2_sqrt);
    adam_elem(p4.w, g4.w, m4.w, v4.w, x4.w, h, neg_step_size, bc2_sqrt);
    *reinterpret_cast<float4*>(P + e) = p4;
    *reinterpret_cast<float4*>(M + e) = m4;
    *reinterpret_cast<float4*>(V + e) = v4;
    if (h.amsgrad) *reinterpret_cast<float4*>(VM + e) = x4;
  } else {
    for (int64_t k = e; k < n && k < e + 4; ++k) {
      float vm = h.amsgrad ? VM[k] : 0.f;
      adam_elem(P[k], Gr[k], M[k], V[k], vm, h, neg_step_size, bc2_sqrt);
      if (h.amsgrad) VM[k] = vm;
    }
  }
}

}  // namespace cgr

using namespace cgr;

extern "C" int cgr_adam_step(const cgr_adam_tensor* tensors, int32_t num_tensors, double lr,
                             double beta1, double beta2, double eps, double weight_decay,
                             int32_t amsgrad, int32_t maximize, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(num_tensors >= 0 && (num_tensors == 0 || tensors != nullptr),
            "cgr_adam_step: bad tensor table");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const AdamHyper h{lr,
                    beta1,
                    beta2,
                    (float)(1.0 - beta1),
                    (float)beta2,
                    (float)(1.0 - beta2),
                    (float)eps,
                    (float)weight_decay,
                    amsgrad ? 1 : 0,
                    maximize ? 1 : 0};
  int dev = -1;
  SideStreams* ss = hipStreamGetDevice(st, &dev) == hipSuccess ? side_streams_of(dev) : nullptr;
  (void)hipGetLastError();
  const int* err = ss && ss->adam_gate ? ss->dev_err : nullptr;
  int* gate = ss ? ss->adam_gate : nullptr;
  AdamGroup G{};
  G.err = err;
  G.gate = gate;
  auto flush = [&]() -> int {
    if (G.n == 0) return 0;
    const int blocks = G.first_block[G.n];
    hipLaunchKernelGGL(k_adam_step_count, dim3(1), dim3(64), 0, st, G);
    HIP_RET(hipGetLastError());
    if (blocks > 0) {
      hipLaunchKernelGGL(k_adam, dim3(blocks), dim3(kAdamThreads), 0, st, G, h);
      HIP_RET(hipGetLastError());
    }
    G = AdamGroup{};
    G.err = err;
    G.gate = gate;
    return 0;
  };
  for (int i = 0; i < num_tensors; ++i) {
    const cgr_adam_tensor& t = tensors[i];
    if (t.grad == nullptr || t.numel <= 0) continue;
    CGR_CHECK(t.param && t.exp_avg && t.exp_avg_sq && t.step && (!amsgrad || t.max_exp_avg_sq),
              "cgr_adam_step: NULL state pointer");
    const int64_t nb = (t.numel + kAdamElemsPerBlock - 1) / kAdamElemsPerBlock;
    CGR_CHECK(nb < (1 << 30), "cgr_adam_step: tensor too large");
    const int k = G.n;
    G.p[k] = t.param;
    G.g[k] = t.grad;
    G.m[k] = t.exp_avg;
    G.v[k] = t.exp_avg_sq;
    G.vmax[k] = t.max_exp_avg_sq;
    G.step[k] = t.step;
    G.numel[k] = t.numel;
    auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    G.vec4[k] = al(t.param) && al(t.grad) && al(t.exp_avg) && al(t.exp_avg_sq) &&
                (!amsgrad || al(t.max_exp_avg_sq));
    G.first_block[k + 1] = G.first_block[k] + (int32_t)nb;
    CGR_CHECK((int64_t)G.first_block[k] + nb < (1LL << 31), "cgr_adam_step: too many blocks");
    G.n = k + 1;
    if (G.n == CGR_ADAM_GROUP) {
      const int rc = flush();
      if (rc) return rc;
    }
  }
  return flush();
}
