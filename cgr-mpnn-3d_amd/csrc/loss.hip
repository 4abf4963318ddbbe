// The training step's loss, torch.nn.MSELoss(reduction="sum") as train.py:120 builds it and
// trainer.py:142-143 applies it to the model's predictions: forward and backward each one launch
// (torch: elementwise + reduce forward, fill + elementwise backward).  Deterministic: one
// workgroup sums in a fixed order.
#include "common.hpp"
#include "gnn_internal.hpp"

namespace cgr {

constexpr int kLossThreads = 256;

__global__ __launch_bounds__(kLossThreads) void k_mse_fwd(const float* __restrict__ y,
                                                          const float* __restrict__ t, int64_t n,
                                                          float scale, float* __restrict__ loss) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kLossThreads) {
    const float d = y[i] - t[i];
    s += d * d;
  }
  __shared__ float red[kLossThreads / 64];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = ((red[0] + red[1]) + (red[2] + red[3])) * scale;
}

// dy = scale2 (y - t) g  (scale2 = 2, or 2 / n for the mean); dt = -dy when requested
__global__ __launch_bounds__(kLossThreads) void k_mse_bwd(const float* __restrict__ y,
                                                          const float* __restrict__ t,
                                                          const float* __restrict__ g, int64_t n,
                                                          float scale2, float* __restrict__ dy,
                                                          float* __restrict__ dt) {
  const int64_t i = (int64_t)blockIdx.x * kLossThreads + threadIdx.x;
  if (i >= n) return;
  const float v = scale2 * (y[i] - t[i]) * g[0];
  if (dy) dy[i] = v;
  if (dt) dt[i] = -v;
}

}  // namespace cgr

using namespace cgr;

extern "C" int cgr_mse_loss_forward(const float* input, const float* target, int64_t n,
                                    int32_t reduction_mean, float* loss, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(n >= 0 && loss && (n == 0 || (input && target)), "cgr_mse_loss_forward: bad args");
  const float scale = reduction_mean ? 1.f / (float)n : 1.f;  // n == 0: 0 * inf = nan, as torch
  hipLaunchKernelGGL(k_mse_fwd, dim3(1), dim3(kLossThreads), 0, static_cast<hipStream_t>(stream),
                     input, target, n, scale, loss);
  HIP_RET(hipGetLastError());
  return 0;
}

extern "C" int cgr_mse_loss_backward(const float* input, const float* target,
                                     const float* grad_loss, int64_t n, int32_t reduction_mean,
                                     float* grad_input, float* grad_target, void* stream) {
  clear_stale_hip_error();
  CGR_CHECK(n >= 0 && grad_loss && (n == 0 || (input && target)),
            "cgr_mse_loss_backward: bad args");
  if (n == 0 || (!grad_input && !grad_target)) return 0;
  const float scale2 = reduction_mean ? 2.f / (float)n : 2.f;
  const int64_t blocks = (n + kLossThreads - 1) / kLossThreads;
  hipLaunchKernelGGL(k_mse_bwd, dim3((unsigned)blocks), dim3(kLossThreads), 0,
                     static_cast<hipStream_t>(stream), input, target, grad_loss, n, scale2,
                     grad_input, grad_target);
  HIP_RET(hipGetLastError());
  return 0;
}
