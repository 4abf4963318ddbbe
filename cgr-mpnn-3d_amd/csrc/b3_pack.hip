// Weight images for the split-bf16 NT GEMMs (gemm_b3.hpp): every weight matrix an NT GEMM reads
// as its B operand is split into three bf16 pieces once per training step (the forward packs
// W_l, W_l^T, [W0[:, :F]; W_n[:, :F]], W_n[:, F:] and W_n[:, F:]^T in one batched launch).
#include "gemm_b3.hpp"

namespace cgr {

// one thread per (k step, image row, lane-group chunk): 8 source values -> 3 pieces -> the chunk's
// swizzled slot in each piece plane.  Row-major sources (ldk == 1) run chunks fastest (adjacent
// threads read adjacent k), transposed sources (ldn == 1) run rows fastest (adjacent n).
__global__ __launch_bounds__(256) void k_b3_pack(B3PackJobs jobs) {
  const B3PackJob& J = jobs.job[blockIdx.y];
  const int64_t total = (int64_t)J.nk * J.rows * 4;
  const bool rowmajor = J.ldk == 1;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int c, nl, ks;
    if (rowmajor) {
      c = (int)(t & 3);
      const int64_t u = t >> 2;
      nl = (int)(u % J.rows);
      ks = (int)(u / J.rows);
    } else {
      nl = (int)(t % J.rows);
      const int64_t u = t / J.rows;
      c = (int)(u & 3);
      ks = (int)(u >> 2);
    }
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = ks * B3_BK + b3_kperm(c, j);
      f[j] = (nl < J.N && k < J.K) ? J.src[(int64_t)nl * J.ldn + (int64_t)k * J.ldk] : 0.f;
    }
    b3_u4 pc[3];
    b3_split8<3>(f, pc);
    const int n = J.n_begin + nl;
    const int slot = c ^ lds_swz(n);
#pragma unroll
    for (int p = 0; p < 3; ++p) J.img[((int64_t)(ks * 3 + p) * J.nimg + n) * 4 + slot] = pc[p];
  }
}

hipError_t b3_pack(const B3PackJobs& jobs, hipStream_t st) {
  if (jobs.n <= 0) return hipSuccess;
  if (jobs.n > kMaxB3PackJobs) return hipErrorInvalidValue;
  int64_t mx = 0;
  for (int i = 0; i < jobs.n; ++i) {
    const int64_t t = (int64_t)jobs.job[i].nk * jobs.job[i].rows * 4;
    mx = t > mx ? t : mx;
  }
  int gx = (int)((mx + 255) / 256);
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  hipLaunchKernelGGL(k_b3_pack, dim3(gx, jobs.n), dim3(256), 0, st, jobs);
  return hipGetLastError();
}

}  // namespace cgr
