// Weight images for the split-bf16 NT GEMMs (gemm_b3.hpp): every weight matrix an NT GEMM reads
// as its B operand is split into three bf16 pieces once per training step (the forward packs
// W_l, W_l^T, [W0[:, :F]; W_n[:, :F]], W_n[:, F:] and W_n[:, F:]^T in one batched launch).
#include "gemm_b3.hpp"

namespace cgr {

// one thread per (k step, image row, lane-group chunk): 8 source values -> 3 pieces -> the chunk's
// swizzled slot in each piece plane.  Row-major sources (ldk == 1) run chunks fastest (adjacent
// threads read adjacent k), transposed sources (ldn == 1) run rows fastest (adjacent n).
__device__ __forceinline__ void b3_pack_job(const B3PackJob& J, int64_t first, int64_t stride) {
  const int64_t total = (int64_t)J.nk * J.rows * 4;
  const bool rowmajor = J.ldk == 1;
  for (int64_t t = first; t < total; t += stride) {
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

__global__ __launch_bounds__(256) void k_b3_pack(B3PackJobs jobs) {
  b3_pack_job(jobs.job[blockIdx.y], (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
              (int64_t)gridDim.x * blockDim.x);
}

// blocks [0, pad_blocks): one float4 of xp per thread (two 8-byte loads when F is even); blocks
// past them: the image jobs, (block - pad_blocks) = job * gx + bx
__global__ __launch_bounds__(256) void k_b3_pack_pad(B3PackJobs jobs, B3PadJob pd, int pad_blocks,
                                                     int gx) {
  if ((int)blockIdx.x < pad_blocks) {
    const int c4n = pd.ldp >> 2;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= pd.N * c4n) return;
    const int64_t r = t / c4n;
    const int k = 4 * (int)(t - r * c4n);
    const float* src = pd.x + r * pd.F;
    float4 v;
    if ((pd.F & 1) == 0) {
      const float2 u = k < pd.F ? *reinterpret_cast<const float2*>(src + k) : make_float2(0.f, 0.f);
      const float2 w =
          k + 2 < pd.F ? *reinterpret_cast<const float2*>(src + k + 2) : make_float2(0.f, 0.f);
      v = make_float4(u.x, u.y, w.x, w.y);
    } else {
      v.x = k < pd.F ? src[k] : 0.f;
      v.y = k + 1 < pd.F ? src[k + 1] : 0.f;
      v.z = k + 2 < pd.F ? src[k + 2] : 0.f;
      v.w = k + 3 < pd.F ? src[k + 3] : 0.f;
    }
    *reinterpret_cast<float4*>(pd.xp + r * pd.ldp + k) = v;
    return;
  }
  const int b = (int)blockIdx.x - pad_blocks;
  const int j = b / gx, bx = b - j * gx;
  b3_pack_job(jobs.job[j], (int64_t)bx * blockDim.x + threadIdx.x, (int64_t)gx * blockDim.x);
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

static int b3_pack_gx(const B3PackJobs& jobs) {
  int64_t mx = 0;
  for (int i = 0; i < jobs.n; ++i) {
    const int64_t t = (int64_t)jobs.job[i].nk * jobs.job[i].rows * 4;
    mx = t > mx ? t : mx;
  }
  int gx = (int)((mx + 255) / 256);
  return gx < 1 ? 1 : (gx > 256 ? 256 : gx);
}

hipError_t b3_pack_pad(const B3PackJobs& jobs, const B3PadJob& pad, hipStream_t st) {
  if (jobs.n > kMaxB3PackJobs) return hipErrorInvalidValue;
  const int64_t tot = pad.N * (pad.ldp >> 2);
  const int pb = (int)((tot + 255) / 256);
  const int gx = b3_pack_gx(jobs);
  const int nb = pb + gx * (jobs.n > 0 ? jobs.n : 0);
  if (nb <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_b3_pack_pad, dim3(nb), dim3(256), 0, st, jobs, pad, pb, gx);
  return hipGetLastError();
}

}  // namespace cgr
