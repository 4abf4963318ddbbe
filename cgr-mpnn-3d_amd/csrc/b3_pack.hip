// Weight images for the split-bf16 NT GEMMs (gemm_b3.hpp): every weight matrix an NT GEMM reads
// as its B operand is split into three bf16 pieces once per training step (the forward packs
// W_l, W_l^T, [W0[:, :F]; W_n[:, :F]], W_n[:, F:] and W_n[:, F:]^T in one batched launch).
#include <algorithm>

#include "bwd_rows.hpp"
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
      if (J.kscale && k < J.K) f[j] *= J.kscale[k];
    }
    b3_u4 pc[3];
    b3_split8<3>(f, pc);
    const int n = J.n_begin + nl;
    const int slot = c ^ lds_swz(n);
#pragma unroll
    for (int p = 0; p < 3; ++p) J.img[((int64_t)(ks * 3 + p) * J.nimg + n) * 4 + slot] = pc[p];
  }
}

// Block ranges of one launch: jobs.n pack jobs of gx blocks each, then the riders' blocks
// (B3PackRiders: transpose tb, zero fill zb, row padding pb blocks, each grid-strided).
struct B3PackGrid {
  int gx, tb, zb, pb;
};

__global__ __launch_bounds__(256) void k_b3_pack(B3PackJobs jobs, B3PackRiders r, B3PackGrid g) {
  int b = blockIdx.x;
  if (b < jobs.n * g.gx) {
    const int j = b / g.gx;
    b3_pack_job(jobs.job[j], (int64_t)(b - j * g.gx) * blockDim.x + threadIdx.x,
                (int64_t)g.gx * blockDim.x);
    return;
  }
  b -= jobs.n * g.gx;
  if (b < g.tb) {  // rows fastest: adjacent threads write adjacent destination words
    const int64_t tot = (int64_t)r.t_rows * r.t_cols;
    for (int64_t t = (int64_t)b * blockDim.x + threadIdx.x; t < tot;
         t += (int64_t)g.tb * blockDim.x) {
      const int row = (int)(t % r.t_rows), c = (int)(t / r.t_rows);
      r.t_dst[(int64_t)c * r.t_ld_dst + row] = r.t_src[(int64_t)row * r.t_ld_src + c];
    }
    return;
  }
  b -= g.tb;
  if (b < g.zb) {
    for (int64_t t = (int64_t)b * blockDim.x + threadIdx.x; t < r.z_u4;
         t += (int64_t)g.zb * blockDim.x)
      static_cast<uint4*>(r.z_dst)[t] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  b -= g.zb;
  const int c4n = r.p_ld >> 2;
  const int64_t tot = r.p_rows * c4n;
  const bool vec2 = !(r.p_F & 1) && !((uintptr_t)r.p_src & 7);
  for (int64_t t = (int64_t)b * blockDim.x + threadIdx.x; t < tot; t += (int64_t)g.pb * blockDim.x)
    pad_row4(r.p_src, r.p_F, r.p_dst, r.p_ld, c4n, t, vec2);
}

hipError_t b3_pack(const B3PackJobs& jobs, hipStream_t st, const B3PackRiders* riders) {
  if (jobs.n < 0 || jobs.n > kMaxB3PackJobs) return hipErrorInvalidValue;
  int64_t mx = 0;
  for (int i = 0; i < jobs.n; ++i) {
    const int64_t t = (int64_t)jobs.job[i].nk * jobs.job[i].rows * 4;
    mx = t > mx ? t : mx;
  }
  B3PackGrid g{};
  g.gx = (int)std::min<int64_t>(std::max<int64_t>((mx + 255) / 256, 1), 256);
  B3PackRiders r{};
  if (riders) {
    r = *riders;
    if (r.t_src && r.t_dst && r.t_rows > 0 && r.t_cols > 0)
      g.tb = (int)std::min<int64_t>(cdiv((int64_t)r.t_rows * r.t_cols, 256), 64);
    if (r.z_dst && r.z_u4 > 0) {
      if ((uintptr_t)r.z_dst & 15) return hipErrorInvalidValue;
      g.zb = (int)std::min<int64_t>(cdiv(r.z_u4, 256), 256);
    }
    if (r.p_src && r.p_dst && r.p_rows > 0) {
      if ((r.p_ld & 3) || r.p_ld < r.p_F || ((uintptr_t)r.p_dst & 15) || ((uintptr_t)r.p_src & 3))
        return hipErrorInvalidValue;
      g.pb = (int)std::min<int64_t>(cdiv(r.p_rows * (r.p_ld >> 2), 256), 2048);
    }
  }
  const int64_t blocks = (int64_t)jobs.n * g.gx + g.tb + g.zb + g.pb;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_b3_pack, dim3((unsigned)blocks), dim3(256), 0, st, jobs, r, g);
  return hipGetLastError();
}

// e-image of X [R, C] (gemm_b3.hpp, B3EImg): thread = (32-row step s, column c, 8-row chunk q),
// chunk fastest, so the four lanes of one column write its 64-byte slot of a plane whole and a
// wave's stores cover 16 consecutive slots; its 8 loads (rows 32 s + 8 q + j, column c) run over
// 16 consecutive columns of 4 rows per instruction.  Rows >= R and columns >= C are written as 0.
__global__ __launch_bounds__(256) void k_b3_eimage(const float* __restrict__ x, int64_t ld,
                                                   int64_t R, int C, int cimg, int64_t steps,
                                                   b3_u4* __restrict__ img) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= steps * cimg * 4) return;
  const int q = (int)(t & 3);
  const int64_t u = t >> 2;
  const int c = (int)(u % cimg);
  const int64_t s = u / cimg;
  const int64_t r0 = s * 32 + 8 * q;
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t r = r0 + j;
    f[j] = (r < R && c < C) ? x[r * ld + c] : 0.f;
  }
  b3_u4 pc[2];
  b3_split8<2>(f, pc);
  img[((s * 2 + 0) * cimg + c) * 4 + q] = pc[0];
  img[((s * 2 + 1) * cimg + c) * 4 + q] = pc[1];
}

hipError_t b3_eimage(const float* x, int64_t ld, int64_t R, int C, b3_u4* img, hipStream_t st) {
  const int64_t steps = (R + 31) / 32;
  const int cimg = b3_eimg_cols(C);
  const int64_t tot = steps * cimg * 4;
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_b3_eimage, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, x, ld, R,
                     C, cimg, steps, img);
  return hipGetLastError();
}

// e-image of the segmented sum G[v, :C] = sum_{j in [ptr[v], ptr[v+1])} X[idx[j], :C] (the node
// weight gradient's Gs = segsum_src(dpre0), gnn_bwd.hip) without G ever reaching memory.  Block =
// one 32-row step s x 64 columns: the sums (thread = (row, float4 column), the segment's rows in
// order, as k_segsum_v4m adds them) go to an LDS tile [32][65], then thread = (column, 8-row chunk),
// chunk fastest, splits its 8 values and writes the two 16-byte chunk slots (a wave's stores cover
// 16 consecutive 64-byte slots).  Rows >= R and columns >= C are written as 0.
constexpr int kSegImgCols = 64;
__global__ __launch_bounds__(256) void k_b3_segsum_eimage(const float* __restrict__ x, int64_t ld_,
                                                          const int* __restrict__ idx,
                                                          const int* __restrict__ ptr, int64_t R,
                                                          int C, int cimg,
                                                          b3_u4* __restrict__ img) {
  __shared__ float tile[32][kSegImgCols + 1];
  const int64_t s = blockIdx.y;
  const int c0 = blockIdx.x * kSegImgCols;
  // two (row, float4 column) items per thread (rows r and r + 16), every load of both in flight
  // together: the first three rows of each segment with clamped indices (segments average ~2
  // rows), the rest in a loop -- the runtime-trip-count loop alone serialised idx -> row -> add
  // (10.3 us in the step at cfg2 for 37 MB)
  static_assert(32 * (kSegImgCols / 4) == 2 * 256, "two items per thread of a 256-thread block");
  const int r0 = threadIdx.x / (kSegImgCols / 4), c4 = threadIdx.x % (kSegImgCols / 4);
  const int cc = c0 + 4 * c4;
  const bool colok = cc < C;
  int b[2], e[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t v = s * 32 + r0 + 16 * h;
    const bool ok = v < R && colok;
    b[h] = ok ? ptr[v] : 0;
    e[h] = ok ? ptr[v + 1] : 0;
  }
  const float* base = x + (colok ? cc : 0);
  auto ld = [&](int j) { return *reinterpret_cast<const float4*>(base + (int64_t)idx[j] * ld_); };
  float4 acc[2], x0[2], x1[2], x2[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // clamped into the segment; an empty segment loads nothing (idx may have no entries)
    const bool any = e[h] > b[h];
    const int last = any ? e[h] - 1 : 0;
    x0[h] = any ? ld(min(b[h], last)) : f4zero();
    x1[h] = any ? ld(min(b[h] + 1, last)) : f4zero();
    x2[h] = any ? ld(min(b[h] + 2, last)) : f4zero();
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int n = e[h] - b[h];
    float4 a = f4zero();
    if (n > 0) a = f4add(a, x0[h]);
    if (n > 1) a = f4add(a, x1[h]);
    if (n > 2) a = f4add(a, x2[h]);
    for (int j = b[h] + 3; j < e[h]; ++j) a = f4add(a, ld(j));
    acc[h] = a;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float a[4] = {acc[h].x, acc[h].y, acc[h].z, acc[h].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) tile[r0 + 16 * h][4 * c4 + k] = (cc + k < C) ? a[k] : 0.f;
  }
  __syncthreads();
  const int q = threadIdx.x & 3, cl = threadIdx.x >> 2;  // 64 columns x 4 chunks
  const int c = c0 + cl;
  if (c >= cimg) return;
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = tile[8 * q + j][cl];
  b3_u4 pc[2];
  b3_split8<2>(f, pc);
  img[((s * 2 + 0) * cimg + c) * 4 + q] = pc[0];
  img[((s * 2 + 1) * cimg + c) * 4 + q] = pc[1];
}

hipError_t b3_segsum_eimage(const float* x, int64_t ld, const int* idx, const int* ptr, int64_t R,
                            int C, b3_u4* img, hipStream_t st) {
  const int64_t steps = (R + 31) / 32;
  const int cimg = b3_eimg_cols(C);
  if (steps <= 0 || C <= 0) return hipSuccess;
  if ((ld & 3) || ld < (C + 3) / 4 * 4 || ((uintptr_t)x & 15)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_b3_segsum_eimage, dim3((cimg + kSegImgCols - 1) / kSegImgCols,
                                              (unsigned)steps), dim3(256), 0, st, x, ld, idx, ptr,
                     R, C, cimg, img);
  return hipGetLastError();
}


// ------------------------------------------------------------------------------------------
// Producers that write the weight-gradient TN's e-image themselves (no k_b3_eimage pass over
// their output): block = one 32-row step x 64 columns.  Phase 1, thread = (row, float4 column):
// the element-wise backward of the row, its fp32 result to global (float4 rows, as before) and
// into an LDS tile; phase 2, thread = (column, 8-row chunk), chunk fastest: the chunk's two
// bf16 pieces into the image (k_b3_eimage's store pattern).  Rows >= R / columns >= C are 0.
// ------------------------------------------------------------------------------------------
constexpr int kImgCols = 64;

__device__ __forceinline__ void b3_tile_to_eimage(const float (&tile)[32][kImgCols + 1], int64_t s,
                                                  int c0, int cimg, b3_u4* __restrict__ img) {
  const int q = threadIdx.x & 3, cl = threadIdx.x >> 2;  // 64 columns x 4 chunks
  const int c = c0 + cl;
  if (c >= cimg) return;
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = tile[8 * q + j][cl];
  b3_u4 pc[2];
  b3_split8<2>(f, pc);
  img[((s * 2 + 0) * cimg + c) * 4 + q] = pc[0];
  img[((s * 2 + 1) * cimg + c) * 4 + q] = pc[1];
}

__device__ __forceinline__ void b3_tile_put(float (&tile)[32][kImgCols + 1], int r, int c4,
                                            int col, int C, const float4& v) {
  tile[r][4 * c4 + 0] = col + 0 < C ? v.x : 0.f;
  tile[r][4 * c4 + 1] = col + 1 < C ? v.y : 0.f;
  tile[r][4 * c4 + 2] = col + 2 < C ? v.z : 0.f;
  tile[r][4 * c4 + 3] = col + 3 < C ? v.w : 0.f;
}

// readout backward (GNN.py:106-110 reversed): dzn[v, n] = dy[graph(v)] wf[n] act'(zn[v, n]); dg
// is never stored.  dzn (nullable) in fp32 and/or its e-image (nullable)
__global__ __launch_bounds__(256) void k_readout_bwd_img(
    const float* __restrict__ dy, const float* __restrict__ wf, const int* __restrict__ node_graph,
    const float* __restrict__ hn, const float* __restrict__ zn, int64_t N, int H, int Hp, int act,
    float* __restrict__ dzn, int colblocks, int cimg, b3_u4* __restrict__ img,
    const float* __restrict__ gscale, const int* __restrict__ pool_arg,
    const float* __restrict__ gpool) {
  __shared__ float tile[32][kImgCols + 1];
  const int64_t s = blockIdx.x / colblocks;
  const int c0 = (int)(blockIdx.x - s * colblocks) * kImgCols;
  for (int it = threadIdx.x; it < 32 * (kImgCols / 4); it += blockDim.x) {
    const int r = it / (kImgCols / 4), c4 = it - r * (kImgCols / 4);
    const int64_t v = s * 32 + r;
    const int n = c0 + 4 * c4;
    float4 o = f4zero();
    if (v < N && n < Hp) {
      const int64_t off = v * Hp + n;
      const int gv = node_graph[v];
      const float d = gscale ? dy[gv] * gscale[gv] : dy[gv];
      o.x = d * wf[min(n, H - 1)];
      o.y = d * wf[min(n + 1, H - 1)];
      o.z = d * wf[min(n + 2, H - 1)];
      o.w = d * wf[min(n + 3, H - 1)];
      if (pool_arg) {  // global_max_pool (pool_head_fwd's record, kernels.hpp)
        const int4 am = *reinterpret_cast<const int4*>(pool_arg + (int64_t)gv * Hp + n);
        const float4 h = *reinterpret_cast<const float4*>(hn + off);
        const float4 gm = *reinterpret_cast<const float4*>(gpool + (int64_t)gv * Hp + n);
        // the first arg-max node (>= 0), or every node holding the max sharing (-count)
        auto pick = [&](float ov, int a, float hv, float gmv) {
          if (a >= 0) return a == v ? ov : 0.f;
          return hv == gmv ? ov / (float)(-a) : 0.f;
        };
        o.x = pick(o.x, am.x, h.x, gm.x);
        o.y = pick(o.y, am.y, h.y, gm.y);
        o.z = pick(o.z, am.z, h.z, gm.z);
        o.w = pick(o.w, am.w, h.w, gm.w);
      }
      if (act == ACT_RELU) {
        const float4 h = *reinterpret_cast<const float4*>(hn + off);
        o.x = h.x > 0.f ? o.x : 0.f;
        o.y = h.y > 0.f ? o.y : 0.f;
        o.z = h.z > 0.f ? o.z : 0.f;
        o.w = h.w > 0.f ? o.w : 0.f;
      } else {
        const float4 z = *reinterpret_cast<const float4*>(zn + off);
        o.x *= act_grad(z.x, act);
        o.y *= act_grad(z.y, act);
        o.z *= act_grad(z.z, act);
        o.w *= act_grad(z.w, act);
      }
      if (dzn) *reinterpret_cast<float4*>(dzn + off) = o;
    }
    if (img) b3_tile_put(tile, r, c4, n, H, o);
  }
  if (!img) return;
  __syncthreads();
  b3_tile_to_eimage(tile, s, c0, cimg, img);
}

hipError_t readout_act_bwd(const float* dy, const float* wf, const int* node_graph,
                           const float* hn, const float* zn, int64_t N, int H, int Hp, int act,
                           float* dzn, void* img, hipStream_t st, const float* gscale,
                           const int* pool_arg, const float* gpool) {
  if (N <= 0 || (!dzn && !img)) return hipSuccess;
  const int colblocks = (int)cdiv(Hp, kImgCols);
  const int64_t blocks = cdiv(N, 32) * colblocks;
  hipLaunchKernelGGL(k_readout_bwd_img, dim3((unsigned)blocks), dim3(256), 0, st, dy, wf,
                     node_graph, hn, zn, N, H, Hp, act, dzn, colblocks, b3_eimg_cols(H),
                     static_cast<b3_u4*>(img), gscale, pool_arg, gpool);
  return hipGetLastError();
}

// top layer of the D-MPNN backward (GNN.py:94-102 reversed): dh_D[i] = ds[dst(i)] ->
// dpre = dh * keep/(1-p) * act'(pre) (bwd_rows.hpp layer_row_apply: dpre in fp32, the
// learnable-skip partial) + dpre's e-image (nullable).  Blocks past the image grid only write
// their (zero) skip partial.  Also zeroes what the fused layer-backward GEMMs accumulate (the
// tile-crossing entries of dag and of the ticket counters, the unpaired grid counters).
int layer_act_bwd_blocks(int64_t E, int Hp) { return (int)(cdiv(E, 32) * cdiv(Hp, kImgCols)); }

__global__ __launch_bounds__(256) void k_layer_bwd_img(LayerBwdArgs a, int colblocks, int cimg,
                                                       b3_u4* __restrict__ img) {
  __shared__ float tile[32][kImgCols + 1];
  __shared__ float red[4];
  const int64_t nimg = cdiv(a.E, 32) * colblocks;
  float dsig = 0.f;
  if (blockIdx.x < nimg) {
    const int64_t s = blockIdx.x / colblocks;
    const int c0 = (int)(blockIdx.x - s * colblocks) * kImgCols;
    const uint64_t key = a.thresh ? *a.seed : 0;
    for (int it = threadIdx.x; it < 32 * (kImgCols / 4); it += blockDim.x) {
      const int r = it / (kImgCols / 4), c4 = it - r * (kImgCols / 4);
      const int64_t i = s * 32 + r;
      const int n = c0 + 4 * c4;
      float4 dp = f4zero();
      if (i < a.E && n < a.Hp) {
        const float4 dh = *reinterpret_cast<const float4*>(a.ds + (int64_t)a.dst_s[i] * a.Hp + n);
        dp = layer_row_apply(a, i, n, dh, key, dsig, layer_row_loads(a, i, n));
      }
      if (img) b3_tile_put(tile, r, c4, n, a.H, dp);
    }
    if (img) {
      __syncthreads();
      b3_tile_to_eimage(tile, s, c0, cimg, img);
    }
  }
  if (a.dag) {  // zero what the fused layer-backward GEMMs accumulate (see EpLayerBwdSeg)
    const int C4 = a.Hp >> 2;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nb = cdiv(a.E, a.tile_rows) - 1;  // interior row-tile boundaries
    if (t < nb * C4) {
      const int64_t m = (t / C4 + 1) * a.tile_rows;
      const int c = (int)(t % C4);
      const int v = a.dst_s[m];
      if (a.dst_s[m - 1] == v) {
        *reinterpret_cast<float4*>(a.dag + (int64_t)v * a.Hp + 4 * c) = f4zero();
        if (c < a.cnt_tiles) a.cnt[(int64_t)v * a.cnt_tiles + c] = 0;
      }
    }
    if (t < CGR_MAX_DEPTH)  // the unpaired form's grid counters, one per fused launch
      a.cnt[a.cnt_nodes * a.cnt_tiles + t] = 0;
  }
  if (a.dsig_part) {
    dsig = wave_sum(dsig);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dsig;
    __syncthreads();
    if (threadIdx.x == 0) a.dsig_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

hipError_t layer_act_bwd(const LayerBwdArgs& a, int nblocks, void* img, hipStream_t st) {
  const int need = layer_act_bwd_blocks(a.E, a.Hp);
  const int nb = nblocks > need ? nblocks : need;  // extra blocks write zero partials
  if (need <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_layer_bwd_img, dim3(nb), dim3(256), 0, st, a, (int)cdiv(a.Hp, kImgCols),
                     b3_eimg_cols(a.H), static_cast<b3_u4*>(img));
  return hipGetLastError();
}

}  // namespace cgr
