// Lab for the plane-operand TN GEMM (csrc/gemm_b3tp.hpp): correctness against an fp64 host
// reference (operands split on the host exactly as the producers will: hi = RNE bf16(x),
// lo = RNE bf16(x - hi)) and timing at the cfg2 shapes beside the staging TN (gemm_b3.hpp).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/b3tp_lab.hip -o tools/b3tp_lab
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_b3tp.hpp"
#include "../cgr-mpnn-3d_amd/csrc/kernels.hip"

using namespace cgr;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

static uint16_t bf16_rne(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  const uint32_t r = 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)((u + r) >> 16);
}
static float bf16_f(uint16_t h) {
  const uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static std::vector<float> hrand(size_t n, unsigned seed, float scale = 1.f) {
  std::vector<float> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((rand() / (float)RAND_MAX) * 2.f - 1.f);
  return h;
}
template <class T>
static T* todev(const std::vector<T>& h) {
  T* d;
  CK(hipMalloc(&d, h.size() * sizeof(T) + 64));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}
static std::vector<float> tohost(const float* d, size_t n) {
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
  return h;
}
template <class F>
static float time_us(F&& f, hipStream_t st, int reps = 20, int rounds = 5) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  f();
  CK(hipStreamSynchronize(st));
  std::vector<float> t;
  for (int r = 0; r < rounds; ++r) {
    CK(hipEventRecord(e0, st));
    for (int k = 0; k < reps; ++k) f();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1000.f / reps);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

// planes of a [R][W] fp32 matrix: rows padded to round_up(R, 32) with zeros, ld = b3tp_ld(W)
struct HostPlanes {
  std::vector<uint16_t> hi, lo;
  int64_t ld;
};
static HostPlanes make_planes(const std::vector<float>& m, int R, int W) {
  HostPlanes p;
  p.ld = b3tp_ld(W + 64);  // covers the last tile's columns for every tiling tested
  const int64_t rows = b3tp_rows(R);
  p.hi.assign(rows * p.ld, 0);
  p.lo.assign(rows * p.ld, 0);
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < W; ++c) {
      const float x = m[(size_t)r * W + c];
      const uint16_t h = bf16_rne(x);
      p.hi[r * p.ld + c] = h;
      p.lo[r * p.ld + c] = bf16_rne(x - bf16_f(h));
    }
  return p;
}

struct DevCase {
  uint16_t *ahi, *alo, *bhi, *blo;
  float* a32;
  B3Planes A, B;
};
static DevCase upload(const HostPlanes& a, const HostPlanes& b, const std::vector<float>& a32) {
  DevCase d;
  d.ahi = todev(a.hi);
  d.alo = todev(a.lo);
  d.bhi = todev(b.hi);
  d.blo = todev(b.lo);
  d.a32 = todev(a32);
  d.A = B3Planes{d.ahi, d.alo, a.ld};
  d.B = B3Planes{d.bhi, d.blo, b.ld};
  return d;
}
static void release(DevCase& d) {
  CK(hipFree(d.ahi));
  CK(hipFree(d.alo));
  CK(hipFree(d.bhi));
  CK(hipFree(d.blo));
  CK(hipFree(d.a32));
}

static void test_tp(int R, int Nout, int Kout, hipStream_t st, int tnn = 25, int tnk = 5) {
  auto A = hrand((size_t)R * Nout, 41 + R), B = hrand((size_t)R * Kout, 42 + Kout);
  const HostPlanes pa = make_planes(A, R, Nout), pb = make_planes(B, R, Kout);
  std::vector<float> a32((size_t)R * ((Nout + 3) & ~3), 0.f);  // fp32 A, 16-byte rows
  const int lda32 = (Nout + 3) & ~3;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < Nout; ++c) a32[(size_t)r * lda32 + c] = A[(size_t)r * Nout + c];
  DevCase d = upload(pa, pb, a32);
  const B3TpPlan p = plan_b3tp(Nout, Kout, R, tnn, tnk, 176);
  const int ldk = (Kout + 3) & ~3;
  float *slab, *bslab, *out, *bias;
  CK(hipMalloc(&slab, (size_t)p.splits * Nout * ldk * 4));
  CK(hipMalloc(&bslab, (size_t)p.splits * Nout * 4));
  CK(hipMalloc(&out, (size_t)Nout * Kout * 4));
  CK(hipMalloc(&bias, (size_t)Nout * 4));
  const hipError_t le = launch_b3tp(d.A, d.B, d.a32, lda32, p, slab, bslab, Nout, Kout, R, true, st);
  if (le != hipSuccess) {
    printf("tp R=%d N=%d K=%d: launch refused (%s)\n", R, Nout, Kout, hipGetErrorString(le));
    return;
  }
  CK(reduce_slabs(slab, bslab, p.splits, Nout, Kout, out, Kout, 0, bias, st));
  CK(hipStreamSynchronize(st));
  auto C = tohost(out, (size_t)Nout * Kout), bb = tohost(bias, Nout);
  double worst = 0, bworst = 0;
  std::vector<double> ref((size_t)Nout * Kout, 0.0), mag((size_t)Nout * Kout, 0.0), bref(Nout, 0.0),
      bmag(Nout, 0.0);
  for (int e = 0; e < R; ++e)
    for (int n = 0; n < Nout; ++n) {
      const double av = A[(size_t)e * Nout + n];
      bref[n] += av;
      bmag[n] += fabs(av);
      for (int k = 0; k < Kout; ++k) {
        const double bv = B[(size_t)e * Kout + k];
        ref[(size_t)n * Kout + k] += av * bv;
        mag[(size_t)n * Kout + k] += fabs(av * bv);
      }
    }
  for (size_t i = 0; i < ref.size(); ++i) worst = std::max(worst, fabs(C[i] - ref[i]) / (mag[i] + 1e-30));
  for (int n = 0; n < Nout; ++n) bworst = std::max(bworst, fabs(bb[n] - bref[n]) / (bmag[n] + 1e-30));
  printf("tp %dx%d R=%d N=%d K=%d splits=%d tiles %dx%d: max err / sum|ab| = %.3e, bias %.3e %s\n",
         tnn, tnk, R, Nout, Kout, p.splits, p.tiles_n, p.tiles_k, worst, bworst,
         (worst < 2e-5 && bworst < 1e-6) ? "OK" : "FAIL");
  release(d);
  CK(hipFree(slab));
  CK(hipFree(bslab));
  CK(hipFree(out));
  CK(hipFree(bias));
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  test_tp(3000, 400, 400, st);
  test_tp(3000, 400, 400, st, 13, 13);
  test_tp(1000, 37, 45, st, 8, 5);
  test_tp(2000, 128, 848, st, 8, 5);
  test_tp(1500, 96, 400, st, 13, 13);
  test_tp(4100, 400, 1248, st);
  test_tp(4100, 400, 1248, st, 13, 13);
  {  // timing at cfg2: layer (E x 400 x 400) and node (N x 400 x 848) weight gradients
    const int E = 15360, Nn = 7680, H = 400, F = 848;
    auto A = hrand((size_t)E * H, 51), B = hrand((size_t)E * H, 52);
    DevCase d = upload(make_planes(A, E, H), make_planes(B, E, H), A);
    float *slab, *bslab;
    CK(hipMalloc(&slab, (size_t)256 * H * 1248 * 4));
    CK(hipMalloc(&bslab, (size_t)256 * H * 4));
    const double fl = 2.0 * E * H * H;
    for (int v = 0; v < 2; ++v) {
      const int tnn = v ? 13 : 25, tnk = v ? 13 : 5;
      for (int target : {128, 176, 256}) {
        const B3TpPlan p = plan_b3tp(H, H, E, tnn, tnk, target);
        float t = time_us([&] { CK(launch_b3tp(d.A, d.B, d.a32, H, p, slab, bslab, H, H, E, true, st)); }, st);
        float tr = time_us([&] { CK(reduce_slabs(slab, bslab, p.splits, H, H, slab + (size_t)200 * H * 1248, H, 0, bslab + 200 * H, st)); }, st);
        printf("tp %dx%d layer wgrad E=%d target %d splits=%d: %.1f us (%.1f TFLOP/s) + reduce %.1f us\n",
               tnn, tnk, E, target, p.splits, t, fl / t * 1e-6, tr);
      }
    }
    release(d);
    auto An = hrand((size_t)Nn * H, 53), Bn = hrand((size_t)Nn * F, 54);
    DevCase dn = upload(make_planes(An, Nn, H), make_planes(Bn, Nn, F), An);
    for (int v = 0; v < 2; ++v) {
      const int tnn = v ? 13 : 25, tnk = v ? 13 : 5;
      const B3TpPlan pn = plan_b3tp(H, F, Nn, tnn, tnk, 176);
      float t = time_us([&] { CK(launch_b3tp(dn.A, dn.B, dn.a32, H, pn, slab, bslab, H, F, Nn, true, st)); }, st);
      printf("tp %dx%d node wgrad N=%d splits=%d: %.1f us (%.1f TFLOP/s)\n", tnn, tnk, Nn, pn.splits, t,
             2.0 * Nn * H * F / t * 1e-6);
    }
    release(dn);
  }
  return 0;
}
