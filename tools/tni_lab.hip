// Lab for the e-image split-bf16 TN (csrc/gemm_b3.hpp gemm_b3tni_kernel): correctness against an
// fp64 host reference and timing at the cfg2 shapes (layer, readout-like, node weight gradients).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude tools/tni_lab.hip
// (the round-3 ablation switches -DCGR_TNI_LAB=mask lived in the shipped header and were removed
// in round 4; their results: DESIGN.md §4, e-image TN lab figures)
//   ablation mask: 1 no B loads, 2 no A loads, 4 no MFMA, 8 no B staging (split + LDS stores)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_b3.hpp"
#include "../cgr-mpnn-3d_amd/csrc/b3_pack.hip"
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

static std::vector<float> hrand(size_t n, unsigned seed, float scale = 1.f) {
  std::vector<float> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((rand() / (float)RAND_MAX) * 2.f - 1.f);
  return h;
}
template <class T>
static T* todev(const std::vector<T>& h) {
  T* d;
  CK(hipMalloc(&d, h.size() * sizeof(T)));
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

// dW[n][k] = sum_e A[e][n] * B(e, k); B plain or a[src] - h[rev]
static void check(int R, int Nout, int Kout, bool gather, hipStream_t st) {
  const int lda = (Nout + 3) & ~3, ldb = (Kout + 3) & ~3;
  const int Nn = R / 2 + 1;
  auto A = hrand((size_t)R * lda, 41);
  auto Bp = hrand((size_t)R * ldb, 42);
  auto a = hrand((size_t)Nn * ldb, 43), h = hrand((size_t)R * ldb, 44);
  std::vector<int> src(R), rev(R);
  srand(45);
  for (int i = 0; i < R; ++i) {
    src[i] = rand() % Nn;
    rev[i] = rand() % R;
  }
  float *dA = todev(A), *dB = todev(Bp), *da = todev(a), *dh = todev(h);
  int *dsrc = todev(src), *drev = todev(rev);
  const B3TnPlan p = b3tn_plan(Nout, Kout, R);
  float *slab, *bslab, *out, *bias;
  b3_u4* img;
  CK(hipMalloc(&img, b3_eimg_bytes(R, Nout)));
  CK(hipMalloc(&slab, (size_t)p.splits * Nout * ldb * 4));
  CK(hipMalloc(&bslab, (size_t)p.splits * Nout * 4));
  CK(hipMalloc(&out, (size_t)Nout * Kout * 4));
  CK(hipMalloc(&bias, (size_t)Nout * 4));
  CK(b3_eimage(dA, lda, R, Nout, img, st));
  const B3EImg ai{img, b3_eimg_cols(Nout)};
  if (gather) {
    LdGatherDiff<false> bl{da, dh, dsrc, drev, ldb};
    CK(launch_b3tni(ai, bl, p, slab, bslab, Nout, Kout, R, true, st));
  } else {
    LdPlain<4> bl{dB, ldb};
    CK(launch_b3tni(ai, bl, p, slab, bslab, Nout, Kout, R, true, st));
  }
  CK(reduce_slabs(slab, bslab, p.splits, Nout, Kout, out, Kout, 0, bias, st));
  CK(hipStreamSynchronize(st));
  auto C = tohost(out, (size_t)Nout * Kout), bb = tohost(bias, Nout);
  double worst = 0, bworst = 0;
  std::vector<double> ref((size_t)Nout * Kout, 0.0), mag((size_t)Nout * Kout, 0.0), bref(Nout, 0.0),
      bmag(Nout, 0.0);
  for (int e = 0; e < R; ++e)
    for (int n = 0; n < Nout; ++n) {
      const double av = A[(size_t)e * lda + n];
      bref[n] += av;
      bmag[n] += fabs(av);
      for (int k = 0; k < Kout; ++k) {
        const double bv = gather ? (double)a[(size_t)src[e] * ldb + k] - (double)h[(size_t)rev[e] * ldb + k]
                                 : (double)Bp[(size_t)e * ldb + k];
        ref[(size_t)n * Kout + k] += av * bv;
        mag[(size_t)n * Kout + k] += fabs(av * bv);
      }
    }
  for (size_t i = 0; i < ref.size(); ++i) worst = std::max(worst, fabs(C[i] - ref[i]) / (mag[i] + 1e-30));
  for (int n = 0; n < Nout; ++n) bworst = std::max(bworst, fabs(bb[n] - bref[n]) / (bmag[n] + 1e-30));
  printf("tni R=%d N=%d K=%d %s splits=%d tiles_k=%d: max err / sum|ab| = %.3e, bias / sum|a| %.3e %s\n",
         R, Nout, Kout, gather ? "gather" : "plain", p.splits, p.tiles_k, worst, bworst,
         (worst < 2e-5 && bworst < 1e-5) ? "OK" : "FAIL");
  CK(hipFree(dA)); CK(hipFree(dB)); CK(hipFree(da)); CK(hipFree(dh)); CK(hipFree(img));
  CK(hipFree(slab)); CK(hipFree(bslab)); CK(hipFree(out)); CK(hipFree(bias));
}

int main(int argc, char** argv) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  check(3000, 400, 400, false, st);
  check(3000, 400, 400, true, st);
  check(1000, 37, 45, false, st);
  check(2000, 512, 512, true, st);
  check(1500, 128, 848, false, st);
  check(1100, 64, 130, true, st);
  const int E = 15360, Nn = 7680, H = 400, Hp = 400, F = 848;
  auto dp = hrand((size_t)E * Hp, 51), a = hrand((size_t)Nn * Hp, 52), h = hrand((size_t)E * Hp, 53);
  auto Gs = hrand((size_t)Nn * Hp, 54), x = hrand((size_t)Nn * F, 55);
  std::vector<int> src(E), rev(E);
  srand(9);
  for (int i = 0; i < E; ++i) {  // T1x-like locality: rows of one reaction
    const int g = i / 60;
    src[i] = g * 30 + rand() % 30;
    rev[i] = g * 60 + (rand() % 60);
  }
  float *ddp = todev(dp), *da = todev(a), *dh = todev(h), *dGs = todev(Gs), *dx = todev(x);
  int *dsrc = todev(src), *drev = todev(rev);
  float *slab, *bslab, *out, *bias;
  b3_u4 *img, *imgn;
  CK(hipMalloc(&img, b3_eimg_bytes(E, H)));
  CK(hipMalloc(&imgn, b3_eimg_bytes(Nn, H)));
  CK(hipMalloc(&slab, (size_t)256 * H * 1248 * 4));
  CK(hipMalloc(&bslab, (size_t)256 * H * 4));
  CK(hipMalloc(&out, (size_t)H * 1248 * 4));
  CK(hipMalloc(&bias, (size_t)H * 4));
  const double fl = 2.0 * E * H * H, fln = 2.0 * Nn * H * F;
  const int target = argc > 1 ? atoi(argv[1]) : kB3TnTarget;
  float t = time_us([&] { CK(b3_eimage(ddp, Hp, E, H, img, st)); }, st);
  printf("eimage E=%d H=%d: %.1f us (%.2f TB/s of 8 B/elem)\n", E, H, t, 8.0 * E * H / t * 1e-6);
  const B3TnPlan p = b3tn_plan(H, H, E, target);
  LdGatherDiff<false> bl{da, dh, dsrc, drev, Hp};
  const B3EImg ai{img, b3_eimg_cols(H)};
  t = time_us([&] { CK(launch_b3tni(ai, bl, p, slab, bslab, H, H, E, true, st)); }, st);
  float tr = time_us([&] { CK(reduce_slabs(slab, bslab, p.splits, H, H, out, H, 0, bias, st)); }, st);
  printf("tni layer wgrad E=%d target=%d splits=%d wgs=%d: %.1f us (%.1f TFLOP/s fp32-equiv) + reduce %.1f us\n",
         E, target, p.splits, p.splits * p.tiles_k, t, fl / t * 1e-6, tr);
  CK(b3_eimage(dGs, Hp, Nn, H, imgn, st));
  const B3TnPlan pn = b3tn_plan(H, F, Nn, 256);
  LdPlain<4> bln{dx, F};
  const B3EImg an{imgn, b3_eimg_cols(H)};
  t = time_us([&] { CK(launch_b3tni(an, bln, pn, slab, bslab, H, F, Nn, false, st)); }, st);
  printf("tni node wgrad N=%d splits=%d: %.1f us (%.1f TFLOP/s)\n", Nn, pn.splits, t, fln / t * 1e-6);
  return 0;
}
