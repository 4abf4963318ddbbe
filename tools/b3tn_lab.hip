// Lab for the split-bf16 TN GEMM (csrc/gemm_b3.hpp, weight gradients): correctness against an
// fp64 host reference and timing at the cfg2 shapes beside the fp32 register-direct kernel.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/b3tn_lab.hip -o tools/b3tn_lab
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_b3.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_tnr.hpp"
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

// dW[n][k] = sum_e A[e][n] * B(e, k); B plain (gather = false) or a[src] - h[rev] (gather = true)
static void test_tn(int R, int Nout, int Kout, bool gather, hipStream_t st) {
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
  CK(hipMalloc(&slab, (size_t)p.splits * Nout * ldb * 4));
  CK(hipMalloc(&bslab, (size_t)p.splits * Nout * 4));
  CK(hipMalloc(&out, (size_t)Nout * Kout * 4));
  CK(hipMalloc(&bias, (size_t)Nout * 4));
  LdPlain<4> al{dA, lda};
  if (gather) {
    LdGatherDiff<false> bl{da, dh, dsrc, drev, ldb};
    CK(launch_b3tn(al, bl, p, slab, bslab, Nout, Kout, R, true, st));
  } else {
    LdPlain<4> bl{dB, ldb};
    CK(launch_b3tn(al, bl, p, slab, bslab, Nout, Kout, R, true, st));
  }
  CK(reduce_slabs(slab, bslab, p.splits, Nout, Kout, out, Kout, 0, bias, st));
  CK(hipStreamSynchronize(st));
  auto C = tohost(out, (size_t)Nout * Kout), bb = tohost(bias, Nout);
  double worst = 0, bworst = 0, gmax = 0;
  std::vector<double> ref((size_t)Nout * Kout, 0.0), mag((size_t)Nout * Kout, 0.0), bref(Nout, 0.0);
  for (int e = 0; e < R; ++e)
    for (int n = 0; n < Nout; ++n) {
      const double av = A[(size_t)e * lda + n];
      bref[n] += av;
      for (int k = 0; k < Kout; ++k) {
        const double bv = gather ? (double)a[(size_t)src[e] * ldb + k] - (double)h[(size_t)rev[e] * ldb + k]
                                 : (double)Bp[(size_t)e * ldb + k];
        ref[(size_t)n * Kout + k] += av * bv;
        mag[(size_t)n * Kout + k] += fabs(av * bv);
      }
    }
  for (size_t i = 0; i < ref.size(); ++i) {
    worst = std::max(worst, fabs(C[i] - ref[i]) / (mag[i] + 1e-30));
    gmax = std::max(gmax, fabs(ref[i]));
  }
  for (int n = 0; n < Nout; ++n) bworst = std::max(bworst, fabs(bb[n] - bref[n]) / (fabs(bref[n]) + 1.0));
  printf("tn R=%d N=%d K=%d %s splits=%d tiles_k=%d: max err / sum|ab| = %.3e, bias %.3e %s\n", R,
         Nout, Kout, gather ? "gather" : "plain", p.splits, p.tiles_k, worst, bworst,
         (worst < 2e-5 && bworst < 1e-5) ? "OK" : "FAIL");
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(da));
  CK(hipFree(dh));
  CK(hipFree(slab));
  CK(hipFree(bslab));
  CK(hipFree(out));
  CK(hipFree(bias));
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  test_tn(3000, 400, 400, false, st);
  test_tn(3000, 400, 400, true, st);
  test_tn(1000, 37, 45, false, st);
  test_tn(2000, 512, 512, true, st);
  test_tn(1500, 128, 848, false, st);
  {  // timing at cfg2: layer weight gradient (E = 15360, dpre^T (a[src] - h[rev])), node TN
    const int E = 15360, Nn = 7680, H = 400, Hp = 400, F = 848;
    auto dp = hrand((size_t)E * Hp, 51), a = hrand((size_t)Nn * Hp, 52), h = hrand((size_t)E * Hp, 53);
    auto Gs = hrand((size_t)Nn * Hp, 54), x = hrand((size_t)Nn * F, 55);
    std::vector<int> src(E), rev(E);
    srand(9);
    for (int i = 0; i < E; ++i) {
      const int g = i / 60;
      src[i] = g * 30 + rand() % 30;
      rev[i] = g * 60 + (rand() % 60);
    }
    float *ddp = todev(dp), *da = todev(a), *dh = todev(h), *dGs = todev(Gs), *dx = todev(x);
    int *dsrc = todev(src), *drev = todev(rev);
    float *slab, *bslab, *out, *bias;
    CK(hipMalloc(&slab, (size_t)256 * H * 1248 * 4));
    CK(hipMalloc(&bslab, (size_t)256 * H * 4));
    CK(hipMalloc(&out, (size_t)H * 1248 * 4));
    CK(hipMalloc(&bias, (size_t)H * 4));
    const double fl = 2.0 * E * H * H, fln = 2.0 * Nn * H * F;
    const B3TnPlan p = b3tn_plan(H, H, E);
    LdPlain<4> al{ddp, Hp};
    LdGatherDiff<false> bl{da, dh, dsrc, drev, Hp};
    float t = time_us([&] { CK(launch_b3tn(al, bl, p, slab, bslab, H, H, E, true, st)); }, st);
    float tr = time_us([&] { CK(reduce_slabs(slab, bslab, p.splits, H, H, out, H, 0, bias, st)); }, st);
    printf("b3  layer wgrad E=%d splits=%d: %.1f us (%.1f TFLOP/s fp32-equiv) + reduce %.1f us\n", E,
           p.splits, t, fl / t * 1e-6, tr);
    const B3TnPlan pn = b3tn_plan(H, F, Nn);
    LdPlain<4> aln{dGs, Hp}, bln{dx, F};
    t = time_us([&] { CK(launch_b3tn(aln, bln, pn, slab, bslab, H, F, Nn, false, st)); }, st);
    tr = time_us([&] { CK(reduce_slabs(slab, bslab, pn.splits, H, F, out, F, 0, nullptr, st)); }, st);
    printf("b3  node wgrad N=%d splits=%d: %.1f us (%.1f TFLOP/s) + reduce %.1f us\n", Nn, pn.splits, t,
           fln / t * 1e-6, tr);
    // fp32 register-direct reference kernel
    const TnrPlan q = plan_tnr<5, 5>(H, H, E, 512);
    t = time_us([&] {
      CK((launch_gemm_tnr<5, 5>(TnrRows{ddp, Hp}, TnrDiff{da, dh, dsrc, drev, Hp}, q, slab, bslab, H,
                                H, E, true, st)));
    }, st);
    tr = time_us([&] { CK(reduce_slabs(slab, bslab, q.splits, H, H, out, H, 0, bias, st)); }, st);
    printf("f32 layer wgrad (tnr) splits=%d: %.1f us (%.1f TFLOP/s) + reduce %.1f us\n", q.splits, t,
           fl / t * 1e-6, tr);
  }
  return 0;
}
