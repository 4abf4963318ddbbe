// TN lab: the register-direct strided-fragment TN kernel (gemm_tnr.hpp) against the LDS-staged
// split-K TN kernel (gemm.hpp) on the layer weight gradient dW = dpre^T (a[src] - h[rev]) at cfg2
// (E 15360, H 400): reduced result compared, kernel times (slab reduction excluded).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tnr_lab.hip -o tools/tnr_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_tnr.hpp"

using namespace cgr;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = (rand() / (float)RAND_MAX) * 2.f - 1.f;
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
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

// host-side fixed-order slab sum (checker only)
static void reduce_host(const float* dslab, const float* dbslab, int splits, int Nout, int Kout,
                        std::vector<double>& W, std::vector<double>& b) {
  const int ldk = (Kout + 3) & ~3;
  std::vector<float> s((size_t)splits * Nout * ldk), bs((size_t)splits * Nout);
  CK(hipMemcpy(s.data(), dslab, s.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bs.data(), dbslab, bs.size() * 4, hipMemcpyDeviceToHost));
  W.assign((size_t)Nout * Kout, 0.0);
  b.assign(Nout, 0.0);
  for (int p = 0; p < splits; ++p)
    for (int n = 0; n < Nout; ++n) {
      for (int k = 0; k < Kout; ++k) W[(size_t)n * Kout + k] += s[((size_t)p * Nout + n) * ldk + k];
      b[n] += bs[(size_t)p * Nout + n];
    }
}

int main() {
  const int E = 15360, N = 7680, H = 400, Hp = 400;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float* a = dev_rand((size_t)N * Hp, 1);
  float* h = dev_rand((size_t)E * Hp, 2);
  float* dpre = dev_rand((size_t)E * Hp, 3);
  std::vector<int> src(E), rev(E);
  srand(9);
  for (int i = 0; i < E; ++i) {
    src[i] = (i / 60) * 30 + rand() % 30;
    rev[i] = (i / 60) * 60 + rand() % 60;
  }
  int *dsrc, *drev;
  CK(hipMalloc(&dsrc, E * 4));
  CK(hipMalloc(&drev, E * 4));
  CK(hipMemcpy(dsrc, src.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drev, rev.data(), E * 4, hipMemcpyHostToDevice));
  float *slab, *bslab;
  CK(hipMalloc(&slab, (size_t)256 * H * Hp * 4));
  CK(hipMalloc(&bslab, (size_t)256 * H * 4));

  // reference: LDS-staged TN (the library's layer weight-gradient configuration)
  LdPlain<4> al{dpre, Hp};
  LdGatherDiff<false> bl{a, h, dsrc, drev, Hp};
  const TnPlan p0 = plan_tn<5, 1, 5, 1>(H, H, E, 1024);
  auto run0 = [&] {
    (void)launch_gemm_tn<5, 1, 5, 1>(al, bl, p0, slab, bslab, H, H, E, true, st);
  };
  run0();
  CK(hipStreamSynchronize(st));
  std::vector<double> W0, b0;
  reduce_host(slab, bslab, p0.splits, H, H, W0, b0);
  const float t0 = time_us(run0, st);
  const double fl = 2.0 * E * H * H;
  printf("tn  (LDS, splits %3d)        %7.2f us  %6.1f TF/s\n", p0.splits, t0, fl / t0 * 1e-6);

  TnrRows sa{dpre, Hp};
  TnrDiff sb{a, h, dsrc, drev, Hp};
  for (int target : {256, 512, 768, 1024, 1536, 2048}) {
    const TnrPlan p = plan_tnr<5, 5>(H, H, E, target);
    auto run = [&] { CK((launch_gemm_tnr<5, 5>(sa, sb, p, slab, bslab, H, H, E, true, st))); };
    CK(hipMemset(slab, 0, (size_t)p.splits * H * Hp * 4));
    run();
    CK(hipStreamSynchronize(st));
    std::vector<double> W, b;
    reduce_host(slab, bslab, p.splits, H, H, W, b);
    double md = 0, mx = 0, mdb = 0, mxb = 0;
    for (size_t i = 0; i < W.size(); ++i) {
      md = std::max(md, std::fabs(W[i] - W0[i]));
      mx = std::max(mx, std::fabs(W0[i]));
    }
    for (int n = 0; n < H; ++n) {
      mdb = std::max(mdb, std::fabs(b[n] - b0[n]));
      mxb = std::max(mxb, std::fabs(b0[n]));
    }
    const float t = time_us(run, st);
    printf("tnr (target %4d, splits %3d) %7.2f us  %6.1f TF/s  W max|diff| %.2e (max %.2e)  b %.2e (%.2e)\n",
           target, p.splits, t, fl / t * 1e-6, md, mx, mdb, mxb);
  }
  return 0;
}
