// Micro-benchmark of the D-MPNN GEMM variants at cfg2 shapes (E 15360, N 7680, H 400).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/gemm_bench.hip -o gemm_bench
// Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); every variant's output
// is compared with the v1 kernel's.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/epilogues.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_dma.hpp"

using namespace cgr;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static float* dev_rand(size_t n, unsigned seed, float scale = 1.f) {
  std::vector<float> h(n);
  srand(seed);
  for (size_t i = 0; i < n; ++i) h[i] = scale * ((rand() / (float)RAND_MAX) * 2.f - 1.f);
  float* d;
  CK(hipMalloc(&d, n * 4));
  CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

struct Variant {
  std::string name;
  double flops;
  std::function<void(hipStream_t)> run;
  float* out;
  size_t out_elems;
  const float* ref;
};

int main(int argc, char** argv) {
  const int E = 15360, N = 7680, H = 400, Hp = 400, F = 846;
  const int rounds = argc > 1 ? atoi(argv[1]) : 5, reps = 20;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float* a = dev_rand((size_t)N * Hp, 1);
  float* h = dev_rand((size_t)E * Hp, 2);
  float* h0 = dev_rand((size_t)E * Hp, 3);
  float* W = dev_rand((size_t)H * H, 4, 0.05f);
  float* bias = dev_rand(H, 5);
  float* x = dev_rand((size_t)N * F, 6);
  float* Wn = dev_rand((size_t)H * (F + H), 7, 0.03f);
  std::vector<int> src(E), rev(E);
  srand(9);
  for (int i = 0; i < E; ++i) {
    const int g = i / 60;  // 60 edges per reaction, 30 atoms
    src[i] = g * 30 + rand() % 30;
    rev[i] = g * 60 + (rand() % 60);
  }
  int *dsrc, *drev;
  CK(hipMalloc(&dsrc, E * 4));
  CK(hipMalloc(&drev, E * 4));
  CK(hipMemcpy(dsrc, src.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drev, rev.data(), E * 4, hipMemcpyHostToDevice));
  auto out_buf = [&](size_t n) {
    float* p;
    CK(hipMalloc(&p, n * 4));
    CK(hipMemset(p, 0, n * 4));
    return p;
  };

  std::vector<Variant> vs;
  const double fl_layer = 2.0 * E * H * H;
  LdGatherDiff<false> gd{a, h, dsrc, drev, Hp};
  LdPlain<4> wl{W, H};
  float* ref_nt = nullptr;
#define NTV(W_, RM_, RN_, KT_, PF_)                                                                  \
  {                                                                                               \
    float* o = out_buf((size_t)E * Hp);                                                           \
    EpLayer ep{bias, nullptr, h0, o, nullptr, Hp, E, H, ACT_RELU, 0u, 1.f, 0, 0};                 \
    vs.push_back({"nt<" #W_ "," #RM_ "," #RN_ "," #KT_ "> pf" #PF_, fl_layer,                   \
                  [=](hipStream_t s) {                                                            \
                    (void)launch_gemm_nt<W_, RM_, RN_, KT_, decltype(gd), decltype(wl), EpLayer, PF_>(gd, wl, ep, E, H, H, s);           \
                  },                                                                              \
                  o, (size_t)E * Hp, ref_nt});                                                    \
    if (!ref_nt) ref_nt = o;                                                                      \
  }
  NTV(4, 1, 5, 1, 1)
  NTV(4, 1, 5, 1, 2)
  NTV(8, 1, 13, 1, 1)
  {
    float* o = out_buf((size_t)E * Hp);
    EpLayer ep{bias, nullptr, h0, o, nullptr, Hp, E, H, ACT_RELU, 0u, 1.f, 0, 0};
    DmaA da{a, h, dsrc, drev, Hp};
    vs.push_back({"dma<5,5,1,gather>", fl_layer,
                  [=](hipStream_t s) {
                    (void)launch_gemm_nt_dma<5, 5, 1, true>(da, W, H, ep, E, H, H, s);
                  },
                  o, (size_t)E * Hp, ref_nt});
  }
  // plain-A NT (dm = dpre W): register-staged vs DMA
  float* dpre0 = dev_rand((size_t)E * Hp, 12);
  float* ref_pl = nullptr;
  {
    float* o = out_buf((size_t)E * Hp);
    EpStore ep{o, Hp, E, H, nullptr};
    LdPlain<4> ap{dpre0, Hp};
    vs.push_back({"plain nt<4,1,5,1> pf1", fl_layer,
                  [=](hipStream_t s) {
                    (void)launch_gemm_nt<4, 1, 5, 1, LdPlain<4>, LdPlain<4>, EpStore, 1>(ap, wl, ep, E, H, H, s);
                  },
                  o, (size_t)E * Hp, nullptr});
    ref_pl = o;
  }
  {
    float* o = out_buf((size_t)E * Hp);
    EpStore ep{o, Hp, E, H, nullptr};
    DmaA da{dpre0, nullptr, nullptr, nullptr, Hp};
    vs.push_back({"plain dma<5,5,1>", fl_layer,
                  [=](hipStream_t s) {
                    (void)launch_gemm_nt_dma<5, 5, 1, false>(da, W, H, ep, E, H, H, s);
                  },
                  o, (size_t)E * Hp, ref_pl});
  }
  int ncu = 256;
  {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    ncu = prop.multiProcessorCount;
  }
#define WSV(RN_, P_, GRP_SCALE)                                                                  \
  {                                                                                               \
    float* o = out_buf((size_t)E * Hp);                                                           \
    EpLayer ep{bias, nullptr, h0, o, nullptr, Hp, E, H, ACT_RELU, 0u, 1.f, 0, 0};                 \
    WsPlan p = plan_ws<RN_, P_>(E, H, H, ncu * GRP_SCALE);                                        \
    vs.push_back({"ws<" #RN_ "," #P_ "> x" #GRP_SCALE, fl_layer,                                 \
                  [=](hipStream_t s) {                                                            \
                    (void)launch_gemm_ws<RN_, P_>(gd, W, H, ep, E, H, H, p, s);                   \
                  },                                                                              \
                  o, (size_t)E * Hp, ref_nt});                                                    \
  }
  // ---- TN layer weight gradient (dpre^T m) ----
  float* dpre = dev_rand((size_t)E * Hp, 11);
  LdPlain<4> ad{dpre, Hp};
  const double fl_tn = 2.0 * E * H * H;
#define TNV(W_, RM_, RN_, KT_, TGT)                                                           \
  {                                                                                           \
    const TnPlan p = plan_tn<W_, RM_, RN_, KT_>(H, H, E, TGT);                                \
    float* slab = out_buf((size_t)p.splits * H * H);                                          \
    float* bslab = out_buf((size_t)p.splits * H);                                             \
    vs.push_back({"tn<" #W_ "," #RM_ "," #RN_ "," #KT_ "> s" + std::to_string(p.splits),     \
                  fl_tn,                                                                      \
                  [=](hipStream_t s) {                                                        \
                    (void)launch_gemm_tn<W_, RM_, RN_, KT_>(ad, gd, p, slab, bslab, H, H, E,  \
                                                            true, s);                         \
                  },                                                                          \
                  slab, 0, nullptr});                                                         \
  }
  TNV(5, 1, 5, 1, 1024)
  // ---- NT readout (x | s) ----
  const double fl_ro = 2.0 * N * (F + H) * H;
  LdConcat<2> cc{x, F, a, Hp, F};
  LdPlain<2> wn{Wn, F + H};
  float* ref_ro = nullptr;
#define ROV(W_, RM_, RN_, KT_, PF_)                                                               \
  {                                                                                           \
    float* o = out_buf((size_t)N * Hp);                                                       \
    EpReadout ep{bias, o, nullptr, Hp, N, H, ACT_RELU};                                       \
    vs.push_back({"ro<" #W_ "," #RM_ "," #RN_ "," #KT_ "> pf" #PF_, fl_ro,                  \
                  [=](hipStream_t s) {                                                        \
                    (void)launch_gemm_nt<W_, RM_, RN_, KT_, decltype(cc), decltype(wn), EpReadout, PF_>(cc, wn, ep, N, H, F + H, s);      \
                  },                                                                          \
                  o, (size_t)N * Hp, ref_ro});                                                \
    if (!ref_ro) ref_ro = o;                                                                  \
  }
  ROV(4, 1, 5, 2, 1)

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs) v.run(st);  // warm + produce outputs
  CK(hipStreamSynchronize(st));
  // correctness vs v1
  for (auto& v : vs) {
    if (!v.ref || !v.out_elems) continue;
    std::vector<float> A(v.out_elems), B(v.out_elems);
    CK(hipMemcpy(A.data(), v.out, v.out_elems * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(B.data(), v.ref, v.out_elems * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (size_t i = 0; i < v.out_elems; ++i) {
      if (i % Hp >= (size_t)H) continue;
      md = std::max(md, (double)fabsf(A[i] - B[i]));
      mx = std::max(mx, (double)fabsf(B[i]));
    }
    printf("check %-28s max|diff| %.3e (max|ref| %.3e)\n", v.name.c_str(), md, mx);
  }
  std::vector<std::vector<float>> t(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, st));
      for (int k = 0; k < reps; ++k) vs[i].run(st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms * 1000.f / reps);
    }
  }
  for (size_t i = 0; i < vs.size(); ++i) {
    auto v = t[i];
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2];
    printf("%-28s median %8.2f us  min %8.2f us  %7.1f TFLOP/s (%.1f%% of 157.3)\n",
           vs[i].name.c_str(), med, v[0], vs[i].flops / med * 1e-6,
           vs[i].flops / med * 1e-6 / 157.3 * 100);
  }
  return 0;
}
