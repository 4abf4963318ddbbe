// Does splitting the layer GEMM into two half-batches on two streams beat one full launch?
// (reaction graphs are disjoint, so half-batches are independent row ranges of every edge /
// node array).  Times, per launch group, with the GPU otherwise idle between groups:
//   full : one NT layer GEMM over E rows
//   halves: two launches over E/2 rows each, on two streams (fork / join with events)
//   seq  : the two half launches on one stream
//   nt+tn: the NT layer GEMM beside the TN layer weight gradient on a second stream (backward)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/concurrency_probe.hip -o cprobe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/epilogues.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"

using namespace cgr;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
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

int main(int argc, char** argv) {
  const int E = 15360, N = 7680, H = 400, Hp = 400;
  const int reps = argc > 1 ? atoi(argv[1]) : 30;
  hipStream_t s0, s1;
  CK(hipStreamCreate(&s0));
  CK(hipStreamCreate(&s1));
  float* a = dev_rand((size_t)N * Hp, 1);
  float* h = dev_rand((size_t)E * Hp, 2);
  float* h0 = dev_rand((size_t)E * Hp, 3);
  float* W = dev_rand((size_t)H * H, 4, 0.05f);
  float* bias = dev_rand(H, 5);
  float* dpre = dev_rand((size_t)E * Hp, 6);
  float* out;
  CK(hipMalloc(&out, (size_t)E * Hp * 4));
  std::vector<int> src(E), rev(E);
  for (int i = 0; i < E; ++i) {  // dst-sorted edges of 256 reactions x 60 edges, 30 atoms
    const int g = i / 60;
    src[i] = g * 30 + rand() % 30;
    rev[i] = g * 60 + (rand() % 60);
  }
  int *dsrc, *drev;
  CK(hipMalloc(&dsrc, E * 4));
  CK(hipMalloc(&drev, E * 4));
  CK(hipMemcpy(dsrc, src.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drev, rev.data(), E * 4, hipMemcpyHostToDevice));
  LdPlain<4> wl{W, H};
  const TnPlan tp = plan_tn<5, 1, 5, 1>(H, H, E, 1024);
  float *slab, *bslab;
  CK(hipMalloc(&slab, (size_t)tp.splits * H * H * 4));
  CK(hipMalloc(&bslab, (size_t)tp.splits * H * 4));

  // rows [r0, r0 + rows) of the layer GEMM: shift the row-indexed pointers (index arrays hold
  // global ids, so the gather sources stay whole)
  auto nt = [&](int r0, int rows, hipStream_t s) {
    LdGatherDiff<false> gd{a, h, dsrc + r0, drev + r0, Hp};
    EpLayer ep{bias, nullptr, h0 + (size_t)r0 * Hp, out + (size_t)r0 * Hp, nullptr, Hp, rows, H,
               ACT_RELU, 0u, 1.f, nullptr, 0};
    CK((launch_gemm_nt<4, 1, 5, 1, decltype(gd), decltype(wl), EpLayer, 2>(gd, wl, ep, rows, H,
                                                                          H, s)));
  };
  auto tn = [&](hipStream_t s) {
    LdPlain<4> ad{dpre, Hp};
    LdGatherDiff<false> gd{a, h, dsrc, drev, Hp};
    CK((launch_gemm_tn<5, 1, 5, 1>(ad, gd, tp, slab, bslab, H, H, E, true, s)));
  };
  hipEvent_t e0, e1, fork, join;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  struct Case {
    std::string name;
    std::function<void()> run;
  };
  std::vector<Case> cs = {
      {"full (1 x E rows)", [&] { nt(0, E, s0); }},
      {"halves, 2 streams", [&] {
         CK(hipEventRecord(fork, s0));
         CK(hipStreamWaitEvent(s1, fork, 0));
         nt(0, E / 2, s0);
         nt(E / 2, E / 2, s1);
         CK(hipEventRecord(join, s1));
         CK(hipStreamWaitEvent(s0, join, 0));
       }},
      {"halves, 1 stream", [&] {
         nt(0, E / 2, s0);
         nt(E / 2, E / 2, s0);
       }},
      {"tn alone", [&] { tn(s0); }},
      {"nt + tn, 2 streams", [&] {
         CK(hipEventRecord(fork, s0));
         CK(hipStreamWaitEvent(s1, fork, 0));
         nt(0, E, s0);
         tn(s1);
         CK(hipEventRecord(join, s1));
         CK(hipStreamWaitEvent(s0, join, 0));
       }},
      {"nt then tn, 1 stream", [&] {
         nt(0, E, s0);
         tn(s0);
       }},
  };
  for (auto& c : cs) c.run();
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(cs.size());
  for (int r = 0; r < reps; ++r) {
    for (size_t i = 0; i < cs.size(); ++i) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s0));
      cs[i].run();
      CK(hipEventRecord(e1, s0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms * 1000.f);
    }
  }
  for (size_t i = 0; i < cs.size(); ++i) {
    auto v = t[i];
    std::sort(v.begin(), v.end());
    printf("%-24s median %8.2f us  min %8.2f us\n", cs[i].name.c_str(), v[v.size() / 2], v[0]);
  }
  return 0;
}
