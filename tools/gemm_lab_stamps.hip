// GEMM lab: time the layer NT GEMM (gathered a[src]-h[rev] rows, EpLayer) and the plain NT GEMM
// (EpStore) over a sweep of row counts M at H = 400, to see how the time depends on the number
// of 64x80 tiles against the 4-per-CU residency (1024 slots on 256 CUs).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gemm_lab.hip -o tools/gemm_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/epilogues.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_rs.hpp"
#ifndef RS_RM_LAB
#define RS_RM_LAB 2
#endif

using namespace cgr;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
      exit(1);                                                                           \
    }                                                                                    \
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

int main_unused() {
  const int Emax = 20480, H = 400, Hp = 400;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float* a = dev_rand((size_t)Emax / 2 * Hp, 1);
  float* h = dev_rand((size_t)Emax * Hp, 2);
  float* h0 = dev_rand((size_t)Emax * Hp, 3);
  float* W = dev_rand((size_t)H * H, 4, 0.05f);
  float* bias = dev_rand(H, 5);
  float* out;
  CK(hipMalloc(&out, (size_t)Emax * Hp * 4));
  std::vector<int> src(Emax), rev(Emax);
  srand(9);
  for (int i = 0; i < Emax; ++i) {
    const int g = i / 60;
    src[i] = g * 30 + rand() % 30;
    rev[i] = g * 60 + (rand() % 60);
  }
  int *dsrc, *drev;
  CK(hipMalloc(&dsrc, Emax * 4));
  CK(hipMalloc(&drev, Emax * 4));
  CK(hipMemcpy(dsrc, src.data(), Emax * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drev, rev.data(), Emax * 4, hipMemcpyHostToDevice));
  LdGatherDiff<false> gd{a, h, dsrc, drev, Hp};
  LdPlain<4> wl{W, H};
  LdPlain<4> ap{h, Hp};
  const int Ms[] = {4096, 8192, 10240, 12288, 13056, 13120, 14336, 15360, 16384, 19456, 20480};
  printf("%6s %6s | %10s %8s | %10s %8s\n", "M", "tiles", "gather us", "TF/s", "plain us", "TF/s");
  for (int M : Ms) {
    const double fl = 2.0 * M * H * H;
    EpLayer ep{bias, nullptr, h0, out, nullptr, Hp, M, H, ACT_RELU, 0u, 1.f, nullptr, 0};
    EpStore es{out, Hp, M, H, nullptr};
    const float tg = time_us(
        [&] {
          (void)launch_gemm_nt<4, 1, 5, 1, LdGatherDiff<false>, LdPlain<4>, EpLayer, 2>(gd, wl, ep, M,
                                                                                      H, H, st);
        },
        st);
    const float tp = time_us(
        [&] {
          (void)launch_gemm_nt<4, 1, 5, 1, LdPlain<4>, LdPlain<4>, EpStore, 2>(ap, wl, es, M, H, H,
                                                                             st);
        },
        st);
    const int tiles = (M + 63) / 64 * 5;
    printf("%6d %6d | %10.2f %8.1f | %10.2f %8.1f\n", M, tiles, tg, fl / tg * 1e-6, tp,
           fl / tp * 1e-6);
  }
  // occupancy / prefetch variants of the layer NT at cfg2 (M = 15360: 1200 tiles)
  {
    const int M = 15360;
    const double fl = 2.0 * M * H * H;
    EpLayer ep{bias, nullptr, h0, out, nullptr, Hp, M, H, ACT_RELU, 0u, 1.f, nullptr, 0};
    EpStore es{out, Hp, M, H, nullptr};
#define VAR(PF_, OCC_)                                                                            \
    {                                                                                             \
      const float tg = time_us([&] { (void)launch_gemm_nt<4, 1, 5, 1, LdGatherDiff<false>, LdPlain<4>, EpLayer, PF_, OCC_>(gd, wl, ep, M, H, H, st); }, st); \
      const float tp = time_us([&] { (void)launch_gemm_nt<4, 1, 5, 1, LdPlain<4>, LdPlain<4>, EpStore, PF_, OCC_>(ap, wl, es, M, H, H, st); }, st); \
      printf("pf%d occ%d  gather %7.2f us %6.1f TF/s | plain %7.2f us %6.1f TF/s\n", PF_, OCC_, tg, fl / tg * 1e-6, tp, fl / tp * 1e-6); \
    }
    VAR(2, 0)
    VAR(1, 0)
  }
  // row-block-stationary kernel vs the tiled kernel: outputs and time
  {
    float* ref;
    CK(hipMalloc(&ref, (size_t)Emax * Hp * 4));
    for (int M : {15360, 13056, 7680, 20480}) {
      const double fl = 2.0 * M * H * H;
      for (int gather = 0; gather < 2; ++gather) {
        EpLayer epr{bias, nullptr, h0, ref, nullptr, Hp, M, H, ACT_RELU, 0u, 1.f, nullptr, 0};
        EpLayer ep{bias, nullptr, h0, out, nullptr, Hp, M, H, ACT_RELU, 0u, 1.f, nullptr, 0};
        CK(hipMemset(out, 0, (size_t)M * Hp * 4));
        auto run_ref = [&] {
          if (gather)
            (void)launch_gemm_nt<4, 1, 5, 1, LdGatherDiff<false>, LdPlain<4>, EpLayer, 2>(gd, wl, epr, M, H, H, st);
          else
            (void)launch_gemm_nt<4, 1, 5, 1, LdPlain<4>, LdPlain<4>, EpLayer, 2>(ap, wl, epr, M, H, H, st);
        };
        auto run_rs1 = [&] {
          if (gather) CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(gd, W, H, ep, M, H, H, st)));
          else CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(ap, W, H, ep, M, H, H, st)));
        };
        auto run_rs2 = [&] {
          if (gather) CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(gd, W, H, ep, M, H, H, st)));
          else CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(ap, W, H, ep, M, H, H, st)));
        };
        run_ref();
        run_rs2();
        CK(hipStreamSynchronize(st));
        std::vector<float> A((size_t)M * Hp), Bv((size_t)M * Hp);
        CK(hipMemcpy(A.data(), out, A.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(Bv.data(), ref, Bv.size() * 4, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < A.size(); ++i) {
          md = std::max(md, (double)fabsf(A[i] - Bv[i]));
          mx = std::max(mx, (double)fabsf(Bv[i]));
        }
        const float t0 = time_us(run_ref, st), t1 = time_us(run_rs1, st), t2 = time_us(run_rs2, st);
        printf("M %5d %s  tiled %6.2f us (%5.1f TF)  rs pf1 %6.2f us (%5.1f TF)  rs pf2 %6.2f us (%5.1f TF)  max|diff| %.2e (max %.2e)\n",
               M, gather ? "gather" : "plain ", t0, fl / t0 * 1e-6, t1, fl / t1 * 1e-6, t2,
               fl / t2 * 1e-6, md, mx);
      }
    }
  }
  return 0;
}

#ifdef CGR_RS_STAMPS
int main() {
  const int E = 15360, H = 400, Hp = 400;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float* a = dev_rand((size_t)E / 2 * Hp, 1);
  float* h = dev_rand((size_t)E * Hp, 2);
  float* h0 = dev_rand((size_t)E * Hp, 3);
  float* W = dev_rand((size_t)H * H, 4, 0.05f);
  float* bias = dev_rand(H, 5);
  float* out;
  CK(hipMalloc(&out, (size_t)E * Hp * 4));
  std::vector<int> src(E), rev(E);
  srand(9);
  for (int i = 0; i < E; ++i) { src[i] = (i / 60) * 30 + rand() % 30; rev[i] = (i / 60) * 60 + rand() % 60; }
  int *dsrc, *drev;
  CK(hipMalloc(&dsrc, E * 4));
  CK(hipMalloc(&drev, E * 4));
  CK(hipMemcpy(dsrc, src.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(drev, rev.data(), E * 4, hipMemcpyHostToDevice));
  LdGatherDiff<false> gd{a, h, dsrc, drev, Hp};
  LdPlain<4> ap{h, Hp};
  const int nb = E / 64;
  unsigned long long* st_d;
  CK(hipMalloc(&st_d, (size_t)nb * 16 * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rs_stamps), &st_d, sizeof(st_d)));
  for (int M : {15360, 7680}) for (int gather = 0; gather < 2; ++gather) {
    EpLayer ep{bias, nullptr, h0, out, nullptr, Hp, M, H, ACT_RELU, 0u, 1.f, nullptr, 0};
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(st_d, 0, (size_t)nb * 16 * 4 * 8));
      if (gather) CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(gd, W, H, ep, M, H, H, st)));
      else CK((launch_gemm_rs<RS_RM_LAB, (RS_RM_LAB == 2 ? 4 : 7)>(ap, W, H, ep, M, H, H, st)));
      CK(hipStreamSynchronize(st));
    }
    std::vector<unsigned long long> v((size_t)nb * 16 * 4);
    CK(hipMemcpy(v.data(), st_d, v.size() * 8, hipMemcpyDeviceToHost));
    const int nbm = (M + 63) / 64;
    unsigned long long t0 = ~0ull, tend = 0;
    double sp[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    for (int b = 0; b < nbm; ++b) for (int w = 0; w < 16; ++w) {
      const unsigned long long* q = &v[((size_t)b * 16 + w) * 4];
      t0 = std::min(t0, q[0]); tend = std::max(tend, q[3]);
      for (int i = 0; i < 3; ++i) { double d = (double)(q[i + 1] - q[i]) * 0.01; sp[i] += d; mx[i] = std::max(mx[i], d); }
    }
    const double n = nbm * 16.0;
    unsigned long long smin = ~0ull, smax = 0;
    for (int b = 0; b < nbm; ++b) { smin = std::min(smin, v[(size_t)b * 64]); smax = std::max(smax, v[(size_t)b * 64]); }
    printf("M %5d %s  span %.1f us | start skew %.1f us | prologue avg %.1f max %.1f | main avg %.1f max %.1f | epilogue avg %.1f max %.1f (us)\n",
           M, gather ? "gather" : "plain ", (tend - t0) * 0.01, (smax - smin) * 0.01, sp[0] / n, mx[0], sp[1] / n, mx[1], sp[2] / n, mx[2]);
  }
  return 0;
}
#endif
