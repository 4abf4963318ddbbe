// Lab for the split-bf16 NT GEMM (csrc/gemm_b3.hpp): correctness against an fp64 host reference
// and timing at the cfg2 shapes, beside the fp32 kernels it replaces.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/b3_lab.hip -o tools/b3_lab
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../cgr-mpnn-3d_amd/csrc/b3_pack.hip"
#include "../cgr-mpnn-3d_amd/csrc/epilogues.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_b3.hpp"
#include "../cgr-mpnn-3d_amd/csrc/gemm_rs.hpp"

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
static float* todev(const std::vector<float>& h) {
  float* d;
  CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  return d;
}
template <class T>
static T* todevT(const std::vector<T>& h) {
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

// B image of B(n, k) = src[n * ldn + k * ldk], N x K
static b3_u4* make_img(const float* dsrc, int64_t ldn, int64_t ldk, int N, int K, hipStream_t st) {
  const size_t u4 = b3_img_u4(N, K);
  b3_u4* img;
  CK(hipMalloc(&img, u4 * 16));
  B3PackJobs j{};
  const B3Cols c = b3_cols(N);
  j.job[0] = B3PackJob{dsrc, ldn, ldk, img, 0, c.nimg, N, K, c.nimg, b3_nk(K)};
  j.n = 1;
  CK(b3_pack(j, st));
  return img;
}

// max over outputs of |c - ref| / sum_k |a||b|  (relative to the magnitude the dot product sums)
static double check(const std::vector<float>& C, int64_t ldc, const std::vector<double>& ref,
                    const std::vector<double>& mag, int M, int N) {
  double worst = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      const double e = fabs((double)C[(size_t)m * ldc + n] - ref[(size_t)m * N + n]) /
                       (mag[(size_t)m * N + n] + 1e-30);
      worst = e > worst ? e : worst;
    }
  return worst;
}

static void test_plain(int M, int N, int K, bool transposed_b, hipStream_t st) {
  const int ld = (K + 3) & ~3;
  auto A = hrand((size_t)M * ld, 11);
  auto B = hrand((size_t)N * K, 12, 0.05f);  // row-major [N][K] (or [K][N] when transposed)
  float *dA = todev(A), *dB = todev(B), *dC;
  CK(hipMalloc(&dC, (size_t)M * ld * 4 + (size_t)M * N * 4));
  const int ldc = N;
  // B(n, k): row-major B[n * K + k] or transposed Bt[k * N + n]
  b3_u4* img = transposed_b ? make_img(dB, 1, N, N, K, st) : make_img(dB, K, 1, N, K, st);
  LdPlain<4> al{dA, ld};
  EpStore ep{dC, ldc, M, N, nullptr};
  CK(launch_b3nt(al, img, ep, M, N, K, st));
  CK(hipStreamSynchronize(st));
  auto C = tohost(dC, (size_t)M * ldc);
  std::vector<double> ref((size_t)M * N), mag((size_t)M * N);
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double s = 0, g = 0;
      for (int k = 0; k < K; ++k) {
        const double b = transposed_b ? B[(size_t)k * N + n] : B[(size_t)n * K + k];
        s += (double)A[(size_t)m * ld + k] * b;
        g += fabs((double)A[(size_t)m * ld + k] * b);
      }
      ref[(size_t)m * N + n] = s;
      mag[(size_t)m * N + n] = g;
    }
  const double e = check(C, ldc, ref, mag, M, N);
  printf("plain M=%d N=%d K=%d %s: max err / sum|ab| = %.3e %s\n", M, N, K,
         transposed_b ? "Bt" : "B", e, e < 4e-7 ? "OK" : "FAIL");
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(dC));
  CK(hipFree(img));
}

#ifdef CGR_B3_STAMPS
static unsigned long long* g_stamps = nullptr;
static void stamps_init() {
  CK(hipMalloc(&g_stamps, 4096 * 16 * 4 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(b3_stamps), &g_stamps, sizeof(g_stamps)));
}
// per-block phase durations (us) of the last launch: percentiles over blocks (wave 0 of each)
static void stamps_report(const char* what, int nblocks, int waves) {
  std::vector<unsigned long long> h((size_t)nblocks * waves * 8);
  CK(hipMemcpy(h.data(), g_stamps, h.size() * 8, hipMemcpyDeviceToHost));
  unsigned long long t0min = ~0ull;
  for (int b = 0; b < nblocks; ++b) t0min = std::min(t0min, h[(size_t)b * waves * 8]);
  std::vector<double> st, pro, loop, epi, end, clk;
  for (int b = 0; b < nblocks; ++b) {
    const unsigned long long* t = &h[(size_t)b * waves * 8];
    clk.push_back((double)(t[6] - t[5]) / ((t[2] - t[1]) * 0.01) * 1e-3);  // GHz over the loop
    st.push_back((t[0] - t0min) * 0.01);
    pro.push_back((t[1] - t[0]) * 0.01);
    loop.push_back((t[2] - t[1]) * 0.01);
    epi.push_back((t[3] - t[2]) * 0.01);
    end.push_back((t[3] - t0min) * 0.01);
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("   %-8s min %6.2f p50 %6.2f p90 %6.2f max %6.2f\n", n, v[0], v[v.size() / 2],
           v[v.size() * 9 / 10], v.back());
  };
  printf("stamps %s (%d blocks):\n", what, nblocks);
  pr("start", st);
  pr("prologue", pro);
  pr("loop", loop);
  pr("epilogue", epi);
  pr("end", end);
  pr("loopGHz", clk);
}
#endif

int main(int argc, char** argv) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
#ifdef CGR_B3_STAMPS
  stamps_init();
#endif
  // ---- correctness ----
  test_plain(200, 400, 400, false, st);
  test_plain(333, 37, 45, false, st);
  test_plain(129, 800, 846, false, st);
  test_plain(77, 400, 400, true, st);
  test_plain(64, 512, 512, false, st);
  test_plain(50, 32, 32, true, st);
  test_plain(1000, 128, 128, false, st);

  // gathered layer GEMM with the layer epilogue vs host (ReLU, skip, no dropout)
  {
    const int E = 3000, Nn = 1500, H = 400, Hp = 400;
    auto a = hrand((size_t)Nn * Hp, 21), h = hrand((size_t)E * Hp, 22), h0 = hrand((size_t)E * Hp, 23);
    auto W = hrand((size_t)H * H, 24, 0.05f), bias = hrand(H, 25);
    std::vector<int> src(E), rev(E);
    srand(26);
    for (int i = 0; i < E; ++i) {
      src[i] = rand() % Nn;
      rev[i] = rand() % E;
    }
    float *da = todev(a), *dh = todev(h), *dh0 = todev(h0), *dW = todev(W), *db = todev(bias), *dout;
    int *dsrc = todevT(src), *drev = todevT(rev);
    CK(hipMalloc(&dout, (size_t)E * Hp * 4));
    b3_u4* img = make_img(dW, H, 1, H, H, st);
    LdGatherDiff<false> al{da, dh, dsrc, drev, Hp};
    EpLayer ep{db, nullptr, dh0, dout, nullptr, Hp, E, H, 0, 0u, 1.f, nullptr, 0};
    CK(launch_b3nt(al, img, ep, E, H, H, st));
    CK(hipStreamSynchronize(st));
    auto out = tohost(dout, (size_t)E * Hp);
    double worst = 0;
    for (int e = 0; e < E; ++e)
      for (int n = 0; n < H; ++n) {
        double s = 0, g = 0;
        for (int k = 0; k < H; ++k) {
          const double m = (double)a[(size_t)src[e] * Hp + k] - (double)h[(size_t)rev[e] * Hp + k];
          s += m * W[(size_t)n * H + k];
          g += fabs(m * W[(size_t)n * H + k]);
        }
        const double z = s + bias[n] + h0[(size_t)e * Hp + n];
        const double r = z > 0 ? z : 0;
        const double err = fabs(out[(size_t)e * Hp + n] - r) / (g + fabs(bias[n]) + fabs(h0[(size_t)e * Hp + n]));
        worst = err > worst ? err : worst;
      }
    printf("layer gather+EpLayer E=%d: max err = %.3e %s\n", E, worst, worst < 4e-7 ? "OK" : "FAIL");
  }

  // ---- timing at cfg2 shapes ----
  {
    const int E = 15360, Nn = 7680, H = 400, Hp = 400, F = 848;
    auto a = hrand((size_t)Nn * Hp, 31), h = hrand((size_t)E * Hp, 32), h0 = hrand((size_t)E * Hp, 33);
    auto W = hrand((size_t)H * H, 34, 0.05f), bias = hrand(H, 35);
    auto x = hrand((size_t)Nn * F, 36), Wx = hrand((size_t)2 * H * F, 37, 0.05f);
    std::vector<int> src(E), rev(E);
    srand(9);
    for (int i = 0; i < E; ++i) {
      const int g = i / 60;
      src[i] = g * 30 + rand() % 30;
      rev[i] = g * 60 + (rand() % 60);
    }
    float *da = todev(a), *dh = todev(h), *dh0 = todev(h0), *dW = todev(W), *db = todev(bias);
    float *dx = todev(x), *dWx = todev(Wx), *dout, *dout2;
    int *dsrc = todevT(src), *drev = todevT(rev);
    CK(hipMalloc(&dout, (size_t)E * Hp * 4));
    CK(hipMalloc(&dout2, (size_t)Nn * 2 * Hp * 4));
    b3_u4* img = make_img(dW, H, 1, H, H, st);
    b3_u4* imgx = make_img(dWx, F, 1, 2 * H, F, st);
    LdGatherDiff<false> al{da, dh, dsrc, drev, Hp};
    EpLayer ep{db, nullptr, dh0, dout, nullptr, Hp, E, H, 0, 0u, 1.f, nullptr, 0};
    const double fl_layer = 2.0 * E * H * H, fl_x = 2.0 * Nn * 2 * H * F, fl_ro = 2.0 * Nn * H * H;
    float t = time_us([&] { CK(launch_b3nt(al, img, ep, E, H, H, st)); }, st);
    printf("b3  layer fwd (gather, EpLayer) E=%d: %.1f us  %.1f TFLOP/s (fp32-equivalent)\n", E, t,
           fl_layer / t * 1e-6);
#ifdef CGR_B3_STAMPS
    CK(launch_b3nt(al, img, ep, E, H, H, st));
    CK(hipStreamSynchronize(st));
    stamps_report("layer fwd", 240, 8);
#endif
    LdPlain<4> alp{dh, Hp};
    EpStore eps{dout, Hp, E, H, nullptr};
    t = time_us([&] { CK(launch_b3nt(alp, img, eps, E, H, H, st)); }, st);
    printf("b3  layer bwd (plain, EpStore) E=%d: %.1f us  %.1f TFLOP/s\n", E, t, fl_layer / t * 1e-6);
#ifdef CGR_B3_STAMPS
    CK(launch_b3nt(alp, img, eps, E, H, H, st));
    CK(hipStreamSynchronize(st));
    stamps_report("layer bwd", 240, 8);
#endif
    LdPlain<4> alx{dx, F};
    EpStore epx{dout2, 2 * Hp, Nn, 2 * H, nullptr};
    t = time_us([&] { CK(launch_b3nt(alx, imgx, epx, Nn, 2 * H, F, st)); }, st);
    printf("b3  x-GEMM N=%d K=%d: %.1f us  %.1f TFLOP/s\n", 2 * H, F, t, fl_x / t * 1e-6);
    LdPlain<4> alr{da, Hp};
    EpStore epr{dout2, Hp, Nn, H, nullptr};
    t = time_us([&] { CK(launch_b3nt(alr, img, epr, Nn, H, H, st)); }, st);
    printf("b3  readout (plain, M=%d): %.1f us  %.1f TFLOP/s\n", Nn, t, fl_ro / t * 1e-6);
    // fp32 references
    t = time_us([&] { CK((launch_gemm_rs<2, 4>(al, dW, H, ep, E, H, H, st))); }, st);
    printf("f32 layer fwd (rs): %.1f us  %.1f TFLOP/s\n", t, fl_layer / t * 1e-6);
    LdPlain<4> blw{dW, H};
    t = time_us([&] { CK((launch_gemm_nt<4, 1, 5, 1>(alp, blw, eps, E, H, H, st))); }, st);
    printf("f32 layer bwd (tiled): %.1f us  %.1f TFLOP/s\n", t, fl_layer / t * 1e-6);
    t = time_us([&] { CK(b3_pack([&] { B3PackJobs j{}; const B3Cols c = b3_cols(H);
                                         j.job[0] = B3PackJob{dW, H, 1, img, 0, c.nimg, H, H, c.nimg, b3_nk(H)};
                                         j.job[1] = B3PackJob{dW, 1, H, img, 0, c.nimg, H, H, c.nimg, b3_nk(H)};
                                         j.n = 2; return j; }(), st)); }, st);
    printf("pack 2 x (400x400): %.1f us\n", t);
  }
  return 0;
}
