// Host cost of one kernel enqueue on this runtime, by API (diagnostic for the eager training
// step): hipLaunchKernelGGL (hipLaunchKernel) vs hipModuleLaunchKernel on the
// hipFunction_t of the same static kernel (hipGetFuncBySymbol), vs hipExtLaunchKernel; an empty
// kernel with a 64-byte argument block (a typical argument size here), 20000 enqueues each, on a
// non-blocking stream, synchronised at the end.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

struct Args64 {
  float* p[8];
};

struct Args1k {
  float* p[128];
};
struct Args3k {
  float* p[384];
};
template <class A>
__global__ void k_emptyT(A a, int n) {
  if (n < 0 && threadIdx.x == 0) a.p[0][0] = 1.f;
}

__global__ void k_empty(Args64 a, int n) {
  if (n < 0 && threadIdx.x == 0) a.p[0][0] = 1.f;  // never taken; keeps the arguments live
}

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Args64 a{};
  const int n = 1;
  const int reps = 20000;
  using clk = std::chrono::steady_clock;
  for (int round = 0; round < 2; ++round) {
    // 1. hipLaunchKernelGGL
    auto t0 = clk::now();
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_empty, dim3(240), dim3(512), 0, st, a, n);
    auto t1 = clk::now();
    CHECK(hipStreamSynchronize(st));
    auto t2 = clk::now();
    printf("round %d hipLaunchKernelGGL      host %.2f us/launch, incl. drain %.2f us\n", round,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / reps);
    // 2. hipModuleLaunchKernel on the static kernel's function handle
    hipFunction_t f;
    CHECK(hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(k_empty)));
    void* params[] = {&a, const_cast<int*>(&n)};
    t0 = clk::now();
    for (int i = 0; i < reps; ++i)
      (void)hipModuleLaunchKernel(f, 240, 1, 1, 512, 1, 1, 0, st, params, nullptr);
    t1 = clk::now();
    CHECK(hipStreamSynchronize(st));
    t2 = clk::now();
    printf("round %d hipModuleLaunchKernel   host %.2f us/launch, incl. drain %.2f us\n", round,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / reps);
    // 3. hipExtLaunchKernel
    void* args2[] = {&a, const_cast<int*>(&n)};
    t0 = clk::now();
    for (int i = 0; i < reps; ++i)
      (void)hipExtLaunchKernel(reinterpret_cast<const void*>(k_empty), dim3(240), dim3(512), args2,
                               0, st, nullptr, nullptr, 0);
    t1 = clk::now();
    CHECK(hipStreamSynchronize(st));
    t2 = clk::now();
    printf("round %d hipExtLaunchKernel      host %.2f us/launch, incl. drain %.2f us\n", round,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / reps,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / reps);
    // 4. argument size: 1 KB, 3 KB blocks through hipLaunchKernelGGL
    {
      Args1k b{};
      t0 = clk::now();
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_emptyT<Args1k>, dim3(240), dim3(512), 0, st, b, n);
      t1 = clk::now();
      CHECK(hipStreamSynchronize(st));
      printf("round %d 1 KB arguments          host %.2f us/launch\n", round,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
      Args3k c{};
      t0 = clk::now();
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_emptyT<Args3k>, dim3(240), dim3(512), 0, st, c, n);
      t1 = clk::now();
      CHECK(hipStreamSynchronize(st));
      printf("round %d 3 KB arguments          host %.2f us/launch\n", round,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
      // alternating two streams (the backward's main / side interleave)
      hipStream_t s3;
      CHECK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
      t0 = clk::now();
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(k_empty, dim3(240), dim3(512), 0, (i & 1) ? s3 : st, a, n);
      t1 = clk::now();
      CHECK(hipDeviceSynchronize());
      printf("round %d alternating two streams host %.2f us/launch\n", round,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
      CHECK(hipStreamDestroy(s3));
    }
    // 5. event record + stream wait (a cross-stream edge)
    hipStream_t s2;
    hipEvent_t ev;
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    t0 = clk::now();
    for (int i = 0; i < reps / 10; ++i) {
      (void)hipEventRecord(ev, st);
      (void)hipStreamWaitEvent(s2, ev, 0);
    }
    t1 = clk::now();
    CHECK(hipStreamSynchronize(s2));
    printf("round %d eventRecord+streamWait host %.2f us/pair\n", round,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / (reps / 10));
    CHECK(hipEventDestroy(ev));
    CHECK(hipStreamDestroy(s2));
  }
  return 0;
}
