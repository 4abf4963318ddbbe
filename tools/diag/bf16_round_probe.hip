// Which rounding does the split's fp32 -> bf16 conversion use on the device, and how does the
// bf16 MFMA round its fp32 accumulation?  (diagnostic for the learnable-skip precision gap)
//   1. v_cvt_pk_bf16_f32 via __builtin_convertvector (gemm_b3.hpp b3_cvt2) on values exactly
//      halfway / just above / just below a bf16 step, vs round-to-nearest-even;
//   2. one v_mfma_f32_16x16x32_bf16 whose exact result is not an fp32 number: acc = 1 + t with
//      t = 2^-25 * 3 (above half an ulp) or 2^-25 (a tie) or -(3 * 2^-25): RNE, truncation or
//      other.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void k_cvt(const float* in, uint32_t* out, int n) {
  int i = threadIdx.x;
  if (i < n) {
    const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(floatx2{in[i], 0.f}, bf16x2));
    out[i] = u & 0xffffu;
  }
}

// every lane: a = (1, 0, ...), b = (1, 0, ...) for k = 0 only in row/col 0; acc preset to c0
__global__ void k_mfma(const float* c0, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)0.f;
    b[j] = (__bf16)0.f;
  }
  // lane groups: lane & 15 = row (a) / column (b), lane >> 4 = k group; k element 0 of group 0
  if (lane == 0) {
    a[0] = (__bf16)1.f;
    b[0] = (__bf16)1.f;
  }
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c0[0];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[lane * 4 + r] = acc[r];
}

// acc (fp32) + a product that is not representable together with it: a = 2^-12 * (1 + 2^-7),
// b = 2^-12 (bf16 exact), acc = 1: exact sum 1 + 2^-24 + 2^-31 (just above half an ulp of 1)
__global__ void k_mfma2(const float* av, const float* bv, const float* c0, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)0.f;
    b[j] = (__bf16)0.f;
  }
  if (lane == 0) {
    a[0] = (__bf16)av[0];
    b[0] = (__bf16)bv[0];
  }
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c0[0];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  out[lane] = acc[0];
}

// row 0 x column 0 over all 32 k: a[k], b[k] (bf16-exact values), acc preset to c0.  Lane l holds
// row / column l & 15, k = b3_kperm-free natural order: elements j of lane group g = k 8 g + j
__global__ void k_mfma32(const float* av, const float* bv, const float* c0, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (lane >> 4) + j;
    a[j] = (__bf16)((lane & 15) == 0 ? av[k] : 0.f);
    b[j] = (__bf16)((lane & 15) == 0 ? bv[k] : 0.f);
  }
  floatx4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = c0[0];
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  out[lane] = acc[0];
}

static uint16_t rne_bf16(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  const uint32_t lsb = (u >> 16) & 1u;
  return (uint16_t)((u + 0x7fffu + lsb) >> 16);
}

int main() {
  // 1. conversions: 1 + k * 2^-23 for k around the bf16 step (2^-7 at 1: 65536 fp32 ulps)
  const int n = 8;
  float h[n];
  const float base = 1.0f;
  const int offs[n] = {0x7fff, 0x8000, 0x8001, 0x18000, 0xffff, 0x10000 + 0x7fff, -0x8000, -0x8001};
  for (int i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, &base, 4);
    u = (uint32_t)((int)u + offs[i]);
    memcpy(&h[i], &u, 4);
  }
  float* din;
  uint32_t* dout;
  hipMalloc(&din, sizeof(h));
  hipMalloc(&dout, 4 * n);
  hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
  k_cvt<<<1, 64>>>(din, dout, n);
  uint32_t o[n];
  hipMemcpy(o, dout, 4 * n, hipMemcpyDeviceToHost);
  int rne_ok = 0, trunc_like = 0;
  for (int i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, &h[i], 4);
    const uint16_t r = rne_bf16(h[i]);
    const uint16_t t = (uint16_t)(u >> 16);
    printf("cvt %08x -> %04x  (RNE %04x, trunc %04x)\n", u, o[i], r, t);
    rne_ok += o[i] == r;
    trunc_like += o[i] == t;
  }
  printf("conversion: %d/%d round-to-nearest-even, %d/%d equal to truncation\n", rne_ok, n,
         trunc_like, n);
  // 2. MFMA accumulation rounding: acc = c0, + 1 * p (p = a b exact in bf16 products)
  float* dc;
  float* da;
  float* db;
  float* dres;
  hipMalloc(&dc, 4);
  hipMalloc(&da, 4);
  hipMalloc(&db, 4);
  hipMalloc(&dres, 4 * 256);
  struct Case {
    float c0, a, b;
    const char* what;
  } cases[] = {
      {1.0f, 0x1.02p-12f, 0x1p-12f, "1 + (2^-24 + 2^-31): above half an ulp -> RNE 1+2^-23"},
      {1.0f, 0x1p-12f, 0x1p-12f, "1 + 2^-24: a tie -> RNE 1 (even)"},
      {1.0f, 0x1.8p-12f, 0x1p-12f, "1 + 1.5*2^-24: above half -> RNE 1+2^-23, RZ 1"},
      {-1.0f, 0x1.8p-12f, -0x1p-12f, "-1 - 1.5*2^-24: RNE -(1+2^-23), RZ -1"},
      {0x1.000002p0f, 0x1.8p-12f, 0x1p-12f, "(1+2^-23) + 1.5*2^-24: RNE 1+2^-22, RZ 1+2^-23"},
      {1.0f, -0x1.8p-12f, 0x1p-12f, "1 - 1.5*2^-24: RNE 1-2^-24 (exact: 1-2^-24 representable)"},
  };
  for (const Case& c : cases) {
    hipMemcpy(dc, &c.c0, 4, hipMemcpyHostToDevice);
    hipMemcpy(da, &c.a, 4, hipMemcpyHostToDevice);
    hipMemcpy(db, &c.b, 4, hipMemcpyHostToDevice);
    k_mfma2<<<1, 64>>>(da, db, dc, dres);
    float r;
    hipMemcpy(&r, dres, 4, hipMemcpyDeviceToHost);
    const double exact = (double)c.c0 + (double)c.a * (double)c.b;
    printf("mfma acc %a + %a*%a = %a (exact %a)  [%s]\n", c.c0, c.a, c.b, r, exact, c.what);
  }
  // 3. several products in one MFMA (the alignment of a multi-term sum)
  float* da32;
  float* db32;
  hipMalloc(&da32, 4 * 32);
  hipMalloc(&db32, 4 * 32);
  struct Case32 {
    float c0;
    int n;
    float a[4], b[4];
    const char* what;
  } c32[] = {
      {0.f, 2, {1.f, 0x1.8p-12f}, {1.f, 0x1p-12f}, "0 + 1 + 1.5*2^-24: RNE 1+2^-23, RZ 1"},
      {1.f, 2, {0x1.8p-13f, 0x1.8p-13f}, {0x1p-12f, 0x1p-12f}, "1 + 2 * 0.75*2^-24: RNE 1+2^-23, RZ 1"},
      {1.f, 2, {0x1.8p-12f, -0x1p-20f}, {0x1p-12f, 0x1p-20f}, "1 + 1.5*2^-24 - 2^-40: RNE 1+2^-23"},
      {1.f, 3, {0x1.8p-12f, 1.f, -1.f}, {0x1p-12f, 0x1p-30f, 0x1p-31f}, "1 + 1.5*2^-24 + 2^-30 - 2^-31"},
      {0.f, 3, {1.f, 0x1.8p-12f, 0x1p-2f}, {1.f, 0x1p-12f, 0x1p-40f}, "1 + 1.5*2^-24 + 2^-42"},
      {-1.f, 2, {-0x1.8p-13f, -0x1.8p-13f}, {0x1p-12f, 0x1p-12f}, "-1 - 1.5*2^-24 (two terms): RNE -(1+2^-23)"},
      {0x1p-10f, 2, {1.f, -1.f}, {1.f, 0x1.fffep-1f}, "2^-10 + 1 - (1-2^-16): cancellation"},
  };
  for (const Case32& c : c32) {
    float ha[32] = {0}, hb[32] = {0};
    double exact = c.c0;
    for (int i = 0; i < c.n; ++i) {
      ha[i * 9 % 32] = c.a[i];  // spread over lane groups / elements
      hb[i * 9 % 32] = c.b[i];
      exact += (double)c.a[i] * (double)c.b[i];
    }
    hipMemcpy(dc, &c.c0, 4, hipMemcpyHostToDevice);
    hipMemcpy(da32, ha, sizeof(ha), hipMemcpyHostToDevice);
    hipMemcpy(db32, hb, sizeof(hb), hipMemcpyHostToDevice);
    k_mfma32<<<1, 64>>>(da32, db32, dc, dres);
    float r;
    hipMemcpy(&r, dres, 4, hipMemcpyDeviceToHost);
    printf("mfma32 %-48s = %a (exact %a, RNE of exact %a)\n", c.what, r, exact, (float)exact);
  }
  return 0;
}
