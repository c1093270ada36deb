// Dependent-chain latency of the fp64 operations on the backward pass's serial chain (gfx950, one
// wave, shader-clock s_memtime). Build: hipcc -O3 --offload-arch=gfx950 lat_f64.hip -o lat_f64
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 2048;

template <int L>
__device__ __forceinline__ double bcast(double v) {
  return __builtin_amdgcn_update_dpp(__builtin_nondeterministic_value(v), v, 0x150 + L, 0xF, 0xF, true);
}
__device__ __forceinline__ double shr1(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(x & 0xffffffffll), 0x111, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), 0x111, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

__global__ void k_lat(double* out, unsigned long long* cyc, double a, double b) {
  __shared__ double lds[64 * 4];
  double x = a + threadIdx.x * 1e-3;
  unsigned long long t0, t1;
  int t = 0;
#define TEST(BODY)                                                  \
  t0 = __builtin_amdgcn_s_memtime();                                \
  for (int i = 0; i < ITERS; i++) { BODY; }                        \
  __asm__ volatile("" : "+v"(x));                                   \
  t1 = __builtin_amdgcn_s_memtime();                                \
  if (threadIdx.x == 0) cyc[t] = t1 - t0;                           \
  t++;
  TEST(x = fma(x, a, b))                                    // 0 fma chain
  TEST(x = x * a)                                           // 1 mul chain
  TEST(x = x + b)                                           // 2 add chain
  TEST(x = sqrt(x) + b)                                     // 3 IEEE sqrt + add
  TEST(x = 1.0 / x + b)                                     // 4 IEEE reciprocal (div) + add
  TEST(x = __builtin_amdgcn_rsq(x) + b)                     // 5 raw v_rsq_f64 + add
  TEST(x = __builtin_amdgcn_rcp(x) + b)                     // 6 raw v_rcp_f64 + add
  TEST(x = bcast<3>(x) + b)                                 // 7 DPP row_newbcast + add
  TEST(x = shr1(x) + b)                                     // 8 DPP row_shr:1 (2 x b32) + add
  TEST(lds[threadIdx.x] = x; __builtin_amdgcn_wave_barrier(); x = lds[threadIdx.x ^ 1] + b)  // 9 LDS round trip + add
  TEST(x = __shfl(x, (threadIdx.x + 1) & 63, 64) + b)      // 10 ds_bpermute + add
  {                                                        // 11 four independent fma chains (issue rate)
    double y0 = x, y1 = x + 1, y2 = x + 2, y3 = x + 3;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; i++) {
      y0 = fma(y0, a, b); y1 = fma(y1, a, b); y2 = fma(y2, a, b); y3 = fma(y3, a, b);
    }
    __asm__ volatile("" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[t] = t1 - t0;
    t++;
    x = y0 + y1 + y2 + y3;
  }
  {                                                        // 12 eight independent fma chains
    double y[8];
    for (int j = 0; j < 8; j++) y[j] = x + j;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
      for (int j = 0; j < 8; j++) y[j] = fma(y[j], a, b);
    }
#pragma unroll
    for (int j = 0; j < 8; j++) __asm__ volatile("" : "+v"(y[j]));
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[t] = t1 - t0;
    t++;
    for (int j = 0; j < 8; j++) x += y[j];
  }
  out[threadIdx.x] = x;
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&cyc, 32 * sizeof(unsigned long long));
  const char* names[] = {"fma", "mul", "add", "sqrt(IEEE)+add", "1/x(IEEE)+add", "v_rsq_f64+add", "v_rcp_f64+add",
                         "dpp bcast64+add", "dpp shr1 2x32+add", "lds st/ld+add", "bpermute+add",
                         "4 indep fma (per fma)", "8 indep fma (per fma)"};
  unsigned long long h[32];
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, out, cyc, 0.999999, 1e-7);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  for (int i = 0; i < 13; i++) {
    double per = (double)h[i] / ITERS;
    if (i == 11) per /= 4;
    if (i == 12) per /= 8;
    printf("%-24s %8.1f cycles\n", names[i], per);
  }
  return 0;
}
