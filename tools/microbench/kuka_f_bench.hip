// Kuka RK3 rollout microbenchmark: the forward pass's dynamics alone (50 knots x 3 Kuka::f per lane,
// 32768 lanes = 4096 trajectories x 8 line-search trials, the config-5 spec round), in variants of the
// model code that must give bit-identical states:
//   0  tables through scalar loads at a laundered joint index (Kuka::f<T, false>)
//   1  tables as compile-time literals (Kuka::f<T, true>)
// each at 256- and 64-lane workgroups, one wave per SIMD. Prints ms per launch and the mismatch count
// against variant 0.
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 kuka_f_bench.hip -o kuka_f_bench
#include "../../trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd/csrc/tog_device.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

using namespace tog;

template <bool LIT>
struct KukaV {
  static constexpr int n = 14, m = 7, id = TOG_MODEL_KUKA;
  template <class T>
  __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    Kuka::f<T, LIT>(xd, x, u);
  }
};

template <bool LIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_roll(const double* __restrict__ X0, const double* __restrict__ U, double* __restrict__ XN, int lanes, int N,
       double dt) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  double x[14], xn[14], u[7];
#pragma unroll
  for (int i = 0; i < 14; i++) x[i] = X0[(size_t)t * 14 + i];
  for (int k = 0; k < N - 1; k++) {
#pragma unroll
    for (int i = 0; i < 7; i++) u[i] = U[((size_t)t * (N - 1) + k) * 7 + i];
    discrete_step<KukaV<LIT>, TOG_RK3>(xn, x, u, dt);
#pragma unroll
    for (int i = 0; i < 14; i++) x[i] = xn[i];
  }
#pragma unroll
  for (int i = 0; i < 14; i++) XN[(size_t)t * 14 + i] = x[i];
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

int main() {
  const int lanes = 32768, N = 51;
  const double dt = 0.01;
  double* hx = (double*)malloc(sizeof(double) * lanes * 14);
  double* hu = (double*)malloc(sizeof(double) * lanes * (N - 1) * 7);
  srand(7);
  for (int i = 0; i < lanes * 14; i++) hx[i] = (i % 14 < 7) ? 0.4 * ((double)rand() / RAND_MAX - 0.5) : 0.0;
  for (int i = 0; i < lanes * (N - 1) * 7; i++) hu[i] = 2.0 * ((double)rand() / RAND_MAX - 0.5);
  double *dx, *du, *dy[4];
  CK(hipMalloc(&dx, sizeof(double) * lanes * 14));
  CK(hipMalloc(&du, sizeof(double) * lanes * (N - 1) * 7));
  for (int v = 0; v < 4; v++) CK(hipMalloc(&dy[v], sizeof(double) * lanes * 14));
  CK(hipMemcpy(dx, hx, sizeof(double) * lanes * 14, hipMemcpyHostToDevice));
  CK(hipMemcpy(du, hu, sizeof(double) * lanes * (N - 1) * 7, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[4] = {"laundered wg256", "laundered wg64", "literal wg256", "literal wg64"};
  double* ref = (double*)malloc(sizeof(double) * lanes * 14);
  double* out = (double*)malloc(sizeof(double) * lanes * 14);
  for (int v = 0; v < 4; v++) {
    const int wg = (v & 1) ? 64 : 256;
    auto launch = [&]() {
      if (v < 2) hipLaunchKernelGGL(k_roll<false>, dim3(lanes / wg), dim3(wg), 0, 0, dx, du, dy[v], lanes, N, dt);
      else hipLaunchKernelGGL(k_roll<true>, dim3(lanes / wg), dim3(wg), 0, 0, dx, du, dy[v], lanes, N, dt);
    };
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 5;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(v == 0 ? ref : out, dy[v], sizeof(double) * lanes * 14, hipMemcpyDeviceToHost));
    long bad = 0, nonfinite = 0;
    for (int i = 0; i < lanes * 14; i++) {
      const double a = (v == 0 ? ref : out)[i];
      if (!isfinite(a)) nonfinite++;
      if (v && memcmp(&ref[i], &out[i], 8)) bad++;
    }
    printf("%-16s %8.3f ms/launch  mismatches vs 0: %ld  nonfinite %ld\n", names[v], ms / reps, bad, nonfinite);
  }
  return 0;
}
