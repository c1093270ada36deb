// A/B of the Kuka team backward kernel's largest product, S·[A B] (S 14x14 upper-triangular, [A B] 14x21),
// on the VALU (the k_bwd_team layout: 16-lane teams, four trajectories per wave, lane c owns column c and
// reads S from LDS) against the fp64 matrix cores (v_mfma_f64_16x16x4_f64: the wave computes each team's
// product in turn, 2 output tiles x 4 k-steps, operands staged through LDS). Both accumulate each output
// entry as the fma chain over l ascending (the MFMA's k-ordered steps), so the results must be equal bit for
// bit. Reports cycles per product set (4 trajectories) from s_memtime, averaged over REPS knots, for
// one wave per SIMD (the tail) and with the full chip busy (the bulk launch).
//   hipcc -O3 --offload-arch=gfx950 team_mfma_ab.hip -o team_mfma_ab && ./team_mfma_ab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

constexpr int n = 14, L = 21, REPS = 256, TPW = 4;
typedef double d4 __attribute__((ext_vector_type(4)));

// VALU: lane c of team t: out[i] = sum_{l >= i} S[i][l] * AB[l][c], l ascending (rolled dense product over
// the upper factor, as k_bwd_team's WPE=2 variant)
__global__ void __launch_bounds__(64) k_valu(const double* S, const double* AB, double* out, unsigned long long* cyc) {
  __shared__ double Sl[TPW][n * n];
  const int team = threadIdx.x / 16, tl = threadIdx.x % 16;
  const size_t w = (size_t)blockIdx.x * TPW + team;
  for (int e = tl; e < n * n; e += 16) Sl[team][e] = S[w * n * n + e];
  double ac[n], bc[n];
  const int c = tl;
  for (int i = 0; i < n; i++) {
    ac[i] = AB[w * n * L + i + n * c];
    bc[i] = (c + 16 < L) ? AB[w * n * L + i + n * (c + 16)] : 0.0;
  }
  __syncthreads();
  double r0[n], r1[n];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < REPS; rep++) {
#pragma unroll
    for (int i = 0; i < n; i++) {
      double x = 0.0, y = 0.0;
      for (int l = i; l < n; l++) {
        const double s = Sl[team][i + n * l];
        x = fma(s, ac[l], x);
        y = fma(s, bc[l], y);
      }
      r0[i] = x;
      r1[i] = y;
    }
#pragma unroll
    for (int i = 0; i < n; i++) ac[i] = ac[i] + r0[i] * 1e-300;  // keep the loop live, values unchanged
    __asm__ volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) {
    out[w * n * L + i + n * c] = r0[i];
    if (c + 16 < L) out[w * n * L + i + n * (c + 16)] = r1[i];
  }
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) / REPS;
}

// MFMA: per team t (in turn) the whole wave: D(16x32) = S(16x16, rows/cols 14,15 zero) * AB(16x32),
// k steps 0..15 by 4, lanes: A row = lane & 15, k = k0 + (lane >> 4); B col = lane & 15 (+16), same k
__global__ void __launch_bounds__(64) k_mfma(const double* S, const double* AB, double* out, unsigned long long* cyc) {
  __shared__ double Sl[TPW][16 * 16];
  __shared__ double Bl[TPW][16 * 32];
  const int lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
  for (int t = 0; t < TPW; t++) {
    const size_t w = (size_t)blockIdx.x * TPW + t;
    for (int e = lane; e < 256; e += 64) {
      const int i = e & 15, l = e >> 4;
      Sl[t][e] = (i < n && l < n && l >= i) ? S[w * n * n + i + n * l] : 0.0;
    }
    for (int e = lane; e < 512; e += 64) {
      const int l = e & 15, c = e >> 4;
      Bl[t][e] = (l < n && c < L) ? AB[w * n * L + l + n * c] : 0.0;
    }
  }
  __syncthreads();
  d4 acc[TPW][2];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < REPS; rep++) {
#pragma unroll
    for (int t = 0; t < TPW; t++) {
#pragma unroll
      for (int tile = 0; tile < 2; tile++) {
        d4 a4 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < 16; k0 += 4) {
          const int kk = k0 + lk;
          const double a = Sl[t][lr + 16 * kk];
          const double b = Bl[t][kk + 16 * (16 * tile + lr)];
          a4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, a4, 0, 0, 0);
        }
        acc[t][tile] = a4;
      }
    }
    __asm__ volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < TPW; t++) {
    const size_t w = (size_t)blockIdx.x * TPW + t;
    for (int tile = 0; tile < 2; tile++)
      for (int q = 0; q < 4; q++) {
        const int row = lk + 4 * q, col = 16 * tile + lr;
        if (row < n && col < L) out[w * n * L + row + n * col] = acc[t][tile][q];
      }
  }
  if (threadIdx.x == 0) cyc[blockIdx.x] = (t1 - t0) / REPS;
}

int main() {
  const int blocks_all = 256 * 4 * 2;  // two waves per SIMD: the bulk launch's occupancy
  const size_t W = (size_t)blocks_all * TPW;
  double *S, *AB, *o1, *o2;
  unsigned long long* cyc;
  hipMalloc(&S, W * n * n * 8);
  hipMalloc(&AB, W * n * L * 8);
  hipMalloc(&o1, W * n * L * 8);
  hipMalloc(&o2, W * n * L * 8);
  hipMalloc(&cyc, blocks_all * 8);
  double* h = (double*)malloc(W * n * L * 8);
  srand(1);
  for (size_t i = 0; i < W * n * n; i++) h[i] = (double)rand() / RAND_MAX - 0.5;
  hipMemcpy(S, h, W * n * n * 8, hipMemcpyHostToDevice);
  for (size_t i = 0; i < W * n * L; i++) h[i] = (double)rand() / RAND_MAX - 0.5;
  hipMemcpy(AB, h, W * n * L * 8, hipMemcpyHostToDevice);
  unsigned long long* hc = (unsigned long long*)malloc(blocks_all * 8);
  double *r1 = (double*)malloc(W * n * L * 8), *r2 = (double*)malloc(W * n * L * 8);
  for (int cfg = 0; cfg < 2; cfg++) {
    const int blocks = cfg == 0 ? 1 : blocks_all;
    double mean[2];
    for (int v = 0; v < 2; v++) {
      for (int rep = 0; rep < 2; rep++) {  // first launch warms up
        if (v == 0) hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64), 0, 0, S, AB, o1, cyc);
        else hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(64), 0, 0, S, AB, o2, cyc);
        hipDeviceSynchronize();
      }
      hipMemcpy(hc, cyc, blocks * 8, hipMemcpyDeviceToHost);
      double s = 0;
      for (int b = 0; b < blocks; b++) s += (double)hc[b];
      mean[v] = s / blocks;
    }
    printf("%s: cycles per 4-trajectory S*[A B]: valu %.0f  mfma %.0f  (mfma/valu %.2f)\n",
           cfg == 0 ? "one wave (tail)" : "2 waves/SIMD, whole chip (bulk)", mean[0], mean[1], mean[1] / mean[0]);
  }
  hipMemcpy(r1, o1, W * n * L * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r2, o2, W * n * L * 8, hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (size_t i = 0; i < W * n * L; i++) diff += memcmp(&r1[i], &r2[i], 8) != 0;
  printf("bitwise differences valu vs mfma: %zu of %zu\n", diff, W * n * L);
  return diff != 0;
}
