// Accumulation order of v_mfma_f64_16x16x4_f64 on gfx950: D = A·B + C for a 16x4 A, 4x16 B, compared
// bit for bit with three host formulas over random operands (with exponents spread so that the order
// matters): (a) the k-ordered fma chain starting from C, fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0,c)))),
// (b) C + ((a0b0 + a1b1) + (a2b2 + a3b3)) rounded per op, (c) the exact sum rounded once (long double
// approximation). Prints the mismatch count of each. Chained MFMAs (K = 16 as 4 steps) are checked
// against the chain over k = 0..15.
//   hipcc -O2 --offload-arch=gfx950 -ffp-contract=off mfma_f64_order.hip -o mfma_f64_order
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef double d4 __attribute__((ext_vector_type(4)));

// one wave per problem: A (16 x K) column-major, B (K x 16) column-major, C/D (16 x 16) column-major
__global__ void k_mfma(const double* A, const double* B, const double* C, double* D, int K) {
  const int p = blockIdx.x, lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
  const double* a = A + (size_t)p * 16 * K;
  const double* b = B + (size_t)p * K * 16;
  const double* c = C + (size_t)p * 256;
  d4 acc;
  for (int r = 0; r < 4; r++) acc[r] = c[(lk + 4 * r) + 16 * lr];
  for (int k0 = 0; k0 < K; k0 += 4) {
    const double av = a[lr + 16 * (k0 + lk)];
    const double bv = b[(k0 + lk) + K * lr];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; r++) D[(size_t)p * 256 + (lk + 4 * r) + 16 * lr] = acc[r];
}

static double rnd(unsigned* s) {
  *s = *s * 1664525u + 1013904223u;
  const double m = ((*s >> 8) & 0xffff) / 65536.0 - 0.5;
  *s = *s * 1664525u + 1013904223u;
  const int e = (int)((*s >> 8) % 40) - 20;
  return ldexp(m, e);
}

int main() {
  const int P = 512;
  int bad_total = 0;
  for (int K = 4; K <= 16; K += 12) {
    const size_t na = (size_t)P * 16 * K, nb = (size_t)P * K * 16, nc = (size_t)P * 256;
    double *A = (double*)malloc(na * 8), *B = (double*)malloc(nb * 8), *C = (double*)malloc(nc * 8),
           *D = (double*)malloc(nc * 8);
    unsigned s = 12345u + K;
    for (size_t i = 0; i < na; i++) A[i] = rnd(&s);
    for (size_t i = 0; i < nb; i++) B[i] = rnd(&s);
    for (size_t i = 0; i < nc; i++) C[i] = (i % 7 == 0) ? 0.0 : rnd(&s);
    double *dA, *dB, *dC, *dD;
    hipMalloc(&dA, na * 8);
    hipMalloc(&dB, nb * 8);
    hipMalloc(&dC, nc * 8);
    hipMalloc(&dD, nc * 8);
    hipMemcpy(dA, A, na * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B, nb * 8, hipMemcpyHostToDevice);
    hipMemcpy(dC, C, nc * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(P), dim3(64), 0, 0, dA, dB, dC, dD, K);
    hipMemcpy(D, dD, nc * 8, hipMemcpyDeviceToHost);
    long bad_chain = 0, bad_pair = 0, bad_once = 0;
    for (int p = 0; p < P; p++)
      for (int j = 0; j < 16; j++)
        for (int i = 0; i < 16; i++) {
          const double* a = A + (size_t)p * 16 * K;
          const double* b = B + (size_t)p * K * 16;
          const double c = C[(size_t)p * 256 + i + 16 * j];
          double chain = c, pair = c;
          long double once = c;
          for (int k0 = 0; k0 < K; k0 += 4) {
            double pr[4];
            for (int k = k0; k < k0 + 4; k++) {
              chain = fma(a[i + 16 * k], b[k + K * j], chain);
              pr[k - k0] = a[i + 16 * k] * b[k + K * j];
              once += (long double)a[i + 16 * k] * (long double)b[k + K * j];
            }
            pair = pair + ((pr[0] + pr[1]) + (pr[2] + pr[3]));
          }
          const double d = D[(size_t)p * 256 + i + 16 * j];
          bad_chain += memcmp(&d, &chain, 8) != 0;
          bad_pair += memcmp(&d, &pair, 8) != 0;
          const double od = (double)once;
          bad_once += memcmp(&d, &od, 8) != 0;
        }
    printf("K=%d entries=%d mismatches: k-ordered fma chain %ld, pairwise %ld, single rounding %ld\n", K, P * 256,
           bad_chain, bad_pair, bad_once);
    bad_total += (int)bad_chain;
    hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dD);
    free(A); free(B); free(C); free(D);
  }
  return 0;
}
