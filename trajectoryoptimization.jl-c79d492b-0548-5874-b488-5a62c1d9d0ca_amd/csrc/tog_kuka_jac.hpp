// tog_kuka_jac.hpp — the Kuka iiwa's RK3 dynamics Jacobian (BASELINE config 5) in stage-chain form.
//
// jacobian!(prob, solver) (src/solvers.jl:126 -> src/model.jl:301-306, 491-522) for Model(urdf) with
// rk3 (src/integration.jl:149-158). The derivative is the one forward-mode duals give through the RK3
// step, evaluated as the chain of three stage Jacobians (oracle
// kuka_rk3_jacobian_chain, same operations in the same order):
//   J_s = ∂f/∂[s; u] at the stage inputs s_1 = x, s_2 = x + k1/2, s_3 = (x - k1) + 2 k2 (duals seeded at
//         the stage input; only rows 7..13, v̇, are not trivial: rows 0..6 are q̇ = v),
//   K1 = J_1 dt, T2 = I + K1/2, F2 = J_2 [T2; E_u], K2 = F2 dt, T3 = (I - K1) + 2 K2, F3 = J_3 [T3; E_u],
//   K3 = F3 dt, [A B] = I + ((K1 + 4 K2) + K3)/6.
// Four launches per Jacobian, all over the knot slots of the active trajectories:
//   k_kuka_points  one lane per knot: the primal stage inputs s_2, s_3 (two RNEA/CRBA/Cholesky solves);
//   k_kuka_sjac<Q> one lane per (knot, stage, q_p): the full dual RBD step, one partial;
//   k_kuka_sjac<V> one lane per (knot, stage, p): the v_p partial at fixed q (no mass-matrix or Cholesky
//                  partials, only the RNEA bias and the solve carry it), then the u_p column
//                  ∂v̇/∂u_p = M⁻¹ e_p by two triangular solves with the lane's primal factor;
//   k_kuka_chain   one wave per knot: the RK3 combination, the two 7x14 · 14x21 chain products on the fp64
//                  matrix cores (v_mfma_f64_16x16x4_f64, k in order — the fma chain of the oracle) and
//                  the store of [A B] (and the infeasible model's identity slack block).
// Exact zeros of the seeded tangents are skipped; the result is the full dual's bit for bit, up to the
// sign of a zero.
#pragma once

namespace tog {

constexpr int KJ_N = 14, KJ_M = 7, KJ_L = 21;
constexpr int KJ_OFF_T2 = 0, KJ_OFF_T3 = 14, KJ_OFF_J = 28;  // per knot: s_2, s_3, J[3][7][21]
constexpr int KJ_WSK = 472;                                   // doubles per knot slot (469, padded)

__device__ __forceinline__ double* kj_slot(const DevBuffers& Bf, long long t) { return Bf.jws + t * KJ_WSK; }

// (traj, knot) of knot slot t (t < slots * (N - 1)); -1 when the trajectory takes no Jacobian this step
__device__ __forceinline__ long long kj_traj(const DevBuffers& Bf, const DevProblem* P, long long t, int* k) {
  const int N = P->N;
  *k = (int)(t % (N - 1));
  const long long b = traj_of_slot(Bf, t / (N - 1), P->B);
  if (b < 0 || !Bf.st[b].active || Bf.st[b].ls_pend) return -1;
  return b;
}

// ∂v̇/∂u_p into J[i][14 + p]: the partials solve() carries when only u_p is seeded (u.p - τ.p = e_p
// exactly; every L, τ partial is zero; the quotient's partial is x.p * (1/L_ii), as kdiv)
__device__ __forceinline__ void kj_u_column(double* J, const double (*L)[7], int p) {
  double y[7], g[7];
#pragma unroll
  for (int i = 0; i < 7; i++) {
    double t = (i == p) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < i; k++) t = t - L[i][k] * y[k];
    y[i] = t * (1.0 / L[i][i]);
  }
#pragma unroll
  for (int i = 6; i >= 0; i--) {
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < 7; k++) t = t - L[k][i] * g[k];
    g[i] = t * (1.0 / L[i][i]);
  }
#pragma unroll
  for (int i = 0; i < 7; i++) J[i * KJ_L + 14 + p] = g[i];
}

// primal f at (x, u): v̇ into vd, and the Cholesky factor of M(q)
__device__ __forceinline__ void kj_primal(double* vd, double (*L)[7], const double* x, const double* u) {
  double tau[7], cq[7], sq[7];
  Kuka::bias(tau, cq, sq, x, x + 7);
  Kuka::mass(L, cq, sq);
  Kuka::chol(L);
  Kuka::solve(vd, L, u, tau);
}

template <class M>
__global__ void __launch_bounds__(64) k_kuka_points(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  constexpr int n = KJ_N, m = M::m;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  int k;
  const long long b = kj_traj(Bf, P, t, &k);
  if (b < 0) return;
  const int N = P->N;
  const double dt = P->dt;
  const double* xg = Bf.X + ((size_t)b * N + k) * n;
  const double* ug = Bf.U + ((size_t)b * (N - 1) + k) * m;
  double x[n], u[7], k1[n], s[n], vd[7], L[7][7];
#pragma unroll
  for (int i = 0; i < n; i++) x[i] = xg[i];
#pragma unroll
  for (int i = 0; i < 7; i++) u[i] = ug[i];
  double* w = kj_slot(Bf, t);
  // stage 1 at x: k1 = f dt, s_2 = x + k1/2 (discrete_step's rk3)
  kj_primal(vd, L, x, u);
#pragma unroll
  for (int i = 0; i < n; i++) {
    k1[i] = (i < 7 ? x[7 + i] : vd[i - 7]) * dt;
    s[i] = x[i] + k1[i] / 2.0;
    w[KJ_OFF_T2 + i] = s[i];
  }
  // stage 2 at s_2: k2 = f dt, s_3 = (x - k1) + 2 k2
  kj_primal(vd, L, s, u);
#pragma unroll
  for (int i = 0; i < n; i++) {
    const double k2 = (i < 7 ? s[7 + i] : vd[i - 7]) * dt;
    s[i] = (x[i] - k1[i]) + 2.0 * k2;
  }
#pragma unroll
  for (int i = 0; i < n; i++) w[KJ_OFF_T3 + i] = s[i];
}

// one lane per (knot, stage, direction p): TYPE 0 the q_p partial (full dual step), TYPE 1 the v_p partial
template <class M, int TYPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TOG_JAC_WAVES)))
k_kuka_sjac(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  constexpr int n = KJ_N, m = M::m;
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total * 21) return;
  const long long t = tid / 21;
  const int r = (int)(tid - t * 21), st = r / 7, p = r - 7 * st;
  int k;
  const long long b = kj_traj(Bf, P, t, &k);
  if (b < 0) return;
  const int N = P->N;
  double* w = kj_slot(Bf, t);
  const double* sg = st == 0 ? Bf.X + ((size_t)b * N + k) * n : w + (st == 1 ? KJ_OFF_T2 : KJ_OFF_T3);
  const double* ug = Bf.U + ((size_t)b * (N - 1) + k) * m;
  double* J = w + KJ_OFF_J + st * 7 * KJ_L;
  if constexpr (TYPE == 0) {
    Dual<1> xs[n], us[7], fd[n];
#pragma unroll
    for (int i = 0; i < n; i++) {
      xs[i].v = sg[i];
      xs[i].g[0] = (i == p) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 7; i++) {
      us[i].v = ug[i];
      us[i].g[0] = 0.0;
    }
    Kuka::f(fd, xs, us);
#pragma unroll
    for (int i = 0; i < 7; i++) J[i * KJ_L + p] = fd[7 + i].g[0];
  } else {
    double q[7], u[7], L[7][7], cq[7], sq[7];
    Dual<1> qd[7], tau[7], vd[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
      q[i] = sg[i];
      qd[i].v = sg[7 + i];
      qd[i].g[0] = (i == p) ? 1.0 : 0.0;
      u[i] = ug[i];
    }
    Kuka::bias(tau, cq, sq, q, qd);
    Kuka::mass(L, cq, sq);
    Kuka::chol(L);
    Kuka::solve(vd, L, u, tau);
#pragma unroll
    for (int i = 0; i < 7; i++) J[i * KJ_L + 7 + p] = vd[i].g[0];
    kj_u_column(J, L, p);
  }
}

// The RK3 combination of one knot per wave. Element e = i + 14 p of a 14 x 21 block is lane (e mod 64),
// register e / 64 (5 registers). T (the stage input's tangent, B operand of the chain product) sits in LDS
// as T[p][16] (rows 14, 15 zero); the product's rows 0..6 (v̇) come back through a 7 x 21 LDS stash.
typedef double kj_d4 __attribute__((ext_vector_type(4)));
constexpr int KJ_E = KJ_N * KJ_L;             // 294 elements
constexpr int KJ_ER = (KJ_E + WAVE - 1) / WAVE;  // 5 per lane
constexpr int KJ_LDS = 441 + 16 * KJ_L + 7 * KJ_L;  // J, T, stash (doubles per wave)

// F rows 7..13 = J_s[:, 0:14] T + J_s[:, 14:21] E_u on the matrix cores: 16 x 16 output tiles (rows
// 0..6 used), 4-deep k steps over j = 0..15 (14, 15 zero); D = A B + C accumulates each step's four
// products as fmas in k order (tools/microbench/mfma_f64_order.hip), from C = the u column.
__device__ __forceinline__ void kj_chain_product(double* stash, const double* Js, const double* T, int lane) {
  const int lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int tile = 0; tile < 2; tile++) {
    const int col = 16 * tile + lr;  // output column p
    kj_d4 acc;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = lk + 4 * q;
      acc[q] = (row < 7 && col >= 14 && col < KJ_L) ? Js[row * KJ_L + col] : 0.0;
    }
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += 4) {
      const int kk = k0 + lk;
      const double a = (lr < 7 && kk < 14) ? Js[lr * KJ_L + kk] : 0.0;
      const double bv = (col < KJ_L) ? T[col * 16 + kk] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = lk + 4 * q;
      if (row < 7 && col < KJ_L) stash[row + 7 * col] = acc[q];
    }
  }
}

// (one-wave workgroups: an inactive knot retires its whole workgroup, and __syncthreads is a wave barrier)
template <class M>
__global__ void __launch_bounds__(64) k_kuka_chain(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  constexpr int n = KJ_N, L = M::n + M::m;  // L = 21 (35 with the infeasible model's slack columns)
  __shared__ double lds[KJ_LDS];
  const int lane = threadIdx.x;
  const long long t = blockIdx.x;
  if (t >= total) return;
  int k;
  const long long b = kj_traj(Bf, P, t, &k);
  if (b < 0) return;
  const int N = P->N;
  const double dt = P->dt;
  double* Jl = lds;
  double* T = Jl + 441;
  double* stash = T + 16 * KJ_L;
  const double* w = kj_slot(Bf, t);
  for (int e = lane; e < 441; e += WAVE) Jl[e] = w[KJ_OFF_J + e];
  for (int e = lane; e < 2 * KJ_L; e += WAVE) T[(e >> 1) * 16 + 14 + (e & 1)] = 0.0;
  double K1[KJ_ER], Ss[KJ_ER];
  // stage 1: K1 = J_1 dt (rows 0..6: ∂q̇/∂v = I), T2 = I + K1/2
#pragma unroll
  for (int r = 0; r < KJ_ER; r++) {
    const int e = lane + WAVE * r, i = e % n, p = e / n;
    if (e < KJ_E) {
      const double f1 = (i < 7) ? ((p == 7 + i) ? 1.0 : 0.0) : Jl[(i - 7) * KJ_L + p];
      K1[r] = f1 * dt;
      T[p * 16 + i] = ((i == p) ? 1.0 : 0.0) + K1[r] / 2.0;
    }
  }
  __syncthreads();
  // stage 2: F2 = J_2 [T2; E_u]; K2 = F2 dt; T3 = (I - K1) + 2 K2; S = K1 + 4 K2
  kj_chain_product(stash, Jl + 7 * KJ_L, T, lane);
  __syncthreads();
  double F[KJ_ER];
#pragma unroll
  for (int r = 0; r < KJ_ER; r++) {
    const int e = lane + WAVE * r, i = e % n, p = e / n;
    if (e < KJ_E) F[r] = (i < 7) ? T[p * 16 + 7 + i] : stash[(i - 7) + 7 * p];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < KJ_ER; r++) {
    const int e = lane + WAVE * r, i = e % n, p = e / n;
    if (e < KJ_E) {
      const double k2 = F[r] * dt;
      T[p * 16 + i] = (((i == p) ? 1.0 : 0.0) - K1[r]) + 2.0 * k2;
      Ss[r] = K1[r] + 4.0 * k2;
    }
  }
  __syncthreads();
  // stage 3: F3 = J_3 [T3; E_u]; K3 = F3 dt; [A B] = I + (S + K3)/6
  kj_chain_product(stash, Jl + 14 * KJ_L, T, lane);
  __syncthreads();
  double* out = Bf.AB + ((size_t)b * (N - 1) + k) * n * L;
#pragma unroll
  for (int r = 0; r < KJ_ER; r++) {
    const int e = lane + WAVE * r, i = e % n, p = e / n;
    if (e < KJ_E) {
      const double f3 = (i < 7) ? T[p * 16 + 7 + i] : stash[(i - 7) + 7 * p];
      const double s = Ss[r] + f3 * dt;
      out[e] = ((i == p) ? 1.0 : 0.0) + tog_div6(s);
    }
  }
  if constexpr (L > KJ_L) {  // add_slack_controls: ∂x⁺/∂s = I (src/model.jl:771-774)
    for (int e = KJ_E + lane; e < n * L; e += WAVE) {
      const int i = e % n, j = e / n - KJ_L;
      out[e] = (i == j) ? 1.0 : 0.0;
    }
  }
}

}  // namespace tog
