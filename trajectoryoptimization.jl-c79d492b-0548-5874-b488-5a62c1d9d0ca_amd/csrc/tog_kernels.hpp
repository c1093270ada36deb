// tog_kernels.hpp — HIP kernels of the batched iLQR / AL-iLQR hot path (gfx950, wave64, fp64).
//
// Kernel map (SURVEY.md §2 "kernel set the build must create"):
//   k_init          solve!/reset! + initial rollout + initial (AL) cost      ilqr_methods.jl:3-20, augmented_lagrangian_methods.jl:2-16
//   k_rollout_open  rollout!(prob)                                           src/rollout.jl:25-38
//   k_jacobian      jacobian!(prob, solver): ForwardDiff duals through RK3/4 src/model.jl:301-306, 491-522
//   k_backward      cost_expansion! + backwardpass! (std / sqrt)             ilqr_methods.jl:55-62, backward_pass.jl:1-192
//   k_forward       forwardpass! line search + solve! bookkeeping + AL dual/penalty update
//                                                                           forward_pass.jl:5-85, ilqr_methods.jl:21-45,
//                                                                           augmented_lagrangian_methods.jl:53-126
//   k_cost / k_rollout / k_update_constraints   step-level entry points
//   k_batch_stats   batch reduction (n_active, ΣJ, max c_max) for stopping / the RCCL all-reduce
//
// Mapping: the Riccati recursion is strictly serial in the knot index, so parallelism comes from
// the batch. k_backward runs one 64-lane wavefront per trajectory with the whole per-knot working
// set (S, [A|B], Q blocks, QR workspaces) in LDS; k_jacobian runs one thread per
// (trajectory, knot, partial-chunk); rollouts run one thread per trajectory.
#pragma once

#include "tog_device.hpp"
#include <string.h>

namespace tog {

// max constraint rows per knot in the LDS backward kernel's layout (problems/quadrotor_maze.jl:
// 12 bound rows + 44 cylinders per stage knot, + 13 slack rows in its infeasible-start problem)
constexpr int PCAP = 72;
template <class M>
__host__ __device__ constexpr int pcap_of() { return PCAP; }
constexpr int WAVE = 64;

// Compacted launches in the convergence tail (DevBuffers::act_list, built by k_list_active at the start
// of a solve step): slot i of a launch is the i-th active trajectory of the step, -1 past the list's
// end; without a list, slot i is trajectory i (-1 at or past B). Kernels then launch over
// ceil(n_active) slots instead of the whole batch, and idle trajectories cost no empty blocks.
__device__ __forceinline__ long long traj_of_slot(const DevBuffers& Bf, long long i, long long B) {
  if (Bf.act_list) return i < (long long)*Bf.act_count ? (long long)Bf.act_list[i] : -1;
  return i < B ? i : -1;
}
__device__ __forceinline__ long long slot_count(const DevBuffers& Bf, long long B) {
  return Bf.act_list ? (long long)*Bf.act_count : B;
}

__device__ __forceinline__ void wsync() { __syncthreads(); }  // one-wave workgroups: s_barrier is ~free

// candidate layout of the line search (k_ls_spec<CAND>): per knot the elements c of [ū_k (m) | x̄_k (n)]
// in quads q = c / 4; element (k, c) of trial j of trajectory b at
//   (((b N + k) Q + q) NCP + j) 4 + c % 4,      Q = ceil((n + m) / 4), NCP = nc rounded up to 8.
// A round's lanes for one trajectory's trials are adjacent: each trial stores 32-byte quads and the 8
// trials of a round fill 256 contiguous bytes, while k_ls_apply reads the winner's quads 32 bytes at a time.
template <class M>
__host__ __device__ constexpr int cand_w() {
  return M::n + M::m;
}
template <class M>
__host__ __device__ constexpr int cand_q() {
  return (M::n + M::m + 3) / 4;
}
__device__ __forceinline__ size_t cand_at(int k, int c, int Q, int ncp) {
  return ((size_t)(k * Q + (c >> 2)) * ncp) * 4 + (c & 3);
}
template <class M>
__host__ __device__ constexpr int nq_of() {
  return M::n + M::m + M::n * M::n + M::m * M::m + M::m * M::n;
}

// =============================================================================================
// Thread-level trajectory helpers
// =============================================================================================

// AL terms λ'c + ½ c'Iμ c of one knot (augmented_lagrangian_methods.jl:298-313), rows in order. The
// multipliers are loaded four rows at a time so their global loads overlap instead of serialising
// one round trip per row. Ck (constraint values out) may be null.
template <class M, class RowPtr, bool NOIDX = false>
__device__ __forceinline__ void al_knot_terms(RowPtr rows, int cnt, const double* lamk, const double* muk,
                                              const double* x, const double* u, double& lc, double& cIc,
                                              double* Ck) {
  for (int base = 0; base < cnt; base += 4) {
    double lv[4], mv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      lv[q] = (base + q < cnt) ? lamk[base + q] : 0.0;
      mv[q] = (base + q < cnt) ? muk[base + q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (base + q < cnt) {
        const ConRow r = uniform_row(load_row(rows + base + q));
        const double c = row_value_m<M, NOIDX>(r, x, u);
        const double l = lv[q];
        const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(r) ? ((c >= 0.0) || (l > 0.0)) : true;
        const double w = a ? mv[q] : 0.0;
        lc = fma(l, c, lc);
        cIc = fma(c * w, c, cIc);
        if (Ck) Ck[base + q] = c;
      }
    }
  }
}

// AL/objective cost of (Xs, Us) for trajectory b (objective.jl:40-48, augmented_lagrangian_methods.jl:298-313).
// Writes the constraint values C when Cout != nullptr (A.10: cost() updates C as a side effect).
template <class M>
__device__ double traj_cost(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, const double* Xs,
                            const double* Us, bool al, double* Cout) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  double J = 0.0, Jc = 0.0;
  for (int k = 0; k < N - 1; k++) J += stage_cost_m<M>(P, k, Xs + (size_t)k * n, Us + (size_t)k * m);
  J += terminal_cost_m<M>(P, Xs + (size_t)(N - 1) * n);
  if (!al) return J;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  for (int k = 0; k < N; k++) {
    const int cnt = knot_count(P, k);
    if (cnt == 0) continue;
    const cptr<ConRow> rows = knot_rows(P, k);
    const double* x = Xs + (size_t)k * n;
    const double* u = (k < N - 1) ? Us + (size_t)k * m : nullptr;
    double lc = 0.0, cIc = 0.0;
    al_knot_terms<M>(rows, cnt, lam + (size_t)k * pmax, mu + (size_t)k * pmax, x, u, lc, cIc,
                  Cout ? Cout + (size_t)k * pmax : nullptr);
    Jc += lc + 0.5 * cIc;
  }
  return J + Jc;
}

// rollout!(prob, solver, α) (src/rollout.jl:2-23): writes X̄, Ū; false on divergence / NaN.
template <class M, int INTEG>
__device__ bool traj_rollout(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, double alpha) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* K = Bf.K + (size_t)b * (N - 1) * m * n;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  double* Xb = Bf.Xb + (size_t)b * N * n;
  double* Ub = Bf.Ub + (size_t)b * (N - 1) * m;
  double xb[n], dx[n], ub[m], xn[n];
#pragma unroll
  for (int i = 0; i < n; i++) {
    xb[i] = Bf.x0[(size_t)b * n + i];
    Xb[i] = xb[i];
  }
  const double smax = P->o.max_state_value, umax = P->o.max_control_value;
  for (int k = 1; k < N; k++) {
    const double* x = X + (size_t)(k - 1) * n;
#pragma unroll
    for (int i = 0; i < n; i++) dx[i] = xb[i] - x[i];
    const double* Kk = K + (size_t)(k - 1) * m * n;
#pragma unroll
    for (int i = 0; i < m; i++) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < n; j++) t = fma(Kk[i + m * j], dx[j], t);
      ub[i] = (U[(size_t)(k - 1) * m + i] + t) + alpha * d[(size_t)(k - 1) * m + i];
      Ub[(size_t)(k - 1) * m + i] = ub[i];
    }
    discrete_step<M, INTEG>(xn, xb, ub, P->dt);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < n; i++) {
      xb[i] = xn[i];
      Xb[(size_t)k * n + i] = xn[i];
      ok = ok && (fabs(xn[i]) < smax);
    }
#pragma unroll
    for (int i = 0; i < m; i++) ok = ok && (fabs(ub[i]) < umax);
    if (!ok) return false;
  }
  return true;
}

// open-loop rollout!(X, model, U, dt) (src/rollout.jl:33-38) into X, if any X is non-finite.
template <class M, int INTEG>
__device__ void traj_rollout_open(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N;
  double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  bool finite = true;
  for (int i = 0; i < n * N; i++) finite = finite && isfinite(X[i]);
  if (finite) return;
  double x[n], xn[n], u[m];
#pragma unroll
  for (int i = 0; i < n; i++) {
    x[i] = Bf.x0[(size_t)b * n + i];
    X[i] = x[i];
  }
  for (int k = 0; k < N - 1; k++) {
#pragma unroll
    for (int i = 0; i < m; i++) u[i] = U[(size_t)k * m + i];
    discrete_step<M, INTEG>(xn, x, u, P->dt);
#pragma unroll
    for (int i = 0; i < n; i++) {
      x[i] = xn[i];
      X[(size_t)(k + 1) * n + i] = xn[i];
    }
  }
}

// compute_gradient (ilqr_methods.jl:104-116): the entries of vcat(Q[1].x, Q[1].u, ..., Q[N].x) of the plain
// cost_expansion! (objective.jl:65-68, augmented_lagrangian_methods.jl:231-276 inside AL solves) at the
// current X, U, in order, passed to visit(value). Same operations as the oracle's expansion_stage /
// expansion_terminal / oc_cost_expansion(sq = 0); the AL terms use the constraint values of X, U (obj.C
// after the accepted trajectory's cost evaluation, A.10) and add each row's gradient entries in row order
// (the oracle's dense loops add exact zeros for the other rows). One lane per trajectory: gradient_type
// :ℓ2 / :ℓinf only.
template <class M, class F>
__device__ void expansion_gradient_entries(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b,
                                           bool al, F&& visit) {
  constexpr int n = M::n, m = M::m, W = n + m;
  constexpr bool MT = ModelTraits<M>::min_time;
  const int N = P->N, pmax = P->pmax;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  for (int k = 0; k < N; k++) {
    const bool term = (k == N - 1);
    const double* x = X + (size_t)k * n;
    const double* u = term ? nullptr : U + (size_t)k * m;
    double q[W];
    if (!term) {
      const CostView C_ = cost_at<n, m>(P, k);
      const double dt = MT ? u[m - 1] * u[m - 1] : P->dt;
      double gx[n], gu[m];
      for (int i = 0; i < n; i++) {
        double a = 0.0, c = 0.0;
        for (int j = 0; j < n; j++) a = fma(C_.Q[i + n * j], x[j], a);
        for (int j = 0; j < m; j++) c = fma(C_.H[j + m * i], u[j], c);
        gx[i] = (a + C_.q[i]) + c;
        q[i] = gx[i] * dt;
      }
      for (int i = 0; i < m; i++) {
        double a = 0.0, c = 0.0;
        for (int j = 0; j < m; j++) a = fma(C_.R[i + m * j], u[j], a);
        for (int j = 0; j < n; j++) c = fma(C_.H[i + m * j], x[j], c);
        gu[i] = (a + C_.r[i]) + c;
        q[n + i] = gu[i] * dt;
      }
      if constexpr (MT) {  // MinTimeCost (minimum_time.jl:155-188): Q.u[end] = τ(2ℓ1 + R), Q.x[end] = R x[end]
        const double R = P->R_min_time, tau = u[m - 1];
        const double l1 = stage_cost_dt<n, m>(P, k, x, u, 1.0);
        q[n + m - 1] = tau * (2.0 * l1 + R);
        q[n - 1] = R * x[n - 1];
      }
    } else {
      for (int i = 0; i < n; i++) {
        double a = 0.0;
        for (int j = 0; j < n; j++) a = fma(P->Qf[i + n * j], x[j], a);
        q[i] = a + P->qf[i];
      }
      if constexpr (MT) q[n - 1] = P->R_min_time * x[n - 1];
    }
    const int p = al ? knot_count(P, k) : 0;
    if (p > 0) {  // Q.x .+= cx'g ; Q.u .+= cu'g,  g = Iμ c + λ over the active set
      const cptr<ConRow> rows = knot_rows(P, k);
      double t[W];
      for (int i = 0; i < W; i++) t[i] = 0.0;
      for (int r = 0; r < p; r++) {
        const ConRow row = load_row(rows + r);
        const double c = row_value_m<M>(row, x, u);
        const double l = lam[(size_t)k * pmax + r];
        const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(row) ? ((c >= 0.0) || (l > 0.0)) : true;
        const double w = a ? mu[(size_t)k * pmax + r] : 0.0;
        const double g = w * c + l;
        int idx[row_grad_cap<M>()];
        double v[row_grad_cap<M>()];
        const int nz = row_grad_m<M>(row, x, u, idx, v);
        for (int z = 0; z < nz; z++)
          if (!term || idx[z] < n) t[idx[z]] = fma(v[z], g, t[idx[z]]);
      }
      for (int i = 0; i < (term ? n : W); i++) q[i] += t[i];
    }
    for (int i = 0; i < (term ? n : W); i++) visit(q[i]);
  }
}

// gradient_todorov (ilqr_methods.jl:122-129, A.3) / gradient_feedforward (:135-137) / :ℓ2, :ℓinf (:96-99:
// LinearAlgebra.generic_normInf; for ℓ2 the unscaled sum of squares in index order of generic_norm2, the
// oracle's jl_norm2 — Julia 1.1 passes these long vectors to BLAS.nrm2, whose accumulation the restatement
// does not reproduce bit for bit)
template <class M>
__device__ __attribute__((noinline)) double traj_gradient_norm(const DevProblem* __restrict__ P,
                                                               const DevBuffers& Bf, long long b, bool al) {
  // (not inlined: its arrays would otherwise cost the bookkeeping kernels' common path registers)
  if (P->o.gradient_type == 3) {
    double r = NAN;
    bool first = true;
    expansion_gradient_entries<M>(P, Bf, b, al, [&](double g) {
      const double v = fabs(g);
      r = first ? v : ((isnan(r) || r > v) ? r : v);
      first = false;
    });
    return r;
  }
  if (P->o.gradient_type == 2) {
    double mx = 0.0;
    long long len = 0;
    expansion_gradient_entries<M>(P, Bf, b, al, [&](double g) {
      mx = tog_jlmax(mx, fabs(g));
      len++;
    });
    if (mx != mx || mx == 0.0 || isinf(mx)) return mx;
    double s = 0.0;
    bool first = true;
    if (isfinite((double)len * mx * mx) && mx * mx != 0.0) {
      expansion_gradient_entries<M>(P, Bf, b, al, [&](double g) {
        s = first ? g * g : s + g * g;
        first = false;
      });
      return sqrt(s);
    }
    expansion_gradient_entries<M>(P, Bf, b, al, [&](double g) {
      const double t = fabs(g) / mx;
      s = first ? t * t : s + t * t;
      first = false;
    });
    return mx * sqrt(s);
  }
  return 0.0;
}

template <class M>
__device__ double traj_gradient(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, bool al) {
  constexpr int m = M::m;
  const int N = P->N;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  if (P->o.gradient_type >= 2) return traj_gradient_norm<M>(P, Bf, b, al);
  if (P->o.gradient_type == 1) {
    double g = 0.0;
    for (int k = 0; k < N - 1; k++) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < m; i++) t = fma(d[k * m + i], d[k * m + i], t);
      g = fmax(g, sqrt(t));
    }
    return g;
  }
  double sum = 0.0;
  for (int k = 0; k < N - 1; k++) {
    double mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < m; i++) {
      const double v = fabs(d[k * m + i]) / (fabs(U[k * m + i]) + 1.0);
      if (v > mx || isnan(v)) mx = v;
    }
    sum += mx;
  }
  return sum / N;
}

// max_violation(solver) (augmented_lagrangian_methods.jl:171-184) from the stored C
__device__ inline double traj_max_violation(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b) {
  const int N = P->N, pmax = P->pmax;
  const double* C = Bf.C + (size_t)b * N * pmax;
  double c_max = 0.0;
  for (int k = 0; k < N; k++) {
    const int cnt = knot_count(P, k);
    if (cnt == 0) continue;
    const cptr<ConRow> rows = knot_rows(P, k);
    double e = 0.0, im = -INFINITY;
    int ni = 0;
    for (int i = 0; i < cnt; i++) {
      const double c = C[(size_t)k * pmax + i];
      if (row_inequality(load_row(rows + i))) {
        ni++;
        im = tog_jlmax(im, c);  // maximum(C.inequality): NaN propagates (Julia max)
      } else {
        e = tog_jlmax(e, fabs(c));  // norm(C.equality, Inf)
      }
    }
    c_max = tog_jlmax(e, c_max);
    if (ni > 0) c_max = tog_jlmax(tog_jlmax(0.0, im), c_max);
  }
  return c_max;
}

__device__ inline void set_tolerances(const DevProblem* __restrict__ P, TrajState& s, int mode) {
  // set_tolerances! (augmented_lagrangian_methods.jl:39-50)
  if (mode == TOG_MODE_AL) {
    const bool last = (s.al_iter == P->o.al_iterations);
    s.cost_tol = last ? P->o.al_cost_tolerance : P->o.al_cost_tolerance_intermediate;
    s.grad_tol = last ? P->o.al_gradient_norm_tolerance : P->o.al_gradient_norm_tolerance_intermediate;
  } else {
    s.cost_tol = P->o.cost_tolerance;
    s.grad_tol = P->o.gradient_norm_tolerance;
  }
}

// =============================================================================================
// k_init: reset! + (AL) multiplier init + rollout!(prob) + initial record_iteration!
// =============================================================================================
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_init(const DevProblem* __restrict__ P, DevBuffers Bf, int mode) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  TrajState s = {};
  s.active = 1;
  s.J = INFINITY;
  traj_rollout_open<M, INTEG>(P, Bf, b);
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  double* C = Bf.C + (size_t)b * N * pmax;
  if (mode == TOG_MODE_AL) {
    for (int i = 0; i < N * pmax; i++) {
      Bf.lam[(size_t)b * N * pmax + i] = 0.0;
      Bf.mu[(size_t)b * N * pmax + i] = P->o.penalty_initial;
    }
    (void)traj_cost<M>(P, Bf, b, X, U, true, C);
    s.c_max = traj_max_violation(P, Bf, b);
    s.mu_max = P->o.penalty_initial;
    s.al_iter = 1;
  }
  set_tolerances(P, s, mode);
  s.J = traj_cost<M>(P, Bf, b, X, U, mode == TOG_MODE_AL, mode == TOG_MODE_AL ? C : nullptr);
  s.iters = 1;  // record_iteration!(…, J_prev, Inf)
  s.dJ = INFINITY;
  s.zero_cnt = 0;
  s.grad = INFINITY;
  if (Bf.hist_in) {
    // the AL solver's initial record (augmented_lagrangian_methods.jl:13, iterations_inner 0 of a reset
    // solver), then the inner solver's (ilqr_methods.jl:20): its gradient is calculate_gradient at the
    // initial trajectory with the solver's current d (zero for a new handle)
    if (mode == TOG_MODE_AL) hist_outer(Bf, b, s, 0, s.J, s.c_max, s.mu_max);
    hist_inner(Bf, b, s, s.J, INFINITY, traj_gradient<M>(P, Bf, b, mode == TOG_MODE_AL));
  }
  Bf.st[b] = s;
}

template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_rollout_open(const DevProblem* __restrict__ P, DevBuffers Bf) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  traj_rollout_open<M, INTEG>(P, Bf, b);
}

template <class M>
__global__ void __launch_bounds__(64) k_cost(const DevProblem* __restrict__ P, DevBuffers Bf, int al, int use_bar,
                                             double* Jout) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  constexpr int n = M::n, m = M::m;
  const int N = P->N;
  const double* X = (use_bar ? Bf.Xb : Bf.X) + (size_t)b * N * n;
  const double* U = (use_bar ? Bf.Ub : Bf.U) + (size_t)b * (N - 1) * m;
  Jout[b] = traj_cost<M>(P, Bf, b, X, U, al != 0, al ? Bf.C + (size_t)b * N * P->pmax : nullptr);
}

template <class M>
__global__ void __launch_bounds__(64) k_update_constraints(const DevProblem* __restrict__ P, DevBuffers Bf) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  for (int k = 0; k < N; k++) {
    const int cnt = knot_count(P, k);
    const cptr<ConRow> rows = knot_rows(P, k);
    for (int i = 0; i < cnt; i++)
      Bf.C[((size_t)b * N + k) * pmax + i] =
          row_value_m<M>(uniform_row(load_row(rows + i)), X + (size_t)k * n, k < N - 1 ? U + (size_t)k * m : nullptr);
  }
}

template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_rollout(const DevProblem* __restrict__ P, DevBuffers Bf, double alpha,
                                                int* ok) {
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  ok[b] = traj_rollout<M, INTEG>(P, Bf, b, alpha) ? 1 : 0;
}

// =============================================================================================
// k_jacobian: ∇F[k] = ∂f_d/∂[x;u] by forward-mode duals, one thread per (traj, knot, chunk)
// src/model.jl:491-512 (ForwardDiff.jacobian! of fd_aug!); the dt column is never consumed by
// iLQR (backward_pass.jl:30,110) and is not materialised.
// =============================================================================================
template <class M, int INTEG, int W>
#ifndef TOG_JAC_WAVES
#define TOG_JAC_WAVES 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TOG_JAC_WAVES)))
k_jacobian(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  // an infeasible model (ModelTraits<M>::slack) differentiates its base model only; its slack
  // columns are the identity (src/model.jl:771-774)
  using Mb = typename ModelTraits<M>::Base;
  constexpr int n = M::n, m = M::m, L = n + m, mb = Mb::m, Lb = n + mb, NCH = (Lb + W - 1) / W;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int N = P->N;
  const int c = (int)(t % NCH);
  const long long bk = t / NCH;
  const int k = (int)(bk % (N - 1));
  const long long b = traj_of_slot(Bf, bk / (N - 1), P->B);
  if (b < 0 || !Bf.st[b].active || Bf.st[b].ls_pend) return;
  const double* x = Bf.X + ((size_t)b * N + k) * n;
  const double* u = Bf.U + ((size_t)b * (N - 1) + k) * m;
  Dual<W> xd[n], ud[mb], xn[n];
#pragma unroll
  for (int i = 0; i < n; i++) {
    xd[i].v = x[i];
#pragma unroll
    for (int w = 0; w < W; w++) xd[i].g[w] = (i == c * W + w) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int i = 0; i < mb; i++) {
    ud[i].v = u[i];
#pragma unroll
    for (int w = 0; w < W; w++) ud[i].g[w] = (n + i == c * W + w) ? 1.0 : 0.0;
  }
  discrete_step<Mb, INTEG>(xn, xd, ud, P->dt);
  double* out = Bf.AB + ((size_t)b * (N - 1) + k) * n * L;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int col = c * W + w;
    if (col < Lb) {
#pragma unroll
      for (int i = 0; i < n; i++) out[i + n * col] = xn[i].g[w];
    }
  }
  if constexpr (ModelTraits<M>::slack > 0) {
    for (int j = c; j < n; j += NCH)
#pragma unroll
      for (int i = 0; i < n; i++) out[i + n * (Lb + j)] = (i == j) ? 1.0 : 0.0;
  }
}

// Staged RK3 Jacobian for the RBD model (config 5). One dual partial per lane through the RK3 step keeps
// the stage state (x, s, t: 3n duals) live across three RNEA + CRBA + Cholesky evaluations; with it the
// lane needs ~750 doubles and spills 4 KB (68 GB of scratch traffic per launch). Here each
// RK3 stage is its own launch: the stage's f runs with only its inputs live, and the running sum s and
// the next stage input t (2n duals per lane, element-major so lanes coalesce) go through HBM in between.
// The operations and their order are discrete_step's RK3 (src/integration.jl:149-158), so the Jacobian
// is bit-identical to k_jacobian's.
#ifndef TOG_JAC_STAGE_W
#define TOG_JAC_STAGE_W 1
#endif
template <class M, int STAGE, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TOG_JAC_WAVES)))
k_jacobian_rk3_stage(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  using Mb = typename ModelTraits<M>::Base;
  constexpr int n = M::n, m = M::m, L = n + m, mb = Mb::m, Lb = n + mb, NCH = (Lb + W - 1) / W;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int N = P->N;
  const int c = (int)(t % NCH);
  const long long bk = t / NCH;
  const int k = (int)(bk % (N - 1));
  const long long b = traj_of_slot(Bf, bk / (N - 1), P->B);
  if (b < 0 || !Bf.st[b].active || Bf.st[b].ls_pend) return;
  const double* x = Bf.X + ((size_t)b * N + k) * n;
  const double* u = Bf.U + ((size_t)b * (N - 1) + k) * m;
  const double dt = P->dt;
  Dual<W> xd[n], ud[mb], kk[n], sv[n], tv[n];
#pragma unroll
  for (int i = 0; i < n; i++) {
    xd[i].v = x[i];
#pragma unroll
    for (int w = 0; w < W; w++) xd[i].g[w] = (i == c * W + w) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int i = 0; i < mb; i++) {
    ud[i].v = u[i];
#pragma unroll
    for (int w = 0; w < W; w++) ud[i].g[w] = (n + i == c * W + w) ? 1.0 : 0.0;
  }
  Dual<W>* ws = reinterpret_cast<Dual<W>*>(Bf.jws);  // element e of lane t at ws[e * total + t]
  if constexpr (STAGE == 0) {
    Mb::f(kk, xd, ud);
#pragma unroll
    for (int i = 0; i < n; i++) {
      kk[i] = kk[i] * dt;
      ws[(size_t)i * total + t] = kk[i];                  // s = k1
      ws[(size_t)(n + i) * total + t] = xd[i] + kk[i] / 2.0;  // t = x + k1/2
    }
  } else {
#pragma unroll
    for (int i = 0; i < n; i++) tv[i] = ws[(size_t)(n + i) * total + t];
    Mb::f(kk, tv, ud);
    // the running sum is read after f, so it is not live (and spilled) across it
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < n; i++) sv[i] = ws[(size_t)i * total + t];
    if constexpr (STAGE == 1) {
#pragma unroll
      for (int i = 0; i < n; i++) {
        kk[i] = kk[i] * dt;
        ws[(size_t)(n + i) * total + t] = (xd[i] - sv[i]) + 2.0 * kk[i];  // t = (x - k1) + 2k2
        ws[(size_t)i * total + t] = sv[i] + 4.0 * kk[i];                  // s = k1 + 4k2
      }
    } else {
      double* out = Bf.AB + ((size_t)b * (N - 1) + k) * n * L;
#pragma unroll
      for (int i = 0; i < n; i++) {
        kk[i] = kk[i] * dt;
        const Dual<W> xn = xd[i] + div6_(sv[i] + kk[i]);
#pragma unroll
        for (int w = 0; w < W; w++)
          if (c * W + w < Lb) out[i + n * (c * W + w)] = xn.g[w];
      }
      if constexpr (ModelTraits<M>::slack > 0) {
        for (int j = c; j < n; j += NCH)
#pragma unroll
          for (int i = 0; i < n; i++) out[i + n * (Lb + j)] = (i == j) ? 1.0 : 0.0;
      }
    }
  }
}

// Minimum-time model (add_min_time_controls, src/solvers/altro/minimum_time.jl:91-96): the base
// model's ForwardDiff Jacobian over [x; u; dt] at dt = h² (partial c of the chunk, dt the last one),
// placed at the augmented columns; the dt column times 2h becomes the h column, and row τ+ = h has a 1
// there. The τ column and the other entries of row τ are zero.
// With an infeasible model inside (MinTime<Infeasible<Mb>>) the differentiated model is Mb (ModelTraits::Core):
// its columns [x; u; dt], the slack columns the identity (src/model.jl:771-774), h the last control.
template <class M, int INTEG, int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TOG_JAC_WAVES)))
k_jacobian_mt(const DevProblem* __restrict__ P, DevBuffers Bf, long long total) {
  using Mb = typename ModelTraits<M>::Core;
  constexpr int n = M::n, m = M::m, L = n + m, nb = Mb::n, mb = Mb::m, Lz = nb + mb + 1, NCH = (Lz + W - 1) / W;
  constexpr int SL = ModelTraits<M>::slack;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int N = P->N;
  const int c = (int)(t % NCH);
  const long long bk = t / NCH;
  const int k = (int)(bk % (N - 1));
  const long long b = traj_of_slot(Bf, bk / (N - 1), P->B);
  if (b < 0 || !Bf.st[b].active || Bf.st[b].ls_pend) return;
  const double* x = Bf.X + ((size_t)b * N + k) * n;
  const double* u = Bf.U + ((size_t)b * (N - 1) + k) * m;
  const double h = u[m - 1];
  Dual<W> xd[nb], ud[mb], xn[nb + 1], dtd;
#pragma unroll
  for (int i = 0; i < nb; i++) {
    xd[i].v = x[i];
#pragma unroll
    for (int w = 0; w < W; w++) xd[i].g[w] = (i == c * W + w) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int i = 0; i < mb; i++) {
    ud[i].v = u[i];
#pragma unroll
    for (int w = 0; w < W; w++) ud[i].g[w] = (nb + i == c * W + w) ? 1.0 : 0.0;
  }
  dtd.v = h * h;
#pragma unroll
  for (int w = 0; w < W; w++) dtd.g[w] = (nb + mb == c * W + w) ? 1.0 : 0.0;
  discrete_step<Mb, INTEG, Dual<W>, Dual<W>>(xn, xd, ud, dtd);
  double* out = Bf.AB + ((size_t)b * (N - 1) + k) * n * L;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int col = c * W + w;
    if (col < nb) {  // x column
#pragma unroll
      for (int i = 0; i < nb; i++) out[i + n * col] = xn[i].g[w];
      out[nb + n * col] = 0.0;
    } else if (col < nb + mb) {  // u column
#pragma unroll
      for (int i = 0; i < nb; i++) out[i + n * (n + col - nb)] = xn[i].g[w];
      out[nb + n * (n + col - nb)] = 0.0;
    } else if (col == nb + mb) {  // h column: (∂f/∂dt) .* (2h); τ+ = h
#pragma unroll
      for (int i = 0; i < nb; i++) out[i + n * (n + m - 1)] = xn[i].g[w] * (2.0 * h);
      out[nb + n * (n + m - 1)] = 1.0;
    }
  }
  if (c == 0) {
#pragma unroll
    for (int i = 0; i < n; i++) out[i + n * nb] = 0.0;  // τ column
    if constexpr (SL > 0) {  // slack columns: Diagonal(1.0I, n) (row τ zero)
#pragma unroll
      for (int j = 0; j < SL; j++)
#pragma unroll
        for (int i = 0; i < n; i++) out[i + n * (n + mb + j)] = (i == j) ? 1.0 : 0.0;
    }
  }
}

}  // namespace tog
#include "tog_kuka_jac.hpp"
namespace tog {

// =============================================================================================
// Wave-level small dense linear algebra on LDS (column-major). All 64 lanes cooperate; sizes are
// compile-time so every loop unrolls. Callers synchronise (wsync) between dependent steps.
// =============================================================================================

// C (R x Cc) [+]= op(A) * op(B);  op(A) is R x Kd, op(B) is Kd x Cc
#ifdef TOG_MFMA
// A/B variant (DESIGN.md §5 "MFMA"): the product on the fp64 matrix cores, v_mfma_f64_16x16x4_f64, in
// 16 x 16 output tiles, 4-deep k steps, operands straight from LDS (A[i][k]: lane i + 16 k, B[k][j]:
// lane j + 16 k; D: col = lane & 15, row = (lane >> 4) + 4 reg). The matrix core's accumulation order
// is not the oracle's fma chain, so this build is not bit-identical to the oracle.
typedef double tog_d4 __attribute__((ext_vector_type(4)));
template <int R, int Kd, int Cc, bool TA, bool TB, bool ACC>
__device__ __forceinline__ void wmm(double* C, const double* A, int lda, const double* B, int ldb) {
  const int lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int ti = 0; ti < (R + 15) / 16; ti++) {
#pragma unroll
    for (int tj = 0; tj < (Cc + 15) / 16; tj++) {
      tog_d4 acc = {0.0, 0.0, 0.0, 0.0};
      const int i = 16 * ti + lr, j = 16 * tj + lr;
#pragma unroll
      for (int k0 = 0; k0 < Kd; k0 += 4) {
        const int l = k0 + lk;
        const double a = (i < R && l < Kd) ? (TA ? A[l + lda * i] : A[i + lda * l]) : 0.0;
        const double bb = (j < Cc && l < Kd) ? (TB ? B[j + ldb * l] : B[l + ldb * j]) : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = 16 * ti + lk + 4 * r, col = 16 * tj + lr;
        if (row < R && col < Cc) C[row + R * col] = ACC ? C[row + R * col] + acc[r] : acc[r];
      }
    }
  }
}
#else
template <int R, int Kd, int Cc, bool TA, bool TB, bool ACC>
__device__ __forceinline__ void wmm(double* C, const double* A, int lda, const double* B, int ldb) {
  for (int e = threadIdx.x; e < R * Cc; e += WAVE) {
    const int i = e % R, j = e / R;
    double s = 0.0;
#pragma unroll
    for (int l = 0; l < Kd; l++) {
      const double a = TA ? A[l + lda * i] : A[i + lda * l];
      const double bb = TB ? B[j + ldb * l] : B[l + ldb * j];
      s = fma(a, bb, s);
    }
    C[i + R * j] = ACC ? C[i + R * j] + s : s;
  }
}
#endif

// Householder QR of the rows x cols matrix A (ld = rows) in place; R ends up in the upper
// triangle of the top cols rows (LAPACK dgeqr2/dlarfg; Julia qr(P).R, backward_pass.jl:172-183).
// wv: LDS scratch >= cols. All lanes participate.
template <int COLS>
__device__ void wqr(double* A, int rows, double* wv) {
  const int lane = threadIdx.x;
  const int kmax = rows < COLS ? rows : COLS;
  for (int j = 0; j < kmax; j++) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // contract v2: 4 interleaved accumulators (oracle qr_R)
    for (int i = j + 1; i < rows; i++) {
      const double a = A[i + rows * j];
      acc[(i - j - 1) & 3] = fma(a, a, acc[(i - j - 1) & 3]);
    }
    const double ss = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (ss == 0.0) continue;  // tau = 0, H = I (uniform branch: every lane computed ss)
    const double alpha = A[j + rows * j];
    const double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
    // contract v3 (oracle qr_R): unnormalised reflector v = [α-β; x], H y = y + v (v'y)/(β(α-β))
    const double vd = alpha - beta;
    const double rd = 1.0 / (beta * vd);
    wsync();
    if (lane > j && lane < COLS) {
      const int c = lane;
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int i = j + 1; i < rows; i++) a4[(i - j - 1) & 3] = fma(A[i + rows * j], A[i + rows * c], a4[(i - j - 1) & 3]);
      const double p = fma(vd, A[j + rows * c], (a4[0] + a4[1]) + (a4[2] + a4[3])) * rd;
      A[j + rows * c] = fma(vd, p, A[j + rows * c]);
      wv[c] = p;
    }
    wsync();
    const int nc = COLS - j - 1, nr = rows - j - 1;
    for (int e = lane; e < nc * nr; e += WAVE) {
      const int i = j + 1 + e % nr, c = j + 1 + e / nr;
      A[i + rows * c] = fma(A[i + rows * j], wv[c], A[i + rows * c]);
    }
    if (lane == 0) A[j + rows * j] = beta;
    wsync();
  }
}

// =============================================================================================
// k_backward: cost expansion + Riccati backward pass, one wave per trajectory
// =============================================================================================
template <class M, bool SQRT>
struct BwdLds {
  static constexpr int n = M::n, m = M::m, L = n + m;
  static constexpr int PC = pcap_of<M>();
  static constexpr int WR = n + (n > PC ? n : PC);  // QR workspace rows ([Q.xx; Iμ cx])
  // QR workspace: [Q.xx; √Iμ cx] (WR x n) and [Q.uu; √Iμ cu] ((m + PC) x m; larger when m > n)
  static constexpr int WQ = WR * n > (m + PC) * m ? WR * n : (m + PC) * m;
  double S[n * n];
  double s[n];
  double AB[n * L];
  double Qxx[n * n];
  double Quu[m * m];
  double Qux[m * n];
  double Qx[n];
  double Qu[m];
  double T1[n * L];
  double Kt[m * n];
  double dd[m];
  double F[m * m];     // LU / Cholesky factor of Quu_reg, or its R factor (sqrt)
  double KtQ[n * m];
  double tmp1[n * m];
  double tmp2[m * m];
  double Wq[WQ];       // QR workspace
  double xk[n];
  double uk[m];
  double cval[PC], wv[PC], wsv[PC], gv[PC];
  double cx[PC * n];
  double cu[PC * m];
  static constexpr int RW = (PC + 63) / 64;
  unsigned long long rmask[(n + m) * RW];  // per variable: the rows whose gradient entry is nonzero
  unsigned long long rbad[RW];             // rows with a non-finite gradient entry or weight: always chained
  double red[WAVE];
  // lane-0 serial scratch (kept in LDS: private arrays with runtime indexing spill to scratch memory)
  double G[m * m];
  double Uc[m * m];
  double Wl[(m + n) * m];
  double Ri[m * m];
  double Aj[m * m];
  double vv[m];
  double mtx[n], mtu[m];  // unscaled Qx, Qu of a minimum-time model's MinTimeCost expansion
  int piv[m];
  int flag;
  int pad;
};

// stage / terminal expansion into the Q blocks (cost.jl:183-198, objective.jl:51-94, AL terms
// augmented_lagrangian_methods.jl:186-276). u == nullptr marks the terminal knot.
template <class M, bool SQRT, bool AL>
__device__ void bwd_expand(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, int k,
                           BwdLds<M, SQRT>& sh) {
  constexpr int n = M::n, m = M::m;
  const int lane = threadIdx.x;
  const int N = P->N;
  const bool term = (k == N - 1);
  constexpr bool MT = ModelTraits<M>::min_time;
  // minimum time: dt = τ² with τ = u[end] (MinTimeCost cost_expansion!, minimum_time.jl:155-188)
  const double dt = (MT && !term) ? sh.uk[m - 1] * sh.uk[m - 1] : P->dt;
  if (!term) {
    const CostView C_ = cost_at<n, m>(P, k);
    if (lane < n) {
      const int i = lane;
      double a = 0.0, bb = 0.0;
#pragma unroll
      for (int j = 0; j < n; j++) a = fma(C_.Q[i + n * j], sh.xk[j], a);
#pragma unroll
      for (int j = 0; j < m; j++) bb = fma(C_.H[j + m * i], sh.uk[j], bb);
      const double g = (a + C_.q[i]) + bb;
      sh.Qx[i] = g * dt;
      if (MT) sh.mtx[i] = g;
    } else if (lane < n + m) {
      const int i = lane - n;
      double a = 0.0, bb = 0.0;
#pragma unroll
      for (int j = 0; j < m; j++) a = fma(C_.R[i + m * j], sh.uk[j], a);
#pragma unroll
      for (int j = 0; j < n; j++) bb = fma(C_.H[i + m * j], sh.xk[j], bb);
      const double g = (a + C_.r[i]) + bb;
      sh.Qu[i] = g * dt;
      if (MT) sh.mtu[i] = g;
    }
    for (int e = lane; e < n * n; e += WAVE) sh.Qxx[e] = SQRT ? C_.cQ[e] : C_.Q[e] * dt;
    for (int e = lane; e < m * m; e += WAVE) sh.Quu[e] = SQRT ? C_.cR[e] : C_.R[e] * dt;
    for (int e = lane; e < m * n; e += WAVE) sh.Qux[e] = C_.H[e] * dt;
    if constexpr (MT) {
      // the τ / h entries: ℓ1 = stage_cost(cost, x, u) (no dt), tmp = 2τ Qu
      wsync();
      const double R = P->R_min_time, tau = sh.uk[m - 1];
      const double l1 = stage_cost_dt<n, m>(P, k, sh.xk, sh.uk, 1.0);
      const double w = 2.0 * l1 + R, t2 = 2.0 * tau;
      if (lane < m - 1) {
        const double tmp = t2 * sh.mtu[lane];
        sh.Quu[lane + m * (m - 1)] = tmp;
        sh.Quu[(m - 1) + m * lane] = tmp;
      } else if (lane == m - 1) {
        sh.Qu[m - 1] = tau * w;
        sh.Quu[(m - 1) + m * (m - 1)] = w;
        sh.Qx[n - 1] = R * sh.xk[n - 1];
        sh.Qxx[(n - 1) + n * (n - 1)] = R;
      }
      if (lane >= WAVE - (n - 1)) {
        const int j = lane - (WAVE - (n - 1));
        sh.Qux[(m - 1) + m * j] = t2 * sh.mtx[j];
      }
    }
  } else {
    for (int e = lane; e < n * n; e += WAVE) sh.Qxx[e] = SQRT ? P->cQf[e] : P->Qf[e];
    if (lane < n) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < n; j++) a = fma(P->Qf[lane + n * j], sh.xk[j], a);
      sh.Qx[lane] = a + P->qf[lane];
    }
    if constexpr (MT) {  // S.xx[end,end] = R_min_time, S.x[end] = R_min_time xN[end]
      wsync();
      if (lane == 0) {
        sh.Qxx[(n - 1) + n * (n - 1)] = P->R_min_time;
        sh.Qx[n - 1] = P->R_min_time * sh.xk[n - 1];
      }
    }
  }
  if (!AL) return;
  const int p = P->knot_cnt[k];
  if (p == 0) return;
  const ConRow* rows = P->rows + P->knot_off[k];
  const int pmax = P->pmax;
  const double* lam = Bf.lam + ((size_t)b * N + k) * pmax;
  const double* mu = Bf.mu + ((size_t)b * N + k) * pmax;
  for (int e = lane; e < p * n; e += WAVE) sh.cx[e] = 0.0;
  for (int e = lane; e < p * m; e += WAVE) sh.cu[e] = 0.0;
  if constexpr (!SQRT) {  // the row masks of the std AL chains below, set as the rows are evaluated
    constexpr int RW = BwdLds<M, SQRT>::RW;
    for (int e = lane; e < (n + m) * RW; e += WAVE) sh.rmask[e] = 0ull;
    if (lane < RW) sh.rbad[lane] = 0ull;
  }
  wsync();
  for (int r = lane; r < p; r += WAVE) {  // p may exceed the wave (PCAP > 64)
    const double c = row_value_m<M>(rows[r], sh.xk, term ? nullptr : sh.uk);
    const double l = lam[r];
    const bool a = row_inequality(rows[r]) ? ((c >= 0.0) || (l > 0.0)) : true;
    const double w = a ? mu[r] : 0.0;
    sh.cval[r] = c;
    sh.wv[r] = w;
    sh.wsv[r] = a ? sqrt(mu[r]) : 0.0;
    sh.gv[r] = w * c + l;
    int idx[row_grad_cap<M>()];
    double v[row_grad_cap<M>()];
    const int nz = row_grad_m<M>(rows[r], sh.xk, term ? nullptr : sh.uk, idx, v);
    for (int z = 0; z < nz; z++) {
      if (idx[z] < n)
        sh.cx[r + p * idx[z]] = v[z];
      else
        sh.cu[r + p * (idx[z] - n)] = v[z];
    }
    if constexpr (!SQRT) {  // row r's bit in the masks of the columns its gradient touches (LDS atomics)
      constexpr int RW = BwdLds<M, SQRT>::RW;
      const int wd = r >> 6;
      const unsigned long long bit = 1ull << (r & 63);
      bool bad = !isfinite(w);
      for (int z = 0; z < nz; z++) {
        if (v[z] != 0.0) atomicOr(&sh.rmask[idx[z] * RW + wd], bit);
        bad = bad || !isfinite(v[z]);
      }
      if (bad) atomicOr(&sh.rbad[wd], bit);
    }
  }
  wsync();
  if (!SQRT) {
    // Q.xx .+= cx'Iμ*cx ; Q.uu .+= cu'Iμ*cu ; Q.ux .+= cu'Iμ*cx. Entry (i, j) is the chain over the rows r
    // ascending; a row with a zero gradient entry in column i or j adds an exact zero (fma(0, ., t) = t: t
    // starts at +0 and never becomes -0), so the chain runs over the rows both columns touch (the AND of
    // their row masks) and gives the dense chain's value bit for bit (round 5: the infeasible quadrotor's
    // 69 rows touch 1-3 columns each). A row with a non-finite gradient entry or weight anywhere is chained
    // in every entry (rbad), so a diverging trajectory's Inf/NaN reaches Q exactly as the dense chain's does.
    // (the masks: rmask[v] has row r's bit when the row's gradient entry in column v is nonzero, rbad the rows
    // with a non-finite gradient entry or weight; both set by the row evaluation above)
    constexpr int RW = BwdLds<M, SQRT>::RW;
    auto chain = [&](const double* ci, const double* cj, int vi, int vj) {
      double t = 0.0;
      for (int w = 0; w < RW; w++) {
        unsigned long long mk = (sh.rmask[vi * RW + w] & sh.rmask[vj * RW + w]) | sh.rbad[w];
        while (mk) {
          const int r = 64 * w + __builtin_ctzll(mk);
          mk &= mk - 1;
          t = fma(ci[r] * sh.wv[r], cj[r], t);
        }
      }
      return t;
    };
    for (int e = lane; e < n * n; e += WAVE) {
      const int i = e % n, j = e / n;
      sh.Qxx[e] += chain(sh.cx + p * i, sh.cx + p * j, i, j);
    }
    if (!term) {
      for (int e = lane; e < m * m; e += WAVE) {
        const int i = e % m, j = e / m;
        sh.Quu[e] += chain(sh.cu + p * i, sh.cu + p * j, n + i, n + j);
      }
      for (int e = lane; e < m * n; e += WAVE) {
        const int i = e % m, j = e / m;
        sh.Qux[e] += chain(sh.cu + p * i, sh.cx + p * j, n + i, j);
      }
    }
  } else {
    // chol_plus!(Q.xx, Iμ_sqrt*cx) ; chol_plus!(Q.uu, Iμ_sqrt*cu)   (no ux term, A.5)
    const int rows_x = n + p;
    for (int e = lane; e < rows_x * n; e += WAVE) {
      const int i = e % rows_x, j = e / rows_x;
      sh.Wq[e] = (i < n) ? sh.Qxx[i + n * j] : sh.wsv[i - n] * sh.cx[(i - n) + p * j];
    }
    wsync();
    wqr<n>(sh.Wq, rows_x, sh.red);
    for (int e = lane; e < n * n; e += WAVE) {
      const int i = e % n, j = e / n;
      sh.Qxx[e] = (i <= j) ? sh.Wq[i + rows_x * j] : 0.0;
    }
    wsync();
    if (!term) {
      const int rows_u = m + p;
      for (int e = lane; e < rows_u * m; e += WAVE) {
        const int i = e % rows_u, j = e / rows_u;
        sh.Wq[e] = (i < m) ? sh.Quu[i + m * j] : sh.wsv[i - m] * sh.cu[(i - m) + p * j];
      }
      wsync();
      wqr<m>(sh.Wq, rows_u, sh.red);
      for (int e = lane; e < m * m; e += WAVE) {
        const int i = e % m, j = e / m;
        sh.Quu[e] = (i <= j) ? sh.Wq[i + rows_u * j] : 0.0;
      }
    }
  }
  // Q.x .+= cx'g ; Q.u .+= cu'g
  if (lane < n) {
    double t = 0.0;
    for (int r = 0; r < p; r++) t = fma(sh.cx[r + p * lane], sh.gv[r], t);
    sh.Qx[lane] += t;
  } else if (!term && lane < n + m) {
    const int i = lane - n;
    double t = 0.0;
    for (int r = 0; r < p; r++) t = fma(sh.cu[r + p * i], sh.gv[r], t);
    sh.Qu[i] += t;
  }
}

template <class M, bool SQRT>
__device__ __forceinline__ void bwd_store_q(double* q, BwdLds<M, SQRT>& sh) {
  constexpr int n = M::n, m = M::m;
  for (int e = threadIdx.x; e < nq_of<M>(); e += WAVE) {
    double v;
    if (e < n) v = sh.Qx[e];
    else if (e < n + m) v = sh.Qu[e - n];
    else if (e < n + m + n * n) v = sh.Qxx[e - n - m];
    else if (e < n + m + n * n + m * m) v = sh.Quu[e - n - m - n * n];
    else v = sh.Qux[e - n - m - n * n - m * m];
    q[e] = v;
  }
}
template <class M, bool SQRT>
__device__ __forceinline__ void bwd_load_q(const double* q, BwdLds<M, SQRT>& sh) {
  constexpr int n = M::n, m = M::m;
  for (int e = threadIdx.x; e < nq_of<M>(); e += WAVE) {
    const double v = q[e];
    if (e < n) sh.Qx[e] = v;
    else if (e < n + m) sh.Qu[e - n] = v;
    else if (e < n + m + n * n) sh.Qxx[e - n - m] = v;
    else if (e < n + m + n * n + m * m) sh.Quu[e - n - m - n * n] = v;
    else sh.Qux[e - n - m - n * n - m * m] = v;
  }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// lane L's value of v in every lane (two v_readlane_b32; L a compile-time constant)
template <int L>
__device__ __forceinline__ double lane_read(double v) {
  const long long x = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), L);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), L);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}

// LU with partial pivoting of the m x m matrix F in place (dgetrf; Julia `\`), lane 0 only.
template <int m>
__device__ __forceinline__ void lu_factor(double* F, int* piv) {
  for (int k = 0; k < m; k++) {
    int p = k;
    double amax = fabs(F[k + m * k]);
    for (int i = k + 1; i < m; i++)
      if (fabs(F[i + m * k]) > amax) {
        amax = fabs(F[i + m * k]);
        p = i;
      }
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < m; j++) {
        const double t = F[k + m * j];
        F[k + m * j] = F[p + m * j];
        F[p + m * j] = t;
      }
    const double akk = F[k + m * k];
    if (akk != 0.0) {
      const double r = 1.0 / akk;
      for (int i = k + 1; i < m; i++) F[i + m * k] *= r;
    }
    for (int j = k + 1; j < m; j++)
      for (int i = k + 1; i < m; i++) F[i + m * j] = fma(-F[i + m * k], F[k + m * j], F[i + m * j]);
  }
}
template <int m>
__device__ __forceinline__ void lu_solve_col(const double* F, const int* piv, double* bcol) {
  // (fully unrolled so that bcol lives in registers)
#pragma unroll
  for (int k = 0; k < m; k++) {
    const int p = piv[k];
#pragma unroll
    for (int i = k + 1; i < m; i++)
      if (i == p) {  // compile-time indices only: bcol stays in registers
        const double t = bcol[k];
        bcol[k] = bcol[i];
        bcol[i] = t;
      }
  }
#pragma unroll
  for (int j = 0; j < m; j++)
#pragma unroll
    for (int i = j + 1; i < m; i++) bcol[i] = fma(-F[i + m * j], bcol[j], bcol[i]);
#pragma unroll
  for (int j = m - 1; j >= 0; j--) {
    bcol[j] /= F[j + m * j];
#pragma unroll
    for (int i = 0; i < j; i++) bcol[i] = fma(-F[i + m * j], bcol[j], bcol[i]);
  }
}
// lu_solve_col with the factor in registers: lane c holds column c of F (gcol); F[i][j] reaches every lane by
// v_readlane from lane j. The same operations in the same order as lu_solve_col. Call in uniform control flow.
template <int m>
__device__ __forceinline__ void lu_solve_col_reg(const double (&gcol)[m], const int* piv, double* bcol) {
#pragma unroll
  for (int k = 0; k < m; k++) {
    const int p = piv[k];
#pragma unroll
    for (int i = k + 1; i < m; i++)
      if (i == p) {
        const double t = bcol[k];
        bcol[k] = bcol[i];
        bcol[i] = t;
      }
  }
  static_for<0, m>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
#pragma unroll
    for (int i = j + 1; i < m; i++) bcol[i] = fma(-lane_read<j>(gcol[i]), bcol[j], bcol[i]);
  });
  static_for<0, m>([&](auto jr) {
    constexpr int j = m - 1 - decltype(jr)::value;
    bcol[j] /= lane_read<j>(gcol[j]);
#pragma unroll
    for (int i = 0; i < j; i++) bcol[i] = fma(-lane_read<j>(gcol[i]), bcol[j], bcol[i]);
  });
}

// 2-norm condition number test cond(R) > 1e8 for an upper-triangular m x m R (backward_pass.jl:129).
// Exact decision via Frobenius bounds cond_2 <= ‖R‖_F‖R⁻¹‖_F <= m·cond_2; a one-sided Jacobi SVD
// settles the (rare) ambiguous band. Lane 0 only.
template <int m>
__device__ bool cond_exceeds(const double* Rm, double thresh, double* Ri, double* A) {
  for (int i = 0; i < m * m; i++) Ri[i] = 0.0;
  for (int c = 0; c < m; c++) {
    Ri[c + m * c] = 1.0;
    for (int j = m - 1; j >= 0; j--) {
      const double xj = Ri[j + m * c] / Rm[j + m * j];
      Ri[j + m * c] = xj;
      for (int i = j - 1; i >= 0; i--) Ri[i + m * c] -= Rm[i + m * j] * xj;
    }
  }
  double nr = 0.0, ni = 0.0;
  for (int i = 0; i < m * m; i++) {
    nr += Rm[i] * Rm[i];
    ni += Ri[i] * Ri[i];
  }
  const double cF = sqrt(nr) * sqrt(ni);
  if (cF <= thresh) return false;
  if (cF / m > thresh) return true;
  // ambiguous: one-sided Jacobi singular values
  for (int i = 0; i < m * m; i++) A[i] = Rm[i];
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0.0;
    for (int p = 0; p < m - 1; p++)
      for (int q = p + 1; q < m; q++) {
        double al = 0, be = 0, ga = 0;
        for (int i = 0; i < m; i++) {
          al += A[i + m * p] * A[i + m * p];
          be += A[i + m * q] * A[i + m * q];
          ga += A[i + m * p] * A[i + m * q];
        }
        if (ga == 0.0) continue;
        const double c0 = fabs(ga) / sqrt(al * be);
        off = fmax(off, c0);
        if (c0 < 1e-15) continue;
        const double zeta = (be - al) / (2.0 * ga);
        const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double cs = 1.0 / sqrt(1.0 + t * t), sn = cs * t;
        for (int i = 0; i < m; i++) {
          const double ap = A[i + m * p], aq = A[i + m * q];
          A[i + m * p] = cs * ap - sn * aq;
          A[i + m * q] = sn * ap + cs * aq;
        }
      }
    if (off < 1e-15) break;
  }
  double smax = 0.0, smin = INFINITY;
  for (int j = 0; j < m; j++) {
    double s2 = 0.0;
    for (int i = 0; i < m; i++) s2 += A[i + m * j] * A[i + m * j];
    smax = fmax(smax, sqrt(s2));
    smin = fmin(smin, sqrt(s2));
  }
  return (smax / smin) > thresh;
}

template <class M, int SQRTI, int ALI>
__global__ void __launch_bounds__(64) k_backward(const DevProblem* __restrict__ P, DevBuffers Bf, int flags) {
  constexpr bool SQRT = SQRTI != 0, AL = ALI != 0;
  constexpr int n = M::n, m = M::m, L = n + m, NQ = nq_of<M>();
  // the wave-parallel Quu factorization, the LU's pivot swap and the ΔV terms give lane j column j
  static_assert(m <= WAVE, "k_backward: more controls than lanes in a wave");
  __shared__ BwdLds<M, SQRT> sh;
  const long long b = traj_of_slot(Bf, blockIdx.x, P->B);
  const int lane = threadIdx.x;
  const int N = P->N;
  if (b < 0 || !Bf.st[b].active || Bf.st[b].ls_pend) return;
  RegState s;
  s.rho = Bf.st[b].rho;
  s.drho = Bf.st[b].drho;
  s.flags = Bf.st[b].flags;
  const bool store_S = (flags & TOG_BP_STORE_S) && Bf.Sdbg;
  const double* Xg = Bf.X + (size_t)b * N * n;
  const double* Ug = Bf.U + (size_t)b * (N - 1) * m;
  double* Kg = Bf.K + (size_t)b * (N - 1) * m * n;
  double* dg = Bf.d + (size_t)b * (N - 1) * m;
  const double* ABg = Bf.AB + (size_t)b * (N - 1) * n * L;
  double* Qs = Bf.Qscr + (size_t)b * N * NQ;
  const double rho0 = s.rho, drho0 = s.drho;
  bool faithful = false;  // replay mode that reproduces the A.1 re-accumulation exactly
  int kmin = N - 1;       // lowest knot whose accumulated Q is stored in Qscr
  int restarts = 0;
  double dV0 = 0.0, dV1 = 0.0;
  const bool state_reg = (P->o.bp_reg_type == 1);

attempt:
  dV0 = 0.0;
  dV1 = 0.0;
  // terminal cost-to-go: S[N] = Q[N] (backward_pass.jl:20-21 / :100-101)
  if (lane < n) sh.xk[lane] = Xg[(size_t)(N - 1) * n + lane];
  wsync();
  bwd_expand<M, SQRT, AL>(P, Bf, b, N - 1, sh);
  wsync();
  for (int e = lane; e < n * n; e += WAVE) sh.S[e] = sh.Qxx[e];
  if (lane < n) sh.s[lane] = sh.Qx[lane];
  wsync();
  if (store_S) {
    for (int e = lane; e < n * n; e += WAVE) Bf.Sdbg[((size_t)b * N + (N - 1)) * n * n + e] = sh.S[e];
    if (lane < n) Bf.sdbg[((size_t)b * N + (N - 1)) * n + lane] = sh.s[lane];
  }

  for (int k = N - 2; k >= 0; k--) {
    // ---- load ∇F[k] = [A|B] and (x_k, u_k)
    const double* abk = ABg + (size_t)k * n * L;
    for (int e = lane; e < n * L; e += WAVE) sh.AB[e] = abk[e];
    if (lane < n) sh.xk[lane] = Xg[(size_t)k * n + lane];
    else if (lane < n + m) sh.uk[lane - n] = Ug[(size_t)k * m + lane - n];
    wsync();
    if (faithful && k >= kmin) {
      bwd_load_q<M, SQRT>(Qs + (size_t)k * NQ, sh);
    } else {
      bwd_expand<M, SQRT, AL>(P, Bf, b, k, sh);
    }
    wsync();
    const double* A = sh.AB;
    const double* Bm = sh.AB + n * n;
    // ---- Q.x += A's ; Q.u += B's
    if (lane < n) {
      double t = 0.0;
#pragma unroll
      for (int l = 0; l < n; l++) t = fma(A[l + n * lane], sh.s[l], t);
      sh.Qx[lane] += t;
    } else if (lane < n + m) {
      const int i = lane - n;
      double t = 0.0;
#pragma unroll
      for (int l = 0; l < n; l++) t = fma(Bm[l + n * i], sh.s[l], t);
      sh.Qu[i] += t;
    }
    if (!SQRT) {
      // T1 = [A B]' S (L x n), then Qxx += (A'S)A ; Quu += (B'S)B ; Qux += (B'S)A  (A.16 association,
      // backward_pass.jl:32-36)
      if constexpr (ModelTraits<M>::slack > 0 && !ModelTraits<M>::min_time) {
        // infeasible model, B = [B_m I] (the slack columns' identity, src/model.jl:771-774): the identity's
        // products are copies -- T1's slack rows are S's rows, Quu's slack columns T1's -- each "+ 0.0", which
        // is the dense chain's value bit for bit (its other terms add exact zeros to a +0 start; barring
        // inf/NaN in S). Round 5: 390 of the 900 length-13 chains of the infeasible quadrotor.
        constexpr int ns = ModelTraits<M>::slack, mb = m - ns;
        for (int e = lane; e < L * n; e += WAVE) {
          const int r = e % L, j = e / L;
          double t;
          if (r < n + mb) {
            t = 0.0;
#pragma unroll
            for (int l = 0; l < n; l++) t = fma(sh.AB[l + n * r], sh.S[l + n * j], t);
          } else {
            t = sh.S[(r - n - mb) + n * j] + 0.0;
          }
          sh.T1[e] = t;
        }
        wsync();
        wmm<n, n, n, false, false, true>(sh.Qxx, sh.T1, L, A, n);
        for (int e = lane; e < m * m; e += WAVE) {
          const int i = e % m, j = e / m;
          double t;
          if (j < mb) {
            t = 0.0;
#pragma unroll
            for (int l = 0; l < n; l++) t = fma(sh.T1[(n + i) + L * l], Bm[l + n * j], t);
          } else {
            t = sh.T1[(n + i) + L * (j - mb)] + 0.0;
          }
          sh.Quu[e] = sh.Quu[e] + t;
        }
        wmm<m, n, n, false, false, true>(sh.Qux, sh.T1 + n, L, A, n);
        wsync();
      } else {
        wmm<L, n, n, true, false, false>(sh.T1, sh.AB, n, sh.S, n);
        wsync();
        wmm<n, n, n, false, false, true>(sh.Qxx, sh.T1, L, A, n);
        wmm<m, n, m, false, false, true>(sh.Quu, sh.T1 + n, L, Bm, n);
        wmm<m, n, n, false, false, true>(sh.Qux, sh.T1 + n, L, A, n);
        wsync();
      }
    } else {
      // tmp_x = S*A, tmp_u = S*B ; Q.xx ← qr([Q.xx; tmp_x]).R ; Q.uu ← qr([Q.uu; tmp_u]).R ;
      // Q.ux += tmp_u'tmp_x   (backward_pass.jl:112-118)
      wmm<n, n, L, false, false, false>(sh.T1, sh.S, n, sh.AB, n);
      wsync();
      wmm<m, n, n, true, false, true>(sh.Qux, sh.T1 + n * n, n, sh.T1, n);
      {
        constexpr int rows = 2 * n;
        for (int e = lane; e < rows * n; e += WAVE) {
          const int i = e % rows, j = e / rows;
          sh.Wq[e] = (i < n) ? sh.Qxx[i + n * j] : sh.T1[(i - n) + n * j];
        }
        wsync();
        wqr<n>(sh.Wq, rows, sh.red);
        for (int e = lane; e < n * n; e += WAVE) {
          const int i = e % n, j = e / n;
          sh.Qxx[e] = (i <= j) ? sh.Wq[i + rows * j] : 0.0;
        }
        wsync();
      }
      {
        constexpr int rows = m + n;
        for (int e = lane; e < rows * m; e += WAVE) {
          const int i = e % rows, j = e / rows;
          sh.Wq[e] = (i < m) ? sh.Quu[i + m * j] : sh.T1[(i - m) + n * (n + j)];
        }
        wsync();
        wqr<m>(sh.Wq, rows, sh.red);
        for (int e = lane; e < m * m; e += WAVE) {
          const int i = e % m, j = e / m;
          sh.Quu[e] = (i <= j) ? sh.Wq[i + rows * j] : 0.0;
        }
        wsync();
      }
    }
    if (faithful) {
      bwd_store_q<M, SQRT>(Qs + (size_t)k * NQ, sh);
      kmin = k < kmin ? k : kmin;
    }
    // ---- regularisation (backward_pass.jl:38-48 / :120-126) and the restart test
    double gcol[m];  // (std pass) lane c: column c of Quu_reg's LU factor, kept in registers for the gains
    if (!SQRT) {
      // Quu_reg = Q.uu + ρI (or + ρB'B), isposdef(Hermitian(Quu_reg)) and its LU factor, wave-parallel (round
      // 5; these ran on lane 0 and were most of a knot for m = 17, the infeasible quadrotor): every entry
      // gets the serial restatement's operations in its order -- the Cholesky test's row j entries are
      // independent given rows < j, the LU's right-looking update is one fma per entry and step, and the
      // pivot search and the diagonal recurrence run redundantly (uniformly) in every lane
      double* G = sh.G;
      for (int e = lane; e < m * m; e += WAVE) {
        double g = sh.Quu[e];
        if (!state_reg) {
          if (e % m == e / m) g += s.rho;
        } else {
          const int i = e % m, j = e / m;
          double t = 0.0;
          for (int l = 0; l < n; l++) t = fma(Bm[l + n * i], Bm[l + n * j], t);
          g += s.rho * t;
        }
        G[e] = g;
      }
      wsync();
      // isposdef(Hermitian(Quu_reg)) and the LU, register-resident (round 6): lane c holds column c of G and of
      // the Cholesky test's U in registers; step j's operands from other columns arrive by v_readlane (the step
      // index is a compile-time constant after unrolling), so the 2m steps run without LDS round trips or
      // barriers. Every value keeps the operations and order of the LDS form (and of the oracle): the test's
      // d0 and the LU's pivot scan, reciprocal and scaled column are formed redundantly (uniformly) in every
      // lane from the broadcast column.
      const int cl = lane < m ? lane : 0;
      double ucol[m];
#pragma unroll
      for (int i = 0; i < m; i++) {
        gcol[i] = G[i + m * cl];
        ucol[i] = 0.0;
      }
      bool pd = true;
      static_for<0, m>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if (!pd) return;
        double uj[j > 0 ? j : 1];
#pragma unroll
        for (int l = 0; l < j; l++) uj[l] = lane_read<j>(ucol[l]);
        double d0 = lane_read<j>(gcol[j]);
#pragma unroll
        for (int l = 0; l < j; l++) d0 -= uj[l] * uj[l];
        if (!(d0 > 0.0)) {
          pd = false;
          return;
        }
        const double ujj = sqrt(d0);
        if (lane == j) ucol[j] = ujj;
        if (lane > j && lane < m) {
          double t = gcol[j];
#pragma unroll
          for (int l = 0; l < j; l++) t -= uj[l] * ucol[l];
          ucol[j] = t / ujj;
        }
      });
      if (lane == 0) sh.flag = pd ? 1 : 0;
      if (pd) {  // lu_factor (partial pivoting)
        static_for<0, m>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          double ck[m];
#pragma unroll
          for (int i = 0; i < m; i++) ck[i] = lane_read<k>(gcol[i]);
          int p = k;
          double amax = fabs(ck[k]);
#pragma unroll
          for (int i = k + 1; i < m; i++) {  // the strict-greater scan over i > k, in order
            if (fabs(ck[i]) > amax) {
              amax = fabs(ck[i]);
              p = i;
            }
          }
          if (lane == 0) sh.piv[k] = p;
          if (p != k) {  // rows k and p of every column (p uniform: a select per candidate row)
#pragma unroll
            for (int i = k + 1; i < m; i++) {
              if (i == p) {
                const double t = gcol[k];
                gcol[k] = gcol[i];
                gcol[i] = t;
                const double tc = ck[k];
                ck[k] = ck[i];
                ck[i] = tc;
              }
            }
          }
          const double akk = ck[k];
          if (akk != 0.0) {
            const double r = 1.0 / akk;
#pragma unroll
            for (int i = k + 1; i < m; i++) ck[i] *= r;  // column k below the diagonal, as lane k scales it
            if (lane == k) {
#pragma unroll
              for (int i = k + 1; i < m; i++) gcol[i] = ck[i];
            }
          }
          if (lane > k && lane < m) {
#pragma unroll
            for (int i = k + 1; i < m; i++) gcol[i] = fma(-ck[i], gcol[k], gcol[i]);
          }
        });
        if (lane < m) {
#pragma unroll
          for (int i = 0; i < m; i++) sh.F[i + m * lane] = gcol[i];
        }
      }
    } else {
      if (lane == 0) {
        // Quu_reg = qr([Q.uu; sqrt(ρ)*I]).R  (:control)  or  qr([Q.uu; sqrt(ρ)*B]).R  (:state)
        const int rows = state_reg ? m + n : 2 * m;
        double* Wl = sh.Wl;
        for (int j = 0; j < m; j++)
          for (int i = 0; i < rows; i++) {
            double v;
            if (i < m) v = sh.Quu[i + m * j];
            else if (state_reg) v = sqrt(s.rho) * Bm[(i - m) + n * j];
            else v = (i - m == j) ? sqrt(s.rho) : 0.0;
            Wl[i + rows * j] = v;
          }
        for (int j = 0; j < m; j++) {  // serial Householder (m x m, tiny; contract v2 as qr_R)
          double acc[4] = {0.0, 0.0, 0.0, 0.0};
          for (int i = j + 1; i < rows; i++)
            acc[(i - j - 1) & 3] = fma(Wl[i + rows * j], Wl[i + rows * j], acc[(i - j - 1) & 3]);
          const double ss = (acc[0] + acc[1]) + (acc[2] + acc[3]);
          if (ss == 0.0) continue;
          const double alpha = Wl[j + rows * j];
          const double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
          const double vd = alpha - beta;  // contract v3 (oracle qr_R)
          const double rd = 1.0 / (beta * vd);
          Wl[j + rows * j] = beta;
          for (int c = j + 1; c < m; c++) {
            double a4[4] = {0.0, 0.0, 0.0, 0.0};
            for (int i = j + 1; i < rows; i++)
              a4[(i - j - 1) & 3] = fma(Wl[i + rows * j], Wl[i + rows * c], a4[(i - j - 1) & 3]);
            const double p = fma(vd, Wl[j + rows * c], (a4[0] + a4[1]) + (a4[2] + a4[3])) * rd;
            Wl[j + rows * c] = fma(vd, p, Wl[j + rows * c]);
            for (int i = j + 1; i < rows; i++) Wl[i + rows * c] = fma(Wl[i + rows * j], p, Wl[i + rows * c]);
          }
        }
        for (int j = 0; j < m; j++)
          for (int i = 0; i < m; i++) sh.F[i + m * j] = (i <= j) ? Wl[i + rows * j] : 0.0;
        sh.flag = cond_exceeds<m>(sh.F, 1e8, sh.Ri, sh.Aj) ? 0 : 1;
      }
    }
    wsync();
    if (!sh.flag) {
      // non-PD / ill-conditioned: increase ρ and restart at N-1 (A.1: Q is NOT re-expanded)
      if (!faithful) {
        // first restart: replay this call from its start in faithful mode so that the
        // re-accumulated Q blocks are exactly the reference's (deterministic replay)
        faithful = true;
        s.rho = rho0;
        s.drho = drho0;
        restarts = 0;
        kmin = N - 1;
        wsync();
        goto attempt;
      }
      reg_increase(P, s);
      restarts++;
      if (restarts > TOG_BP_MAX_RESTARTS) {  // restart cap (tog.h): the trajectory stops
        s.flags |= TOG_TRAJ_MAX_REG | TOG_TRAJ_BP_ABORTED;
        break;
      }
      wsync();
      goto attempt;
    }
    // ---- gains: K = -(Quu_reg \ Qux_reg), d = -(Quu_reg \ Q.u)
    // (std pass: every lane runs the substitutions -- lanes past n on a zero column -- so that the LU factor's
    // entries can come from the owning lanes' registers by v_readlane in uniform control flow)
    if (!SQRT || lane <= n) {
      double col[m];
      if (lane < n) {
#pragma unroll
        for (int i = 0; i < m; i++) {
          double v = sh.Qux[i + m * lane];
          if (state_reg) {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < n; l++) t = fma(Bm[l + n * i], A[l + n * lane], t);
            v += s.rho * t;
          }
          col[i] = v;
        }
      } else if (lane == n) {
#pragma unroll
        for (int i = 0; i < m; i++) col[i] = sh.Qu[i];
      } else {
#pragma unroll
        for (int i = 0; i < m; i++) col[i] = 0.0;
      }
      if (!SQRT) {
        lu_solve_col_reg<m>(gcol, sh.piv, col);
      } else {
        // Quu_reg' \ col (forward substitution), then Quu_reg \ (back substitution); contract v2:
        // multiply by the diagonal reciprocals
        double rF[m];
#pragma unroll
        for (int j = 0; j < m; j++) rF[j] = 1.0 / sh.F[j + m * j];
#pragma unroll
        for (int j = 0; j < m; j++) {
          const double xj = col[j] * rF[j];
          col[j] = xj;
#pragma unroll
          for (int i = j + 1; i < m; i++) col[i] = fma(-sh.F[j + m * i], xj, col[i]);
        }
#pragma unroll
        for (int j = m - 1; j >= 0; j--) {
          const double xj = col[j] * rF[j];
          col[j] = xj;
#pragma unroll
          for (int i = j - 1; i >= 0; i--) col[i] = fma(-sh.F[i + m * j], xj, col[i]);
        }
      }
      if (lane < n) {
#pragma unroll
        for (int i = 0; i < m; i++) sh.Kt[i + m * lane] = -1.0 * col[i];
      } else if (lane == n) {
#pragma unroll
        for (int i = 0; i < m; i++) sh.dd[i] = -1.0 * col[i];
      }
    }
    wsync();
    // ---- write K[k], d[k]
    for (int e = lane; e < m * n; e += WAVE) Kg[(size_t)k * m * n + e] = sh.Kt[e];
    if (lane < m) dg[(size_t)k * m + lane] = sh.dd[lane];
    if (!SQRT) {
      // KtQ = K' * Q.uu (n x m)
      wmm<n, m, m, true, false, false>(sh.KtQ, sh.Kt, m, sh.Quu, m);
      wsync();
      // S[k].x = Q.x + (K'Q.uu) d + K' Q.u + Q.ux' d
      if (lane < n) {
        double a = 0.0, bb = 0.0, c = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) {
          a = fma(sh.KtQ[lane + n * l], sh.dd[l], a);
          bb = fma(sh.Kt[l + m * lane], sh.Qu[l], bb);
          c = fma(sh.Qux[l + m * lane], sh.dd[l], c);
        }
        sh.s[lane] = ((sh.Qx[lane] + a) + bb) + c;
      }
      // S[k].xx = Q.xx + (K'Q.uu)K + K'Q.ux + Q.ux'K, symmetrised (into T1 then S)
      for (int e = lane; e < n * n; e += WAVE) {
        const int i = e % n, j = e / n;
        double a = 0.0, bb = 0.0, c = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) {
          a = fma(sh.KtQ[i + n * l], sh.Kt[l + m * j], a);
          bb = fma(sh.Kt[l + m * i], sh.Qux[l + m * j], bb);
          c = fma(sh.Qux[l + m * i], sh.Kt[l + m * j], c);
        }
        sh.T1[e] = ((sh.Qxx[e] + a) + bb) + c;
      }
      wsync();
      for (int e = lane; e < n * n; e += WAVE) {
        const int i = e % n, j = e / n;
        sh.S[e] = 0.5 * (sh.T1[i + n * j] + sh.T1[j + n * i]);
      }
      // ΔV terms: t_j = Σ_i 0.5 d_i Quu[i, j] by lane j, then lane 0's chains over them in order
      if (lane < m) {
        double t = 0.0;
        for (int i = 0; i < m; i++) t = fma(0.5 * sh.dd[i], sh.Quu[i + m * lane], t);
        sh.red[lane] = t;
      }
      wsync();
      if (lane == 0) {
        double a = 0.0, bb = 0.0;
        for (int i = 0; i < m; i++) a = fma(sh.dd[i], sh.Qu[i], a);
        for (int j = 0; j < m; j++) bb = fma(sh.red[j], sh.dd[j], bb);
        dV0 += a;
        dV1 += bb;
      }
      wsync();
    } else {
      // Ud = Q.uu d (m) and KtQ = K'Q.uu' (n x m)
      if (lane < m) {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) t = fma(sh.Quu[lane + m * l], sh.dd[l], t);
        sh.red[lane] = t;
      }
      for (int e = lane; e < n * m; e += WAVE) {
        const int i = e % n, j = e / n;
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) t = fma(sh.Kt[l + m * i], sh.Quu[j + m * l], t);
        sh.KtQ[e] = t;
      }
      // tmp1 = (Q.xx') \ Q.ux'   (n x m; forward substitution with the lower-triangular Q.xx')
      if (lane < m) {
        const int c = lane;
        double col[n];
#pragma unroll
        for (int i = 0; i < n; i++) col[i] = sh.Qux[c + m * i];
        double rq[n];
#pragma unroll
        for (int j = 0; j < n; j++) rq[j] = 1.0 / sh.Qxx[j + n * j];
#pragma unroll
        for (int j = 0; j < n; j++) {
          const double xj = col[j] * rq[j];
          col[j] = xj;
#pragma unroll
          for (int i = j + 1; i < n; i++) col[i] = fma(-sh.Qxx[j + n * i], xj, col[i]);
        }
#pragma unroll
        for (int i = 0; i < n; i++) sh.tmp1[i + n * c] = col[i];
      }
      wsync();
      // S[k].x = Q.x + (K'Q.uu')(Q.uu d) + K'Q.u + Q.ux'd
      if (lane < n) {
        double a = 0.0, bb = 0.0, c = 0.0;
#pragma unroll
        for (int l = 0; l < m; l++) {
          a = fma(sh.KtQ[lane + n * l], sh.red[l], a);
          bb = fma(sh.Kt[l + m * lane], sh.Qu[l], bb);
          c = fma(sh.Qux[l + m * lane], sh.dd[l], c);
        }
        sh.s[lane] = ((sh.Qx[lane] + a) + bb) + c;
      }
      // tmp2 = chol_minus(Q.uu, tmp1): lowrankdowndate! with each row of tmp1 (backward_pass.jl:186-192)
      if (lane == 0) {
        double* U = sh.Uc;
        double* v = sh.vv;
        for (int e = 0; e < m * m; e++) U[e] = sh.Quu[e];
        double rdg[MMAX];  // contract v4 (oracle chol_minus): diagonal reciprocals carried by products
        for (int i = 0; i < m; i++) rdg[i] = 1.0 / U[i + m * i];
        bool okd = true;
        for (int r = 0; r < n && okd; r++) {
          for (int j = 0; j < m; j++) v[j] = sh.tmp1[r + n * j];
          for (int i = 0; i < m; i++) {
            const double Aii = U[i + m * i];
            const double sn = v[i] * rdg[i];
            const double s2 = sn * sn;
            if (s2 > 1.0) {
              okd = false;
              break;
            }
            const double y = 1.0 - s2;
            const double rc = tog_rsqrt(y);
            const double c = tog_rs_c(y, rc);
            U[i + m * i] = c * Aii;
            rdg[i] = rdg[i] * rc;
            for (int j = i + 1; j < m; j++) {
              const double tmp = (U[i + m * j] - sn * v[j]) * rc;
              v[j] = c * v[j] - sn * tmp;
              U[i + m * j] = tmp;
            }
          }
        }
        for (int e = 0; e < m * m; e++) sh.tmp2[e] = U[e];
        // ΔV
        double a = 0.0, bb = 0.0;
        for (int i = 0; i < m; i++) a = fma(sh.dd[i], sh.Qu[i], a);
        for (int i = 0; i < m; i++) bb = fma(sh.red[i], sh.red[i], bb);
        dV0 += a;
        dV1 += 0.5 * bb;
        sh.flag = okd ? 1 : 0;
      }
      wsync();
      if (!sh.flag) {  // lowrankdowndate! throws PosDefException: this trajectory's solve stops
        s.flags |= TOG_TRAJ_SQRT_PD_FAIL | TOG_TRAJ_BP_ABORTED;
        break;
      }
      // S[k].xx = qr([Q.xx + tmp1*K; tmp2*K]).R
      {
        constexpr int rows = n + m;
        for (int e = lane; e < rows * n; e += WAVE) {
          const int i = e % rows, j = e / rows;
          double v = 0.0;
          if (i < n) {
#pragma unroll
            for (int l = 0; l < m; l++) v = fma(sh.tmp1[i + n * l], sh.Kt[l + m * j], v);
            v = sh.Qxx[i + n * j] + v;
          } else {
            const int ii = i - n;
#pragma unroll
            for (int l = 0; l < m; l++) v = fma(sh.tmp2[ii + m * l], sh.Kt[l + m * j], v);
          }
          sh.Wq[e] = v;
        }
        wsync();
        wqr<n>(sh.Wq, rows, sh.red);
        for (int e = lane; e < n * n; e += WAVE) {
          const int i = e % n, j = e / n;
          sh.S[e] = (i <= j) ? sh.Wq[i + rows * j] : 0.0;
        }
        wsync();
      }
    }
    if (store_S) {
      for (int e = lane; e < n * n; e += WAVE) Bf.Sdbg[((size_t)b * N + k) * n * n + e] = sh.S[e];
      if (lane < n) Bf.sdbg[((size_t)b * N + k) * n + lane] = sh.s[lane];
    }
  }
  const bool aborted = (s.flags & TOG_TRAJ_BP_ABORTED) != 0;
  if (!aborted) reg_decrease(P, s);  // regularization_update!(solver, :decrease) (backward_pass.jl:82 / :166)
  if (lane == 0) {
    TrajState& g = Bf.st[b];
    g.rho = s.rho;
    g.drho = s.drho;
    g.flags = s.flags;
    g.dV0 = aborted ? 0.0 : dV0;
    g.dV1 = aborted ? 0.0 : dV1;
    g.bp_restarts = restarts + (faithful ? 1 : 0);
    if (aborted) g.active = 0;  // no forward pass, no bookkeeping: the trajectory is finished
  }
}

// =============================================================================================
// k_forward: forwardpass! + solve! bookkeeping + AL outer update.
//
// The reference's backtracking line search (forward_pass.jl:19-65) tries α = 1, 1/2, 1/4, ... one
// rollout at a time. Trial j always uses α = 2^-j, and whether it is accepted depends only on its own
// rollout (ok_j, J_j) and on the trials before it. So a FTEAM-lane team per trajectory evaluates
// FTEAM trials speculatively in one round (cost only, no writes), lane 0 replays the sequential
// acceptance logic over (ok_j, J_j) in order -- bit-identical decisions -- and the accepted α is
// replayed once more, writing the new trajectory in place. One round covers iterations_linesearch=20.
// =============================================================================================
// Section timers of the knot loop (build with -DTOG_BWD_PROF; read with tog_bwd_prof_read): shader
// clock deltas (s_memtime) summed per wave into SGPR accumulators, flushed once per wave.
#ifdef TOG_BWD_PROF
constexpr int BPROF_N = 32;  // 0-19 the backward kernels, 20-27 the tail rollouts
static __device__ unsigned long long tog_bwd_prof[BPROF_N];
// per-block LDS accumulators (non-returning ds_add_u64: no wait), only the last stamp in SGPRs
#define BPROF_DECL                                             \
  __shared__ unsigned long long bp_lds[BPROF_N];               \
  if (threadIdx.x < BPROF_N) bp_lds[threadIdx.x] = 0ull;       \
  __syncthreads();                                             \
  unsigned long long bp_t = __builtin_amdgcn_s_memtime();
#define BPROF(id)                                                        \
  {                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
    if (threadIdx.x == 0) atomicAdd(&bp_lds[id], t_ - bp_t);             \
    bp_t = t_;                                                           \
  }
#define BPROF_FLUSH                                                      \
  __syncthreads();                                                       \
  if (threadIdx.x < BPROF_N) atomicAdd(&tog_bwd_prof[threadIdx.x], bp_lds[threadIdx.x]);
#else
#define BPROF_DECL
#define BPROF(id) {}
#define BPROF_FLUSH
#endif

// Per-wave section timers (tools/duo_prof.py): shader-clock deltas summed by lane 0 of each wave.
#ifdef TOG_BWD_PROF
#define DPROF(id)                                                        \
  {                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
    if ((threadIdx.x & 63) == 0) atomicAdd(&bp_lds[id], t_ - bp_t);      \
    bp_t = t_;                                                           \
  }
#else
#define DPROF(id) {}
#endif

constexpr int FTEAM = 32;
constexpr int LS_MAX_ROUNDS = 2;  // speculative line-search rounds per forward pass
// ls_count slots: [0] undecided after the first round, [1] inner solves finished (k_al_outer),
// [2] line searches that ran out of trials (k_ls_fallback)
constexpr int LS_COUNT_SLOTS = 4;
#ifndef TOG_LS_FIRST
#define TOG_LS_FIRST 8
#endif
constexpr int LS_FIRST = TOG_LS_FIRST;  // width of the first round

__device__ __forceinline__ void team_sync() {  // one-wave blocks: order LDS traffic within the wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One closed-loop rollout at α (src/rollout.jl:2-23) fused with the cost of the rolled-out
// trajectory (objective.jl:40-48 / AL cost augmented_lagrangian_methods.jl:298-313), summed in the
// oracle's order. WMODE 0: cost only. WMODE 1: also write X̄, Ū. WMODE 2: write the new trajectory in
// place into X, U (the accepted step; old X[k] is read before it is overwritten) and return the
// todorov gradient of the new U (ilqr_methods.jl:122-129). WMODE 3: write the rolled-out trajectory
// into the candidate slot `cw` (knot-major, n+m doubles per knot: x̄_k then ū_k), for k_ls_apply.
// Constraint-row tables of the rollouts: the global ones, or a block's LDS copy (block_row_tables), both
// through generic pointers (the bulk rollout, k_ls_spec, measured 808 µs this way against 1,030 µs with
// the copy read through the local address space or the tables through scalar loads: the flat loads'
// waits cost less there than the serialised per-row LDS / scalar round trips). The tail rollout
// (k_ls_spec_tail), one wave per trajectory with its inputs staged in LDS, reads the rows through the
// constant address space (const_row_tables): a flat load's wait would drain its staging loads.
struct RowTables {
  const ConRow* rows;
  const int* koff;
  const int* kcnt;
};
__device__ __forceinline__ RowTables global_row_tables(const DevProblem* P) {
  return RowTables{P->rows, P->knot_off, P->knot_cnt};
}
template <class RP, class IP>
struct RowTablesT {
  RP rows;
  IP koff;
  IP kcnt;
};
using RowTablesC = RowTablesT<cptr<ConRow>, cptr<int>>;
__device__ __forceinline__ RowTablesC const_row_tables(const DevProblem* P) {
  return RowTablesC{as_const(P->rows), as_const(P->knot_off), as_const(P->knot_cnt)};
}
// LDS bytes of block_row_tables' copy; 0 when it exceeds the budget (the rollouts then use the global tables)
__host__ __device__ constexpr int row_tables_bytes(int nrows, int N) {
  return (int)(sizeof(ConRow) * nrows + sizeof(int) * 2 * N) <= 32 * 1024
             ? (int)(sizeof(ConRow) * nrows + sizeof(int) * 2 * N)
             : 0;
}
// Cooperative copy of the deduplicated row table and per-knot tables into dynamic LDS (all threads of
// the block must call it). Needs row_tables_bytes(P->nrows, P->N) bytes at `lds`.
__device__ __forceinline__ RowTables block_row_tables(const DevProblem* P, void* lds) {
  ConRow* rc = reinterpret_cast<ConRow*>(lds);
  int* ko = reinterpret_cast<int*>(rc + P->nrows);
  int* kc = ko + P->N;
  const double* src = reinterpret_cast<const double*>(P->rows);
  double* dst = reinterpret_cast<double*>(rc);
  for (int e = threadIdx.x; e < P->nrows * (int)(sizeof(ConRow) / 8); e += blockDim.x) dst[e] = src[e];
  for (int e = threadIdx.x; e < P->N; e += blockDim.x) {
    ko[e] = P->knot_off[e];
    kc[e] = P->knot_cnt[e];
  }
  __syncthreads();
  return RowTables{rc, ko, kc};
}

template <class M, int INTEG, int WMODE, int DC = 0, class RT_T = RowTables>
__device__ bool rollout_cost(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, double alpha,
                             bool al, double& Jout, double* grad_out, const RT_T& RT,
                             double* __restrict__ cw = nullptr, int ncp = 0) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  double* X = Bf.X + (size_t)b * N * n;
  double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* K = Bf.K + (size_t)b * (N - 1) * m * n;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  double* Xb = Bf.Xb + (size_t)b * N * n;
  double* Ub = Bf.Ub + (size_t)b * (N - 1) * m;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  const double smax = P->o.max_state_value, umax = P->o.max_control_value;
  double xb[n], xold[n], ub[m], xn[n];
  double J = 0.0, Jc = 0.0, gsum = 0.0;
#pragma unroll
  for (int i = 0; i < n; i++) {
    xb[i] = Bf.x0[(size_t)b * n + i];
    xold[i] = X[i];
    if (WMODE == 1) Xb[i] = xb[i];
    if (WMODE == 2) X[i] = xb[i];
  }
  // Software pipeline: the inputs of the next knot (K, U, d, X and the first RB multipliers) are
  // loaded while the current knot computes, so every knot does not wait for its own HBM round trip.
  // Not for large gain blocks (the Kuka's 7 x 14 K): held across the knot's RBD evaluations they spill.
  constexpr int RB = 8;
  constexpr bool PREF = m * n <= 64;
  double Kp[m * n], up[m], dp[m], xp[n], lp[RB], mp[RB];
  auto prefetch = [&](int k) {  // inputs of the update that produces knot k+1
    const double* Kk = K + (size_t)k * m * n;
#pragma unroll
    for (int e = 0; e < m * n; e++) Kp[e] = Kk[e];
#pragma unroll
    for (int i = 0; i < m; i++) {
      up[i] = U[(size_t)k * m + i];
      dp[i] = d[(size_t)k * m + i];
    }
    if (al) {
      const int cnt = RT.kcnt[k];
#pragma unroll
      for (int q = 0; q < RB; q++) {
        lp[q] = (q < cnt) ? lam[(size_t)k * pmax + q] : 0.0;
        mp[q] = (q < cnt) ? mu[(size_t)k * pmax + q] : 0.0;
      }
    }
  };
  if (PREF) prefetch(0);
  for (int k = 1; k < N; k++) {
    if (!PREF) prefetch(k - 1);
    double Kk[m * n], uk[m], dk[m], lk[RB], mk[RB];
#pragma unroll
    for (int e = 0; e < m * n; e++) Kk[e] = Kp[e];
#pragma unroll
    for (int i = 0; i < m; i++) {
      uk[i] = up[i];
      dk[i] = dp[i];
    }
#pragma unroll
    for (int q = 0; q < RB; q++) {
      lk[q] = lp[q];
      mk[q] = mp[q];
    }
    if (PREF && k < N - 1) prefetch(k);
#pragma unroll
    for (int i = 0; i < n; i++) xp[i] = X[(size_t)k * n + i];  // x_k of the current iterate (next x_old)
#pragma unroll
    for (int i = 0; i < m; i++) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < n; j++) t = fma(Kk[i + m * j], xb[j] - xold[j], t);
      ub[i] = (uk[i] + t) + alpha * dk[i];
    }
    if (WMODE == 1) {
#pragma unroll
      for (int i = 0; i < m; i++) Ub[(size_t)(k - 1) * m + i] = ub[i];
    }
    if (WMODE == 3) {
#pragma unroll
      for (int i = 0; i < m; i++) __builtin_nontemporal_store(ub[i], cw + cand_at(k - 1, i, cand_q<M>(), ncp));
    }
    if (WMODE == 2) {
      double mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < m; i++) {
        U[(size_t)(k - 1) * m + i] = ub[i];
        const double v = fabs(dk[i]) / (fabs(ub[i]) + 1.0);
        if (v > mx || isnan(v)) mx = v;
      }
      gsum += mx;
    }
    // stage cost and AL terms of knot k-1 (x̄_{k-1}, ū_{k-1})
    J += stage_cost_m<M, DC>(P, k - 1, xb, ub);
    if (al) {
      const int cnt = RT.kcnt[k - 1];
      if (cnt) {
        const auto rows = RT.rows + RT.koff[k - 1];
        double lc = 0.0, cIc = 0.0;
#pragma unroll
        for (int q = 0; q < RB; q++) {
          if (q < cnt) {
            const ConRow r = uniform_row(load_row(rows + q));
            const double c = row_value_m<M>(r, xb, ub);
            const double l = lk[q];
            const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(r) ? ((c >= 0.0) || (l > 0.0)) : true;
            const double w = a ? mk[q] : 0.0;
            lc = fma(l, c, lc);
            cIc = fma(c * w, c, cIc);
          }
        }
        if (cnt > RB)
          al_knot_terms<M>(rows + RB, cnt - RB, lam + (size_t)(k - 1) * pmax + RB,
                                               mu + (size_t)(k - 1) * pmax + RB, xb, ub, lc, cIc, nullptr);
        Jc += lc + 0.5 * cIc;
      }
    }
    discrete_step<M, INTEG>(xn, xb, ub, P->dt);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < n; i++) {
      xb[i] = xn[i];
      ok = ok && (fabs(xn[i]) < smax);
    }
#pragma unroll
    for (int i = 0; i < m; i++) ok = ok && (fabs(ub[i]) < umax);
#pragma unroll
    for (int i = 0; i < n; i++) xold[i] = xp[i];
    if (WMODE == 2) {
#pragma unroll
      for (int i = 0; i < n; i++) X[(size_t)k * n + i] = xn[i];
    }
    if (WMODE == 1) {
#pragma unroll
      for (int i = 0; i < n; i++) Xb[(size_t)k * n + i] = xn[i];
    }
    if (WMODE == 3) {
#pragma unroll
      for (int i = 0; i < n; i++) __builtin_nontemporal_store(xn[i], cw + cand_at(k, m + i, cand_q<M>(), ncp));
    }
    if (!ok) return false;
  }
  J += terminal_cost_m<M, DC>(P, xb);
  if (al) {
    const int cnt = RT.kcnt[N - 1];
    if (cnt) {
      const auto rows = RT.rows + RT.koff[N - 1];
      double lc = 0.0, cIc = 0.0;
      al_knot_terms<M>(rows, cnt, lam + (size_t)(N - 1) * pmax, mu + (size_t)(N - 1) * pmax,
                                           xb, nullptr, lc, cIc, nullptr);
      Jc += lc + 0.5 * cIc;
    }
    J = J + Jc;
  }
  Jout = J;
  if (grad_out) *grad_out = gsum / N;
  return true;
}

// solve! bookkeeping after an accepted forward pass (ilqr_methods.jl:21-42) and the AL outer update
// when the inner solve finished (augmented_lagrangian_methods.jl:53-126). One lane per trajectory.
// Inner part: returns true when the AL outer update is due (inner solve finished in AL mode).
__device__ inline bool inner_bookkeeping(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b,
                                         TrajState& s, double J, double grad, int mode) {
  const tog_options& o = P->o;
  const bool al = (mode == TOG_MODE_AL);
  s.total_steps++;
  bool inner_done = false;
  if (J > o.max_cost_value) {  // ilqr_methods.jl:25-28 (@warn, return without copying X̄)
    s.flags |= TOG_TRAJ_COST_BLOWUP;
    inner_done = true;
  } else {
    s.dJ = fabs(J - s.J);
    s.J = J;
    s.iters++;
    s.grad = grad;
    s.zero_cnt = (s.dJ == 0.0) ? s.zero_cnt + 1 : 0;
    hist_inner(Bf, b, s, s.J, s.dJ, s.grad);
    // evaluate_convergence (ilqr_methods.jl:139-162)
    if ((0.0 < s.dJ && s.dJ < s.cost_tol) || s.grad < s.grad_tol || s.iters >= o.iterations ||
        s.zero_cnt > o.dJ_counter_limit) {
      inner_done = true;
      if (s.iters >= o.iterations) s.flags |= TOG_TRAJ_MAX_ITERS;
    }
  }
  if (!inner_done) return false;
  if (!al) {
    s.flags |= TOG_TRAJ_CONVERGED;
    s.active = 0;
    return false;
  }
  return true;
}

// AL outer update after the inner solve (augmented_lagrangian_methods.jl:53-126): cost(prob) to refresh
// C, dual_update!, penalty_update!, max_violation, convergence, and the next outer iteration's reset.
// Jal: cost(prob) at the inner solve's X, U before the multiplier update (:59, the AL record's cost);
// grad_next: calculate_gradient for the next inner solve's initial record (used with histories only).
__device__ inline void al_outer_finish(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, TrajState& s,
                                       double mumax, double c_max, double Jal, double Jnext, double grad_next,
                                       int mode) {
  const tog_options& o = P->o;
  s.mu_max = mumax;
  s.c_max = c_max;
  hist_outer(Bf, b, s, s.iters, Jal, c_max, mumax);
  const bool conv = (o.kickout_max_penalty && mumax == o.penalty_max) || (s.c_max < o.constraint_tolerance);
  if (conv) {
    s.flags |= TOG_TRAJ_AL_CONVERGED;
    s.active = 0;
  } else if (s.al_iter >= o.al_iterations) {
    s.flags |= TOG_TRAJ_AL_MAX_ITERS;
    s.active = 0;
  } else {
    // next outer iteration: reset!(solver_uncon), set_tolerances!, solve! init (rollout is a no-op)
    s.al_iter++;
    set_tolerances(P, s, mode);
    s.rho = 0.0;
    s.drho = 0.0;
    s.J = Jnext;
    s.iters = 1;
    s.dJ = INFINITY;
    s.zero_cnt = 0;
    hist_inner(Bf, b, s, Jnext, INFINITY, grad_next);
  }
}

template <class M>
__device__ void step_bookkeeping(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b, TrajState& s,
                                 double J, bool copied, double grad, int mode) {
  (void)copied;
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  const tog_options& o = P->o;
  if (!inner_bookkeeping(P, Bf, b, s, J, grad, mode)) return;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  double* C = Bf.C + (size_t)b * N * pmax;
  double* lam = Bf.lam + (size_t)b * N * pmax;
  double* mu = Bf.mu + (size_t)b * N * pmax;
  const double Jal = traj_cost<M>(P, Bf, b, X, U, true, C);  // J = cost(prob): updates C
  double mumax = 0.0;
  for (int k = 0; k < N; k++) {
    const int cnt = knot_count(P, k);
    const cptr<ConRow> rows = knot_rows(P, k);
    for (int i = 0; i < cnt; i++) {
      const size_t q = (size_t)k * pmax + i;
      double l = lam[q] + mu[q] * C[q];  // dual_update! (:107-118)
      l = tog_jlmax(o.dual_min, tog_jlmin(o.dual_max, l));
      if (row_inequality(load_row(rows + i))) l = tog_jlmax(0.0, l);
      lam[q] = l;
      mu[q] = fmax(0.0, fmin(o.penalty_max, o.penalty_scaling * mu[q]));  // penalty_update! (:121-126)
      mumax = fmax(mumax, mu[q]);
    }
  }
  const double c_max = traj_max_violation(P, Bf, b);
  const bool conv = (o.kickout_max_penalty && mumax == o.penalty_max) || (c_max < o.constraint_tolerance);
  const bool next = !(conv || s.al_iter >= o.al_iterations);
  const double Jnext = next ? traj_cost<M>(P, Bf, b, X, U, true, C) : 0.0;
  const double gnext = (next && Bf.hist_in) ? traj_gradient<M>(P, Bf, b, true) : 0.0;
  al_outer_finish(P, Bf, b, s, mumax, c_max, Jal, Jnext, gnext, mode);
}

// Does the sequential acceptance logic of forwardpass! (forward_pass.jl:19-65) settle within the
// first `hi` speculative trials? (Same loop as k_ls_commit, reading the stored trial results.)
__device__ __forceinline__ bool ls_decided_within(const tog_options& o, const DevBuffers& Bf, long long b, int NC,
                                                  double J_prev, double dV0, double dV1, int hi) {
  double J = INFINITY, z = -1.0;
  for (int jj = 0;; jj++) {
    if (!((z <= o.line_search_lower_bound || z > o.line_search_upper_bound) && J >= J_prev)) return true;
    if (jj > o.iterations_linesearch) return true;
    if (jj >= hi) return false;
    if (!Bf.lsok[b * NC + jj]) continue;
    const double aj = ldexp(1.0, -jj);
    J = Bf.lsJ[b * NC + jj];
    const double expected = -aj * (dV0 + aj * dV1);
    z = (expected > 0.0) ? (J_prev - J) / expected : -1.0;
  }
}

// speculative trials: one lane per (trajectory, trial j), α_j = 2^-j, cost only. Trials [lo, lo+cnt).
// The first round covers every trajectory; later rounds only the trajectories listed by
// k_ls_compact (list != nullptr, length *count) — the earlier trials did not settle them. Lanes past
// the list's end exit at once, so whole waves retire (the step-level path passes its J_prev through
// Jprev_in).
// LRT: the rows are read from the block's LDS copy of the tables (AL mode, tables within
// row_tables_bytes' budget), else through the constant address space.
template <class M, int INTEG, bool CAND, bool LRT, int DC>
__device__ __forceinline__ void ls_spec_body(const DevProblem* __restrict__ P, const DevBuffers& Bf, int mode, int lo,
                                             int cnt, const int* __restrict__ list, const int* __restrict__ count) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nb = list ? (long long)*count : slot_count(Bf, P->B);
  if ((long long)blockIdx.x * blockDim.x >= nb * cnt) return;  // block past the list: retire at once
  extern __shared__ double spec_lds[];
  auto body = [&](const auto& RT) {
    const int NC = Bf.nc;
    if (t >= nb * cnt) return;
    const long long i = t / cnt;
    const long long b = list ? (long long)list[i] : traj_of_slot(Bf, i, P->B);
    const TrajState& st = Bf.st[b];
    const int j = lo + st.ls_pend + (int)(t % cnt);  // a pending line search continues after its stored trials
    if (!st.active || j >= NC) return;
    double Jj = INFINITY;
    bool ok;
    if constexpr (CAND) {  // every trial keeps its rollout: the accepted one is copied, not replayed
      double* cw = static_cast<double*>(
          __builtin_assume_aligned(Bf.cand + ((size_t)b * P->N * cand_q<M>() * Bf.ncp + j) * 4, 32));
      ok = rollout_cost<M, INTEG, 3, DC>(P, Bf, b, ldexp(1.0, -j), mode == TOG_MODE_AL, Jj, nullptr, RT, cw, Bf.ncp);
    } else {
      ok = rollout_cost<M, INTEG, 0, DC>(P, Bf, b, ldexp(1.0, -j), mode == TOG_MODE_AL, Jj, nullptr, RT);
    }
    Bf.lsJ[b * NC + j] = Jj;
    Bf.lsok[b * NC + j] = ok ? 1 : 0;
  };
  if constexpr (LRT) {
    body(block_row_tables(P, spec_lds));
  } else {
    body(global_row_tables(P));
  }
}
// DC: the cost's structure (stage_cost_dt): 1 when the launch knows the cost is diagonal (x̄, ū then stay
// in registers; the dense loops index them at run time), else 0
template <class M, int INTEG, bool CAND, bool LRT, int DC>
__global__ void __launch_bounds__(256) k_ls_spec(const DevProblem* __restrict__ P, DevBuffers Bf, int mode, int lo,
                                                 int cnt, const int* __restrict__ list, const int* __restrict__ count) {
  ls_spec_body<M, INTEG, CAND, LRT, DC>(P, Bf, mode, lo, cnt, list, count);
}
// The same rollouts for the models whose gain block exceeds 64 entries (the Kuka, its minimum-time and
// infeasible variants, the infeasible quadrotor): one wave per SIMD may hold 512 registers (the
// architectural file plus the accumulation registers as spill space). Their rollouts keep the RBD
// evaluation's per-joint arrays live; at 256 registers they spilled to scratch (1,136 B per lane, round 4
// profile), and their launches are at most a wave per SIMD anyway (B x 8 trials lanes).
template <class M, int INTEG, bool CAND, bool LRT, int DC>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_ls_spec_w1(const DevProblem* __restrict__ P, DevBuffers Bf, int mode, int lo, int cnt, const int* __restrict__ list,
             const int* __restrict__ count) {
  ls_spec_body<M, INTEG, CAND, LRT, DC>(P, Bf, mode, lo, cnt, list, count);
}

// ---------------------------------------------------------------------------------------------
// k_ls_spec_tail: the speculative trials of the convergence tail (few trajectories, every trial in one
// round, candidate slots). One wave per listed trajectory, lane j = trial j. The trials share the
// trajectory's per-knot inputs (K_k, ū_k, d_k, λ_k, μ_k and the x_{k+1} of the current iterate), so the
// wave stages them into LDS a chunk of spec_tail_tc knots at a time: coalesced loads for chunk c+1 are
// issued into registers when chunk c starts and written to LDS when it ends, and the lanes read the
// chunk's knots from LDS (broadcast reads). The serial knot loop then never waits on a global load; the
// per-lane k_ls_spec, whose lanes each prefetch one knot ahead, waited a memory round trip per knot at
// one trajectory per launch (601 µs for 100 knots). Same operations in the same order as rollout_cost
// WMODE 3, so the trial costs, flags and candidate rollouts are bit-identical.
// LDS image of one chunk (doubles, field-major): [K: TC·mn | ū: TC·m | d: TC·m | x: TC·n | λ: TC·p | μ: TC·p].
__host__ __device__ constexpr int spec_tail_tc(int n, int m) { return (m * n <= 64) ? 16 : 8; }
__host__ __device__ constexpr int spec_tail_rec(int n, int m, int pmax) { return m * n + 2 * m + n + 2 * pmax; }
constexpr int SPEC_TAIL_PMAX = 16;  // larger row counts per knot take k_ls_spec

template <class M, int INTEG, int DC>
__global__ void __launch_bounds__(64) k_ls_spec_tail(const DevProblem* __restrict__ P, DevBuffers Bf, int mode,
                                                      int lo, int cnt) {
  constexpr int n = M::n, m = M::m, MN = m * n;
  constexpr int TC = spec_tail_tc(n, m);
  constexpr int SREG = (TC * spec_tail_rec(n, m, SPEC_TAIL_PMAX) + WAVE - 1) / WAVE;  // staged doubles per lane
  const long long b = traj_of_slot(Bf, blockIdx.x, P->B);
  if (b < 0) return;
  const TrajState& st = Bf.st[b];
  const int j = lo + st.ls_pend + (int)threadIdx.x;
  if (!st.active || lo + st.ls_pend >= Bf.nc) return;  // (uniform over the block)
  extern __shared__ double tl[];
  const int lane = threadIdx.x;
  const int N = P->N, pmax = P->pmax, NC = Bf.nc;
  const bool al = (mode == TOG_MODE_AL);
  const int PL = al ? pmax : 0;  // λ, μ are staged in AL mode only
  const int OU = TC * MN, OD = OU + TC * m, OX = OD + TC * m, OL = OX + TC * n, OM = OL + TC * PL, TCR = OM + TC * PL;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* K = Bf.K + (size_t)b * (N - 1) * MN;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  // element e of chunk image starting at step s0 (steps s = k-1 in [0, N-1)); past the chunk's last step
  // the address is clamped into the field (the value is never read)
  auto src = [&](int e, int s0, int ns) -> const double* {
    auto at = [&](const double* base, int sz, int off) {
      const int r = e - off;  // element of this field in the chunk
      return base + (size_t)s0 * sz + (r < ns * sz ? r : 0);
    };
    if (e < OU) return at(K, MN, 0);
    if (e < OD) return at(U, m, OU);
    if (e < OX) return at(d, m, OD);
    if (e < OL) return at(X + n, n, OX);  // x_{s+1}: the next knot's x of the current iterate
    if (e < OM) return at(lam, PL, OL);
    return at(mu, PL, OM);
  };
  double sv[SREG];
  auto stage_load = [&](int s0) {
    const int ns = min(TC, N - 1 - s0);
#pragma unroll
    for (int i = 0; i < SREG; i++) {
      const int e = lane + WAVE * i;
      sv[i] = *src(e < TCR ? e : 0, s0, ns);
    }
  };
  auto stage_store = [&]() {
#pragma unroll
    for (int i = 0; i < SREG; i++) {
      const int e = lane + WAVE * i;
      if (e < TCR) tl[e] = sv[i];
    }
  };
  // the terminal knot's λ, μ (AL mode) sit after the chunk image: [λ_N: p | μ_N: p], loaded with chunk 0
  double tv = 0.0;
  if (al) {
    const int e = lane < 2 * PL ? lane : 0;
    tv = (e < PL) ? lam[(size_t)(N - 1) * pmax + e] : mu[(size_t)(N - 1) * pmax + (e - PL)];
  }
  const bool on = (lane < cnt) && (j < NC);
  double* cw = on ? static_cast<double*>(__builtin_assume_aligned(
                        Bf.cand + ((size_t)b * N * cand_q<M>() * Bf.ncp + j) * 4, 32))
                  : nullptr;
  const int ncp = Bf.ncp;
  const double alpha = ldexp(1.0, -j);
  const double smax = P->o.max_state_value, umax = P->o.max_control_value;
  const RowTablesC RT = const_row_tables(P);
  double xb[n], xold[n], ub[m], xn[n];
  double J = 0.0, Jc = 0.0;
  bool live = on;
#pragma unroll
  for (int i = 0; i < n; i++) {
    xb[i] = Bf.x0[(size_t)b * n + i];
    xold[i] = X[i];
  }
  stage_load(0);
#pragma unroll 1
  for (int s0 = 0; s0 < N - 1; s0 += TC) {
    if (s0 == 0 && lane < 2 * PL) tl[TCR + lane] = tv;
    stage_store();  // chunk s0 (its loads were issued a chunk ago)
    wsync();
    const int ns = min(TC, N - 1 - s0);
    if (s0 + TC < N - 1) stage_load(s0 + TC);
    if (live) {
#pragma unroll 1
      for (int c = 0; c < ns; c++) {
        const int k = s0 + c + 1;  // produces knot k from knot k-1
        const double* Kk = tl + c * MN;
#pragma unroll
        for (int i = 0; i < m; i++) {
          double t = 0.0;
#pragma unroll
          for (int jj = 0; jj < n; jj++) t = fma(Kk[i + m * jj], xb[jj] - xold[jj], t);
          ub[i] = (tl[OU + c * m + i] + t) + alpha * tl[OD + c * m + i];
        }
#pragma unroll
        for (int i = 0; i < m; i++) __builtin_nontemporal_store(ub[i], cw + cand_at(k - 1, i, cand_q<M>(), ncp));
        J += stage_cost_m<M, DC>(P, k - 1, xb, ub);
        if (al) {
          const int pc = RT.kcnt[k - 1];
          if (pc) {
            const auto rows = RT.rows + RT.koff[k - 1];
            double lc = 0.0, cIc = 0.0;
            for (int q = 0; q < pc; q++) {
              const ConRow r = uniform_row(load_row(rows + q));
              const double cv = row_value_m<M, true>(r, xb, ub);
              const double l = tl[OL + c * PL + q];
              const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(r) ? ((cv >= 0.0) || (l > 0.0)) : true;
              const double w = a ? tl[OM + c * PL + q] : 0.0;
              lc = fma(l, cv, lc);
              cIc = fma(cv * w, cv, cIc);
            }
            Jc += lc + 0.5 * cIc;
          }
        }
        discrete_step<M, INTEG>(xn, xb, ub, P->dt);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < n; i++) {
          xb[i] = xn[i];
          ok = ok && (fabs(xn[i]) < smax);
        }
#pragma unroll
        for (int i = 0; i < m; i++) ok = ok && (fabs(ub[i]) < umax);
#pragma unroll
        for (int i = 0; i < n; i++) xold[i] = tl[OX + c * n + i];
#pragma unroll
        for (int i = 0; i < n; i++) __builtin_nontemporal_store(xn[i], cw + cand_at(k, m + i, cand_q<M>(), ncp));
        if (!ok) {
          live = false;
          break;
        }
      }
    }
    wsync();  // every lane is done with the chunk before the next one overwrites it
  }
  if (!on) return;
  double Jj = INFINITY;
  if (live) {
    J += terminal_cost_m<M, DC>(P, xb);
    if (al) {  // terminal rows (al_knot_terms' order), multipliers from LDS
      const int pc = RT.kcnt[N - 1];
      if (pc) {
        const cptr<ConRow> rows = RT.rows + RT.koff[N - 1];
        double lc = 0.0, cIc = 0.0;
        for (int q = 0; q < pc; q++) {
          const ConRow r = uniform_row(load_row(rows + q));
          const double cv = row_value_m<M, true>(r, xb, nullptr);
          const double l = tl[TCR + q];
          const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(r) ? ((cv >= 0.0) || (l > 0.0)) : true;
          const double w = a ? tl[TCR + PL + q] : 0.0;
          lc = fma(l, cv, lc);
          cIc = fma(cv * w, cv, cIc);
        }
        Jc += lc + 0.5 * cIc;
      }
      J = J + Jc;
    }
    Jj = J;
  }
  Bf.lsJ[b * NC + j] = Jj;
  Bf.lsok[b * NC + j] = live ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// k_ls_spec_tail2: k_ls_spec_tail on three waves (at most 32 trials). Wave A runs the dynamics chain
// (ū + K δx + α d, the RK step, the divergence test) and hands each step's (x_s, u_s) to the cost waves
// through an LDS ring of SPEC_RQ steps; one group of steps behind, wave B adds the stage costs, issues the
// candidate stores and stages the next chunk of K, ū, d, x, λ, μ into the other half of a double-buffered
// image, and wave C adds the AL row terms. The two running sums are rollout_cost's own (J over the stage
// costs, Jc over the row terms, J + Jc at the end), each in knot order, so splitting them between waves
// keeps every bit. One workgroup barrier per group of SPEC_RQ steps. (With the rows on wave B as well,
// wave A waited on B for a fifth of the rollout: profiles/r4o_trio_sections_b1.txt.)
constexpr int SPEC_RQ = 4;      // steps per ring slot (and per barrier)
constexpr int SPEC_LANES = 32;  // trials per workgroup
// layout: two staging images (each with the terminal λ, μ after it), the ring, then SPEC_LANES ints of
// wave A's verdicts (live_out), rounded up to whole doubles
__host__ __device__ constexpr int spec_tail2_ring_off(int n, int m, int pmax) {
  return 2 * (spec_tail_tc(n, m) * spec_tail_rec(n, m, pmax) + 2 * pmax);
}
__host__ __device__ constexpr int spec_tail2_doubles(int n, int m, int pmax) {
  return spec_tail2_ring_off(n, m, pmax) + 2 * SPEC_RQ * (n + m) * SPEC_LANES +
         (SPEC_LANES * (int)sizeof(int) + (int)sizeof(double) - 1) / (int)sizeof(double) + SPEC_LANES;
}
static_assert(spec_tail2_doubles(13, 4, 13) - spec_tail2_ring_off(13, 4, 13) - 2 * SPEC_RQ * 17 * SPEC_LANES ==
                  SPEC_LANES / 2 + SPEC_LANES,
              "live_out needs SPEC_LANES ints after the ring, then SPEC_LANES doubles for wave C's Jc");

template <class M, int INTEG, int DC>
__global__ void __launch_bounds__(192) k_ls_spec_tail2(const DevProblem* __restrict__ P, DevBuffers Bf, int mode,
                                                        int lo, int cnt) {
  constexpr int n = M::n, m = M::m, MN = m * n, W = n + m;
  constexpr int TC = spec_tail_tc(n, m);
  static_assert(TC % SPEC_RQ == 0, "a ring group never straddles two staging chunks");
  constexpr int GPC = TC / SPEC_RQ;  // ring groups per staging chunk
  static_assert(GPC >= 2, "the next chunk is stored while the previous one is still read");
  constexpr int SREG = (TC * spec_tail_rec(n, m, SPEC_TAIL_PMAX) + WAVE - 1) / WAVE;
  const long long b = traj_of_slot(Bf, blockIdx.x, P->B);
  if (b < 0) return;
  const TrajState& st = Bf.st[b];
  if (!st.active || lo + st.ls_pend >= Bf.nc) return;  // (uniform over the block)
  extern __shared__ double tl2[];
  BPROF_DECL
  const int wv = threadIdx.x >> 6;  // 0: chain wave A, 1: cost wave B, 2: row wave C
  const int lane = threadIdx.x & (WAVE - 1);
  const int j = lo + st.ls_pend + lane;
  const int N = P->N, pmax = P->pmax, NC = Bf.nc;
  const bool al = (mode == TOG_MODE_AL);
  const int PL = al ? pmax : 0;
  const int OU = TC * MN, OD = OU + TC * m, OX = OD + TC * m, OL = OX + TC * n, OM = OL + TC * PL, TCR = OM + TC * PL;
  const int IMG = TCR + 2 * PL;                 // one staging image, the terminal λ, μ after it
  double* ring = tl2 + 2 * IMG;                 // [slot][step][element][lane]
  int* live_out = reinterpret_cast<int*>(ring + 2 * SPEC_RQ * W * SPEC_LANES);
  double* jc_out = ring + 2 * SPEC_RQ * W * SPEC_LANES + (SPEC_LANES * (int)sizeof(int) + 7) / 8;  // (wave C's Jc)
  // (2 * IMG <= spec_tail2_ring_off(n, m, pmax): PL <= pmax, so live_out[SPEC_LANES) ends inside the
  // spec_tail2_doubles(n, m, pmax) the runtime allocates)
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* K = Bf.K + (size_t)b * (N - 1) * MN;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  auto src = [&](int e, int s0, int ns) -> const double* {
    auto at = [&](const double* base, int sz, int off) {
      const int r = e - off;
      return base + (size_t)s0 * sz + (r < ns * sz ? r : 0);
    };
    if (e < OU) return at(K, MN, 0);
    if (e < OD) return at(U, m, OU);
    if (e < OX) return at(d, m, OD);
    if (e < OL) return at(X + n, n, OX);
    if (e < OM) return at(lam, PL, OL);
    return at(mu, PL, OM);
  };
  double sv[SREG];
  auto stage_load = [&](int s0) {  // (wave B)
    const int ns = min(TC, N - 1 - s0);
#pragma unroll
    for (int i = 0; i < SREG; i++) {
      const int e = lane + WAVE * i;
      sv[i] = *src(e < TCR ? e : 0, s0, ns);
    }
  };
  auto stage_store = [&](double* img) {  // (wave B)
#pragma unroll
    for (int i = 0; i < SREG; i++) {
      const int e = lane + WAVE * i;
      if (e < TCR) img[e] = sv[i];
    }
  };
  const bool on = (lane < cnt) && (j < NC);
  const int NS = N - 1;                          // steps
  const int G = (NS + SPEC_RQ - 1) / SPEC_RQ;    // ring groups
  // chunk 0 and the terminal multipliers (both waves wait at the first barrier)
  if (wv == 1) {
    stage_load(0);
    stage_store(tl2);
    if (al && lane < 2 * PL)
      tl2[TCR + lane] = (lane < PL) ? lam[(size_t)(N - 1) * pmax + lane] : mu[(size_t)(N - 1) * pmax + (lane - PL)];
  }
  __syncthreads();
  if (wv == 0) {
    // ---------------------------------------------------------------- wave A: the dynamics chain
    const double alpha = ldexp(1.0, -j);
    const double smax = P->o.max_state_value, umax = P->o.max_control_value;
    double xb[n], xold[n], ub[m], xn[n];
    bool live = on;
#pragma unroll
    for (int i = 0; i < n; i++) {
      xb[i] = Bf.x0[(size_t)b * n + i];
      xold[i] = X[i];
    }
#pragma unroll 1
    for (int g = 0; g <= G; g++) {
      if (g < G && live) {
        const double* img = tl2 + ((g / GPC) & 1) * IMG;
        double* slot = ring + (size_t)(g & 1) * SPEC_RQ * W * SPEC_LANES;
#pragma unroll 1
        for (int q = 0; q < SPEC_RQ; q++) {
          const int s = g * SPEC_RQ + q;
          if (s >= NS) break;
          const int c = s % TC;
          const double* Kk = img + c * MN;
#pragma unroll
          for (int i = 0; i < m; i++) {
            double t = 0.0;
#pragma unroll
            for (int jj = 0; jj < n; jj++) t = fma(Kk[i + m * jj], xb[jj] - xold[jj], t);
            ub[i] = (img[OU + c * m + i] + t) + alpha * img[OD + c * m + i];
          }
          double* e = slot + (size_t)q * W * SPEC_LANES + lane;
#pragma unroll
          for (int i = 0; i < n; i++) e[i * SPEC_LANES] = xb[i];  // x_s
#pragma unroll
          for (int i = 0; i < m; i++) e[(n + i) * SPEC_LANES] = ub[i];  // u_s
          discrete_step<M, INTEG>(xn, xb, ub, P->dt);
          bool ok = true;
#pragma unroll
          for (int i = 0; i < n; i++) {
            xb[i] = xn[i];
            ok = ok && (fabs(xn[i]) < smax);
          }
#pragma unroll
          for (int i = 0; i < m; i++) ok = ok && (fabs(ub[i]) < umax);
#pragma unroll
          for (int i = 0; i < n; i++) xold[i] = img[OX + c * n + i];
          if (!ok) {
            live = false;
            break;
          }
        }
      }
      DPROF(20);
      __syncthreads();
      DPROF(21);
    }
    // the final state and the verdict for the cost waves (x_{N-1} in ring slot 0, step 0)
    if (lane < SPEC_LANES) {
#pragma unroll
      for (int i = 0; i < n; i++) ring[(size_t)i * SPEC_LANES + lane] = xb[i];
      live_out[lane] = live ? 1 : 0;
    }
    __syncthreads();
    __syncthreads();  // (wave C's Jc to wave B)
  } else if (wv == 1) {
    // ---------------------------------------------------------------- wave B: stage costs, stores, staging
    double* cw = on ? static_cast<double*>(__builtin_assume_aligned(
                          Bf.cand + ((size_t)b * N * cand_q<M>() * Bf.ncp + j) * 4, 32))
                    : nullptr;
    const int ncp = Bf.ncp;
    double J = 0.0;
#pragma unroll 1
    for (int g = 0; g <= G; g++) {
      // staging of the next chunk: loads in the chunk's second group, stores in its last one
      const int cg = g % GPC, ch = g / GPC;
      if (cg == (GPC > 1 ? 1 : 0) && (ch + 1) * TC < NS) stage_load((ch + 1) * TC);
      if (g >= 1 && on) {
        const int gp = g - 1;
        const double* slot = ring + (size_t)(gp & 1) * SPEC_RQ * W * SPEC_LANES;
#pragma unroll 1
        for (int q = 0; q < SPEC_RQ; q++) {
          const int s = gp * SPEC_RQ + q;
          if (s >= NS) break;
          const double* e = slot + (size_t)q * W * SPEC_LANES + lane;
          double x[n], u[m];
#pragma unroll
          for (int i = 0; i < n; i++) x[i] = e[i * SPEC_LANES];
#pragma unroll
          for (int i = 0; i < m; i++) u[i] = e[(n + i) * SPEC_LANES];
#pragma unroll
          for (int i = 0; i < m; i++) __builtin_nontemporal_store(u[i], cw + cand_at(s, i, cand_q<M>(), ncp));
          if (s >= 1) {
#pragma unroll
            for (int i = 0; i < n; i++) __builtin_nontemporal_store(x[i], cw + cand_at(s, m + i, cand_q<M>(), ncp));
          }
          J += stage_cost_m<M, DC>(P, s, x, u);
        }
      }
      DPROF(22);
      if (cg == GPC - 1 && (ch + 1) * TC < NS) stage_store(tl2 + ((ch + 1) & 1) * IMG);
      DPROF(23);
      __syncthreads();
      DPROF(24);
    }
    __syncthreads();  // wave A's final state and verdict
    double x[n];
    bool live = false;
    if (on) {
      live = live_out[lane] != 0;
#pragma unroll
      for (int i = 0; i < n; i++) x[i] = ring[(size_t)i * SPEC_LANES + lane];
#pragma unroll
      for (int i = 0; i < n; i++) __builtin_nontemporal_store(x[i], cw + cand_at(NS, m + i, cand_q<M>(), ncp));
      if (live) J += terminal_cost_m<M, DC>(P, x);
    }
    __syncthreads();  // wave C's Jc
    if (on) {
      double Jj = INFINITY;
      if (live) Jj = al ? J + jc_out[lane] : J;
      Bf.lsJ[b * NC + j] = Jj;
      Bf.lsok[b * NC + j] = live ? 1 : 0;
    }
  } else {
    // ---------------------------------------------------------------- wave C: the AL row terms
    const RowTablesC RT = const_row_tables(P);
    double Jc = 0.0;
    auto row_terms = [&](const cptr<ConRow> rows, int pc, const double* x, const double* u, const double* lp,
                         const double* mp) {
      double lc = 0.0, cIc = 0.0;
      constexpr int RU = 8;  // the first RU rows unrolled (their table loads issue together)
#pragma unroll
      for (int r = 0; r < RU; r++) {
        if (r < pc) {
          const ConRow row = uniform_row(load_row(rows + r));
          const double cv = row_value_m<M, true>(row, x, u);
          const double l = lp[r];
          const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(row) ? ((cv >= 0.0) || (l > 0.0)) : true;
          const double w = a ? mp[r] : 0.0;
          lc = fma(l, cv, lc);
          cIc = fma(cv * w, cv, cIc);
        }
      }
      for (int r = RU; r < pc; r++) {
        const ConRow row = uniform_row(load_row(rows + r));
        const double cv = row_value_m<M, true>(row, x, u);
        const double l = lp[r];
        const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(row) ? ((cv >= 0.0) || (l > 0.0)) : true;
        const double w = a ? mp[r] : 0.0;
        lc = fma(l, cv, lc);
        cIc = fma(cv * w, cv, cIc);
      }
      Jc += lc + 0.5 * cIc;
    };
#pragma unroll 1
    for (int g = 0; g <= G; g++) {
      if (al && g >= 1 && on) {
        const int gp = g - 1;
        const double* img = tl2 + ((gp / GPC) & 1) * IMG;
        const double* slot = ring + (size_t)(gp & 1) * SPEC_RQ * W * SPEC_LANES;
#pragma unroll 1
        for (int q = 0; q < SPEC_RQ; q++) {
          const int s = gp * SPEC_RQ + q;
          if (s >= NS) break;
          const int pc = RT.kcnt[s];
          if (!pc) continue;
          const int c = s % TC;
          const double* e = slot + (size_t)q * W * SPEC_LANES + lane;
          double x[n], u[m];
#pragma unroll
          for (int i = 0; i < n; i++) x[i] = e[i * SPEC_LANES];
#pragma unroll
          for (int i = 0; i < m; i++) u[i] = e[(n + i) * SPEC_LANES];
          row_terms(RT.rows + RT.koff[s], pc, x, u, img + OL + c * PL, img + OM + c * PL);
        }
      }
      __syncthreads();
    }
    __syncthreads();  // wave A's final state and verdict
    if (al && on && live_out[lane] != 0) {  // terminal rows (al_knot_terms' order), multipliers from the image
      const int pc = RT.kcnt[N - 1];
      if (pc) {
        double x[n];
#pragma unroll
        for (int i = 0; i < n; i++) x[i] = ring[(size_t)i * SPEC_LANES + lane];
        row_terms(RT.rows + RT.koff[N - 1], pc, x, nullptr, tl2 + TCR, tl2 + TCR + PL);
      }
      jc_out[lane] = Jc;
    }
    __syncthreads();
  }
  BPROF_FLUSH
}

// After trials [0, hi): list the active trajectories the acceptance logic has not settled yet
// (input: every trajectory when in_list == nullptr, else in_list[0, *in_count)). One thread per
// entry; a wave reserves its slots with one atomic (ballot + popcount). The list order varies from
// run to run, the per-trajectory results do not. (Templated on the model only to give every model's
// translation unit its own instance.)
template <class M>
__global__ void __launch_bounds__(256) k_ls_compact(const DevProblem* __restrict__ P, DevBuffers Bf, int hi,
                                                    int bookkeeping, const double* __restrict__ Jprev_in,
                                                    const int* __restrict__ in_list, const int* __restrict__ in_count,
                                                    int* __restrict__ out_list, int* __restrict__ out_count) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nb = in_list ? (long long)*in_count : slot_count(Bf, P->B);
  bool und = false;
  long long b = 0;
  if (t < nb) {
    b = in_list ? (long long)in_list[t] : traj_of_slot(Bf, t, P->B);
    const TrajState& st = Bf.st[b];
    und = st.active && !ls_decided_within(P->o, Bf, b, Bf.nc, bookkeeping ? st.J : Jprev_in[b], st.dV0, st.dV1, hi);
  }
  const unsigned long long mask = __ballot(und);
  if (mask == 0) return;
  const int lane = threadIdx.x & (WAVE - 1);
  const int leader = __ffsll((long long)mask) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(out_count, __popcll(mask));
  base = __shfl(base, leader);
  if (und) out_list[base + __popcll(mask & ((1ull << lane) - 1))] = (int)b;
}

// decision (sequential acceptance logic replayed over the speculative trials, forward_pass.jl:19-65),
// commit (in-place replay of the accepted α, or the max-iterations fallback) and bookkeeping.
// One thread per trajectory.
// phase 0: every active trajectory. phase 1: only those the trials [0, hi) settle (ls_decided_within);
// phase 2: only the listed ones (k_ls_compact's list after trials [0, hi)). Phases 1 and 2 partition
// the active trajectories, so phase 1 can run on a second stream while the second speculative round
// evaluates the listed trajectories.
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_ls_commit(const DevProblem* __restrict__ P, DevBuffers Bf, int mode,
                                                  int bookkeeping, const double* Jprev_in, double* Jout, int phase,
                                                  int hi, const int* __restrict__ list, const int* __restrict__ count) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nb = (phase == 2) ? (long long)*count : slot_count(Bf, P->B);
  if ((long long)blockIdx.x * blockDim.x >= nb) return;  // whole block past the list: retire early
  extern __shared__ double rt_lds[];
  const RowTables RT =
      (mode == TOG_MODE_AL && Bf.rows_lds > 0) ? block_row_tables(P, rt_lds) : global_row_tables(P);
  if (t >= nb) return;
  const long long b = (phase == 2) ? (long long)list[t] : traj_of_slot(Bf, t, P->B);
  if (!Bf.st[b].active) return;
  if (phase == 1 && !ls_decided_within(P->o, Bf, b, Bf.nc, bookkeeping ? Bf.st[b].J : Jprev_in[b], Bf.st[b].dV0,
                                       Bf.st[b].dV1, hi))
    return;
  constexpr int n = M::n, m = M::m;
  const tog_options& o = P->o;
  const bool al = (mode == TOG_MODE_AL);
  const int N = P->N, NC = Bf.nc;
  TrajState s = Bf.st[b];
  const double J_prev = bookkeeping ? s.J : Jprev_in[b];
  double J = INFINITY, z = -1.0, expected = 0.0, alpha_last = 0.0;
  int trials = 0, state = 0;
  for (int jj = 0;; jj++) {
    if (!((z <= o.line_search_lower_bound || z > o.line_search_upper_bound) && J >= J_prev)) {
      state = 1;
      break;
    }
    if (jj > o.iterations_linesearch) {
      state = 2;
      break;
    }
    trials++;
    const double aj = ldexp(1.0, -jj);
    bool ok;
    double Jj;
    if (jj < NC) {
      ok = Bf.lsok[b * NC + jj] != 0;
      Jj = Bf.lsJ[b * NC + jj];
    } else {  // beyond the speculative window (iterations_linesearch >= 64): evaluate in place
      ok = rollout_cost<M, INTEG, 0>(P, Bf, b, aj, al, Jj, nullptr, RT);
    }
    if (!ok) continue;
    J = Jj;
    expected = -aj * (s.dV0 + aj * s.dV1);
    z = (expected > 0.0) ? (J_prev - J) / expected : -1.0;
    alpha_last = aj;
  }
  double grad = 0.0;
  bool copied = false;
  if (state == 2) {
    // max line-search iterations: X̄ = X, J = cost(X̄), ρ↑ and ρ += bp_reg_fp (forward_pass.jl:22-37)
    const double* X = Bf.X + (size_t)b * N * n;
    const double* U = Bf.U + (size_t)b * (N - 1) * m;
    if (!bookkeeping) {
      double* Xb = Bf.Xb + (size_t)b * N * n;
      double* Ub = Bf.Ub + (size_t)b * (N - 1) * m;
      for (int i = 0; i < N * n; i++) Xb[i] = X[i];
      for (int i = 0; i < (N - 1) * m; i++) Ub[i] = U[i];
    }
    J = traj_cost<M>(P, Bf, b, X, U, al, al ? Bf.C + (size_t)b * N * P->pmax : nullptr);
    z = 0.0;
    expected = 0.0;
    alpha_last = 0.0;
    reg_increase(P, s);
    s.rho += o.bp_reg_fp;
    grad = traj_gradient<M>(P, Bf, b, al);
    copied = true;
  } else if (!bookkeeping) {
    double Jw;
    rollout_cost<M, INTEG, 1>(P, Bf, b, alpha_last, al, Jw, nullptr, RT);  // writes X̄, Ū
  } else if (!(J > o.max_cost_value)) {
    double Jw;
    rollout_cost<M, INTEG, 2>(P, Bf, b, alpha_last, al, Jw, &grad, RT);  // X, U <- X̄, Ū in place
    copied = true;
  }
  // the rollout sums the todorov terms; the other gradient types need the new X, U (or d) whole
  if (bookkeeping && copied && state != 2 && o.gradient_type != 0) grad = traj_gradient<M>(P, Bf, b, al);
  s.alpha = alpha_last;
  s.z = z;
  s.expected = expected;
  s.ls_trials = trials;
  if (J > J_prev) s.flags |= TOG_TRAJ_COST_INCREASED;
  if (Jout) Jout[b] = J;
  if (bookkeeping) {
    if (s.flags & TOG_TRAJ_COST_INCREASED) {
      s.active = 0;  // reference: error("Cost increased during Forward Pass")
    } else {
      step_bookkeeping<M>(P, Bf, b, s, J, copied, grad, mode);
    }
  }
  Bf.st[b] = s;
}


// ---------------------------------------------------------------------------------------------
// Candidate-copy line search (DevBuffers::cand != nullptr). The speculative trials keep their
// rollouts (k_ls_spec<CAND>), so the accepted trajectory is copied instead of replayed:
//   k_ls_decide  forwardpass!'s sequential acceptance loop over the stored trials (forward_pass.jl:
//                19-65), one lane per trajectory; the ones trials [0, hi) do not settle are listed
//                for the next round;
//   k_ls_apply   winner's X̄, Ū -> X, U (or X̄, Ū at step level), one lane per element, plus the
//                per-knot todorov gradient terms (ilqr_methods.jl:122-129);
//   k_ls_book    J, flags, gradient sum and solve! / AL bookkeeping (ilqr_methods.jl:21-42,
//                augmented_lagrangian_methods.jl:53-126), one lane per trajectory.
// Decisions, trajectories and sums are those of k_ls_commit bit for bit: the copy holds exactly the
// values its replay recomputes, and the gradient terms are summed in the replay's knot order.
// ls_win: accepted trial j >= 0; -2: max line-search iterations (X̄ = X fallback); -3: accepted with
// no evaluated trial (J_prev NaN), replayed at α = 0 by k_ls_book.
template <class M>
__global__ void __launch_bounds__(256) k_ls_decide(const DevProblem* __restrict__ P, DevBuffers Bf, int hi,
                                                   int bookkeeping, const double* __restrict__ Jprev_in,
                                                   const int* __restrict__ in_list, const int* __restrict__ in_count,
                                                   int* __restrict__ out_list, int* __restrict__ out_count, int pend) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nb = in_list ? (long long)*in_count : slot_count(Bf, P->B);
  bool und = false;
  long long b = 0;
  if (t < nb) {
    b = in_list ? (long long)in_list[t] : traj_of_slot(Bf, t, P->B);
    TrajState* st = Bf.st + b;
    if (st->active) {
      const tog_options& o = P->o;
      const int NC = Bf.nc;
      const double J_prev = bookkeeping ? st->J : Jprev_in[b];
      const double dV0 = st->dV0, dV1 = st->dV1;
      if (pend) hi = (st->ls_pend + hi < NC) ? st->ls_pend + hi : NC;  // trials stored so far
      double J = INFINITY, z = -1.0, expected = 0.0, alpha_last = 0.0;
      int trials = 0, state = 0, win = -1;
      for (int jj = 0;; jj++) {
        if (!((z <= o.line_search_lower_bound || z > o.line_search_upper_bound) && J >= J_prev)) {
          state = 1;
          break;
        }
        if (jj > o.iterations_linesearch) {
          state = 2;
          break;
        }
        if (jj >= hi) break;  // not settled by the trials evaluated so far
        trials++;
        if (!Bf.lsok[b * NC + jj]) continue;
        const double aj = ldexp(1.0, -jj);
        J = Bf.lsJ[b * NC + jj];
        expected = -aj * (dV0 + aj * dV1);
        z = (expected > 0.0) ? (J_prev - J) / expected : -1.0;
        alpha_last = aj;
        win = jj;
      }
      if (state == 0) {
        und = true;
        if (pend) {  // continue in the next batch step (no Jacobians / backward pass for it meanwhile)
          st->ls_pend = hi;
          Bf.ls_win[b] = -9;
        }
      } else {
        st->ls_pend = 0;
        if (state == 2) {  // forward_pass.jl:22-37: z = expected = α = 0, J from cost(X) (k_ls_fallback)
          win = -2;
          z = 0.0;
          expected = 0.0;
          alpha_last = 0.0;
          if (Bf.ls_fb) Bf.ls_fb[atomicAdd(Bf.ls_count + 2, 1)] = (int)b;
        } else if (win < 0) {
          win = -3;
        }
        st->alpha = alpha_last;
        st->z = z;
        st->expected = expected;
        st->ls_trials = trials;
        Bf.ls_win[b] = win;
        Bf.ls_Jw[b] = J;
      }
    }
  }
  if (!out_list || pend) return;
  const unsigned long long mask = __ballot(und);
  if (mask == 0) return;
  const int lane = threadIdx.x & (WAVE - 1);
  const int leader = __ffsll((long long)mask) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(out_count, __popcll(mask));
  base = __shfl(base, leader);
  if (und) out_list[base + __popcll(mask & ((1ull << lane) - 1))] = (int)b;
}

template <class M>
__global__ void __launch_bounds__(256) k_ls_apply(const DevProblem* __restrict__ P, DevBuffers Bf, int bookkeeping) {
  // one lane per (trajectory, knot, quad): reads the winner's 32-byte quad, writes its X / U elements
  constexpr int n = M::n, m = M::m, Q = cand_q<M>();
  const int N = P->N;
  const unsigned per = (unsigned)N * Q;
  const unsigned long long t = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long slot = (long long)(t / per);
  if (slot >= slot_count(Bf, P->B)) return;
  const long long b = traj_of_slot(Bf, slot, P->B);
  const unsigned r = (unsigned)(t - (unsigned long long)slot * per);
  const int k = (int)(r / Q), q = (int)(r - (unsigned)k * Q);
  if (!Bf.st[b].active) return;
  const int w = Bf.ls_win[b];
  if (w < 0) return;
  if (bookkeeping && Bf.ls_Jw[b] > P->o.max_cost_value) return;  // ilqr_methods.jl:25-28: X̄ not copied
  const int ncp = Bf.ncp;
  const double* tb = Bf.cand + (size_t)b * per * ncp * 4;  // trajectory b's candidates
  const double* src = tb + ((size_t)r * ncp + w) * 4;      // quad q of knot k of trial w
  double v[4];
#pragma unroll
  for (int e = 0; e < 4; e++) v[e] = src[e];
  double* Xd = (bookkeeping ? Bf.X : Bf.Xb) + ((size_t)b * N + k) * n;
  double* Ud = (bookkeeping ? Bf.U : Bf.Ub) + ((size_t)b * (N - 1) + k) * m;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int c = 4 * q + e;
    if (c < m) {
      if (k < N - 1) Ud[c] = v[e];
    } else if (c < m + n) {
      Xd[c - m] = (k == 0) ? Bf.x0[(size_t)b * n + c - m] : v[e];
    }
  }
  if (bookkeeping && q == 0 && k < N - 1) {  // max_i |d_i| / (|ū_i| + 1) of knot k (rollout_cost WMODE 2)
    const double* dk = Bf.d + ((size_t)b * (N - 1) + k) * m;
    double mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < m; i++) {
      const double ui = (i < 4) ? v[i] : tb[cand_at(k, i, Q, ncp) + (size_t)w * 4];
      const double vv = fabs(dk[i]) / (fabs(ui) + 1.0);
      if (vv > mx || isnan(vv)) mx = vv;
    }
    Bf.gk[(size_t)b * N + k] = mx;
  }
}

// k_ls_book's replay of an accepted trajectory without an evaluated trial (win -3, J_prev NaN): a serial
// rollout, kept out of line so that the bookkeeping kernel's common path does not carry its registers
template <class M, int INTEG>
__device__ __noinline__ void replay_cost(const DevProblem* __restrict__ P, const DevBuffers& Bf, long long b,
                                         double alpha, bool al, int bookkeeping, double max_cost, double J,
                                         double& grad, bool& copied, const RowTables& RT) {
  double Jw;
  if (!bookkeeping) {
    rollout_cost<M, INTEG, 1>(P, Bf, b, alpha, al, Jw, nullptr, RT);
  } else if (!(J > max_cost)) {
    rollout_cost<M, INTEG, 2>(P, Bf, b, alpha, al, Jw, &grad, RT);
    copied = true;
  }
}

// forwardpass! when every trial failed (forward_pass.jl:22-37): X̄ = X and J = cost(prob.obj, X̄, Ū), which
// also refreshes C (A.10). One wave per trajectory k_ls_decide listed, lanes over knots: per knot the
// constraint values, the stage (terminal) cost, the AL terms λ'c + ½c'Iμc (al_knot_terms' operations) and
// the todorov term max_i |d_i| / (|u_i| + 1) into gk; lane 0 sums the knots in traj_cost's order (stage
// costs, terminal cost, then the AL terms), so J is traj_cost's bit for bit. (On one lane per trajectory
// this was a serial 101-knot chain of scattered loads: 50 µs at one trajectory, 0.5 ms at 16-128.)
template <class M>
__global__ void __launch_bounds__(64) k_ls_fallback(const DevProblem* __restrict__ P, DevBuffers Bf, int al,
                                                    const int* __restrict__ list, const int* __restrict__ count) {
  if ((int)blockIdx.x >= *count) return;
  extern __shared__ double fb_lds[];
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  const long long b = list[blockIdx.x];
  const int lane = threadIdx.x;
  double* sk = fb_lds;       // [N] stage / terminal cost of knot k
  double* ak = fb_lds + N;   // [N] AL terms of knot k
  int* hk = reinterpret_cast<int*>(fb_lds + 2 * N);  // [N] knot has rows
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  const double* d = Bf.d + (size_t)b * (N - 1) * m;
  double* C = Bf.C + (size_t)b * N * pmax;
  const double* lam = Bf.lam + (size_t)b * N * pmax;
  const double* mu = Bf.mu + (size_t)b * N * pmax;
  for (int k = lane; k < N; k += WAVE) {
    const double* x = X + (size_t)k * n;
    const double* u = (k < N - 1) ? U + (size_t)k * m : nullptr;
    sk[k] = (k < N - 1) ? stage_cost_m<M>(P, k, x, u) : terminal_cost_m<M>(P, x);
    const int cnt = al ? knot_count(P, k) : 0;
    const cptr<ConRow> rows = knot_rows(P, k);
    double lc = 0.0, cIc = 0.0;
    for (int i = 0; i < cnt; i++) {  // al_knot_terms' operations (rows differ across lanes: no uniform_row)
      const size_t q = (size_t)k * pmax + i;
      const ConRow r = load_row(rows + i);
      const double c = row_value_m<M>(r, x, u);
      const double l = lam[q];
      const bool a = row_inequality<(ModelTraits<M>::slack > 0)>(r) ? ((c >= 0.0) || (l > 0.0)) : true;
      const double w = a ? mu[q] : 0.0;
      lc = fma(l, c, lc);
      cIc = fma(c * w, c, cIc);
      C[q] = c;
    }
    ak[k] = lc + 0.5 * cIc;
    hk[k] = cnt;
    if (k < N - 1) {
      double mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < m; i++) {
        const double v = fabs(d[(size_t)k * m + i]) / (fabs(u[i]) + 1.0);
        if (v > mx || isnan(v)) mx = v;
      }
      Bf.gk[(size_t)b * N + k] = mx;
    }
  }
  __syncthreads();
  if (lane != 0) return;
  double J = 0.0, Jc = 0.0;
  for (int k = 0; k < N - 1; k++) J += sk[k];
  J += sk[N - 1];
  for (int k = 0; k < N; k++)
    if (hk[k]) Jc += ak[k];
  Bf.ls_Jw[b] = al ? J + Jc : J;
}

template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_ls_book(const DevProblem* __restrict__ P, DevBuffers Bf, int mode,
                                                int bookkeeping, const double* Jprev_in, double* Jout) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  extern __shared__ double rt_lds[];
  const RowTables RT =
      (mode == TOG_MODE_AL && Bf.rows_lds > 0) ? block_row_tables(P, rt_lds) : global_row_tables(P);
  if (t >= slot_count(Bf, P->B)) return;
  const long long b = traj_of_slot(Bf, t, P->B);
  if (!Bf.st[b].active) return;
  constexpr int n = M::n, m = M::m;
  const tog_options& o = P->o;
  const bool al = (mode == TOG_MODE_AL);
  const int N = P->N;
  const int win = Bf.ls_win[b];
  if (win == -9) return;  // line search still pending
  TrajState s = Bf.st[b];
  double J = Bf.ls_Jw[b];
  const double J_prev = bookkeeping ? s.J : Jprev_in[b];
  double grad = 0.0;
  bool copied = false;
  if (win == -2) {  // max line-search iterations (forward_pass.jl:22-37), as k_ls_commit
    if (!bookkeeping) {
      const double* X = Bf.X + (size_t)b * N * n;
      const double* U = Bf.U + (size_t)b * (N - 1) * m;
      double* Xb = Bf.Xb + (size_t)b * N * n;
      double* Ub = Bf.Ub + (size_t)b * (N - 1) * m;
      for (int i = 0; i < N * n; i++) Xb[i] = X[i];
      for (int i = 0; i < (N - 1) * m; i++) Ub[i] = U[i];
    }
    // J = cost(X̄ = X) and C(X) from k_ls_fallback (ls_Jw), its todorov terms in gk
    reg_increase(P, s);
    s.rho += o.bp_reg_fp;
    if (o.gradient_type == 0) {
      const double* g = Bf.gk + (size_t)b * N;
      double gsum = 0.0;
      for (int k = 0; k < N - 1; k++) gsum += g[k];
      grad = gsum / N;
    } else {
      grad = traj_gradient<M>(P, Bf, b, al);
    }
    copied = true;
  } else if (win == -3) {
    replay_cost<M, INTEG>(P, Bf, b, s.alpha, al, bookkeeping, o.max_cost_value, J, grad, copied, RT);
  } else if (bookkeeping && !(J > o.max_cost_value)) {
    const double* g = Bf.gk + (size_t)b * N;
    double gsum = 0.0;
    for (int k = 0; k < N - 1; k++) gsum += g[k];
    grad = gsum / N;
    copied = true;
  }
  // apply summed the todorov terms; the other gradient types need the new X, U (or d) whole
  if (bookkeeping && copied && win != -2 && o.gradient_type != 0) grad = traj_gradient<M>(P, Bf, b, al);
  if (J > J_prev) s.flags |= TOG_TRAJ_COST_INCREASED;
  if (Jout) Jout[b] = J;
  (void)copied;
  if (bookkeeping) {
    if (s.flags & TOG_TRAJ_COST_INCREASED) {
      s.active = 0;  // reference: error("Cost increased during Forward Pass")
    } else if (inner_bookkeeping(P, Bf, b, s, J, grad, mode)) {
      // the AL outer update runs wave-parallel over the knots in k_al_outer
      Bf.ls_done[atomicAdd(Bf.ls_count + 1, 1)] = (int)b;
    }
  }
  Bf.st[b] = s;
}

// AL outer update (augmented_lagrangian_methods.jl:53-126) of the trajectories k_ls_book listed, one
// wave per trajectory, lanes over knots. Per knot: C (update_constraints!, the side effect of
// cost(prob)), dual_update! and penalty_update! of its rows, the max_violation and μ_max partials,
// and the knot's stage cost and AL terms at the updated multipliers (the next outer iteration's J).
// The knot terms are summed by lane 0 in traj_cost's order, so J is bit-identical to the serial
// update's; the maxima are order-independent (NaN-propagating max).
template <class M>
__global__ void __launch_bounds__(64) k_al_outer(const DevProblem* __restrict__ P, DevBuffers Bf, int mode,
                                                 const int* __restrict__ list, const int* __restrict__ count) {
  if ((int)blockIdx.x >= *count) return;
  extern __shared__ double alo_lds[];
  constexpr int n = M::n, m = M::m;
  constexpr bool SL = ModelTraits<M>::slack > 0;
  const int N = P->N, pmax = P->pmax;
  const tog_options& o = P->o;
  const long long b = list[blockIdx.x];
  const int lane = threadIdx.x;
  double* sk = alo_lds;       // [N] stage / terminal cost of knot k
  double* ak = alo_lds + N;   // [N] λ'c + ½c'Iμc of knot k (NaN-free flag in hk)
  int* hk = reinterpret_cast<int*>(alo_lds + 2 * N);  // [N] knot has rows
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  double* C = Bf.C + (size_t)b * N * pmax;
  double* lam = Bf.lam + (size_t)b * N * pmax;
  double* mu = Bf.mu + (size_t)b * N * pmax;
  double mumax = 0.0, cmax = 0.0;
  for (int k = lane; k < N; k += WAVE) {
    const double* x = X + (size_t)k * n;
    const double* u = (k < N - 1) ? U + (size_t)k * m : nullptr;
    sk[k] = (k < N - 1) ? stage_cost_m<M>(P, k, x, u) : terminal_cost_m<M>(P, x);
    const int cnt = knot_count(P, k);
    const cptr<ConRow> rows = knot_rows(P, k);
    double lc = 0.0, cIc = 0.0, e = 0.0, im = -INFINITY;
    int ni = 0;
    for (int i = 0; i < cnt; i++) {
      const size_t q = (size_t)k * pmax + i;
      const ConRow r = load_row(rows + i);
      const double c = row_value_m<M>(r, x, u);
      C[q] = c;
      const bool ineq = row_inequality<SL>(r);
      double l = lam[q] + mu[q] * c;  // dual_update! (:107-118)
      l = tog_jlmax(o.dual_min, tog_jlmin(o.dual_max, l));
      if (ineq) l = tog_jlmax(0.0, l);
      const double mn = fmax(0.0, fmin(o.penalty_max, o.penalty_scaling * mu[q]));  // penalty_update! (:121-126)
      lam[q] = l;
      mu[q] = mn;
      mumax = fmax(mumax, mn);
      if (ineq) {  // max_violation (:171-184)
        ni++;
        im = tog_jlmax(im, c);
      } else {
        e = tog_jlmax(e, fabs(c));
      }
      const bool a = ineq ? ((c >= 0.0) || (l > 0.0)) : true;  // active set at the new multipliers
      const double w = a ? mn : 0.0;
      lc = fma(l, c, lc);
      cIc = fma(c * w, c, cIc);
    }
    if (cnt) {
      cmax = tog_jlmax(e, cmax);
      if (ni > 0) cmax = tog_jlmax(tog_jlmax(0.0, im), cmax);
    }
    ak[k] = lc + 0.5 * cIc;
    hk[k] = cnt;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    mumax = fmax(mumax, __shfl_xor(mumax, off));
    cmax = tog_jlmax(cmax, __shfl_xor(cmax, off));
  }
  __syncthreads();
  if (lane != 0) return;
  TrajState s = Bf.st[b];
  const bool conv = (o.kickout_max_penalty && mumax == o.penalty_max) || (cmax < o.constraint_tolerance);
  double Jnext = 0.0;
  if (!conv && s.al_iter < o.al_iterations) {  // traj_cost's order: stage terms, terminal, then AL terms
    double J = 0.0, Jc = 0.0;
    for (int k = 0; k < N - 1; k++) J += sk[k];
    J += sk[N - 1];
    for (int k = 0; k < N; k++)
      if (hk[k]) Jc += ak[k];
    Jnext = J + Jc;
  }
  // the AL record's cost(prob) is the inner solve's last J: the same objective at the same X, U and
  // multipliers, summed in the same order (rollout_cost / traj_cost)
  const double gnext = (Bf.hist_in && !conv && s.al_iter < o.al_iterations) ? traj_gradient<M>(P, Bf, b, true) : 0.0;
  al_outer_finish(P, Bf, b, s, mumax, cmax, s.J, Jnext, gnext, mode);
  Bf.st[b] = s;
}

// =============================================================================================
// Per-model launch table
// =============================================================================================
}  // namespace tog
#include "tog_bwd_team.hpp"
#include "tog_bwd_quad.hpp"
#include "tog_pn.hpp"
namespace tog {

// slack_controls(prob) (src/solvers/altro/infeasible.jl:63-80), one thread per trajectory:
// x_1 = x0; x_{k+1} = f_d(x_k, u_k) on the base model; s_k = X_{k+1} - x_{k+1}; x_{k+1} += s_k.
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_slack_controls(const DevProblem* __restrict__ P, DevBuffers Bf) {
  using Mb = typename ModelTraits<M>::Base;
  constexpr int n = M::n, m = M::m;
  const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P->B) return;
  const int N = P->N;
  const double* X = Bf.X + (size_t)b * N * n;
  double* U = Bf.U + (size_t)b * (N - 1) * m;
  double x[n], xn[n];
#pragma unroll
  for (int i = 0; i < n; i++) x[i] = Bf.x0[(size_t)b * n + i];
  for (int k = 0; k < N - 1; k++) {
    double* u = U + (size_t)k * m;
    discrete_step<Mb, INTEG>(xn, x, u, P->dt);
#pragma unroll
    for (int i = 0; i < n; i++) {
      const double sl = X[(size_t)(k + 1) * n + i] - xn[i];
      u[Mb::m + i] = sl;
      x[i] = xn[i] + sl;
    }
  }
}

// =============================================================================================
// k_cost_expansion: cost_expansion!(prob, solver) on its own (the backward kernels fuse it knot by
// knot), one thread per (trajectory, knot) into Q (nq, N, B) = [Q.x; Q.u; Q.xx; Q.uu; Q.ux].
// ilqr_methods.jl:55-62 -> objective.jl:51-94, cost.jl:183-198; AL terms
// augmented_lagrangian_methods.jl:186-276 with the constraint values last evaluated (A.10).
// Same operation order as oc_cost_expansion (oracle/tog_oracle.c). Inspection path: the dense
// per-thread row Jacobians and QR workspace live in scratch memory.
// =============================================================================================
__device__ inline bool dev_chol_upper(double* U, const double* A, int n) {  // dpotrf 'U', A read-only
  for (int i = 0; i < n * n; i++) U[i] = 0.0;
  for (int j = 0; j < n; j++) {
    double s = A[j + n * j];
    for (int k = 0; k < j; k++) s -= U[k + n * j] * U[k + n * j];
    if (!(s > 0.0)) return false;
    const double ujj = sqrt(s);
    U[j + n * j] = ujj;
    for (int c = j + 1; c < n; c++) {
      double t = A[j + n * c];
      for (int k = 0; k < j; k++) t -= U[k + n * j] * U[k + n * c];
      U[j + n * c] = t / ujj;
    }
  }
  return true;
}

// R (cols x cols) of qr(Pm) for Pm (rows x cols), LAPACK dgeqr2/dlarfg as oracle qr_R
__device__ inline void dev_qr_R(double* R, double* Pm, int rows, int cols) {
  const int kmax = rows < cols ? rows : cols;
  for (int j = 0; j < kmax; j++) {
    const double alpha = Pm[j + rows * j];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // contract v2 (oracle qr_R)
    for (int i = j + 1; i < rows; i++) acc[(i - j - 1) & 3] = fma(Pm[i + rows * j], Pm[i + rows * j], acc[(i - j - 1) & 3]);
    const double ss = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    if (ss == 0.0) continue;
    const double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
    const double vd = alpha - beta;  // contract v3 (oracle qr_R)
    const double rd = 1.0 / (beta * vd);
    Pm[j + rows * j] = beta;
    for (int c = j + 1; c < cols; c++) {
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int i = j + 1; i < rows; i++) a4[(i - j - 1) & 3] = fma(Pm[i + rows * j], Pm[i + rows * c], a4[(i - j - 1) & 3]);
      const double p = fma(vd, Pm[j + rows * c], (a4[0] + a4[1]) + (a4[2] + a4[3])) * rd;
      Pm[j + rows * c] = fma(vd, p, Pm[j + rows * c]);
      for (int i = j + 1; i < rows; i++) Pm[i + rows * c] = fma(Pm[i + rows * j], p, Pm[i + rows * c]);
    }
  }
  for (int j = 0; j < cols; j++)
    for (int i = 0; i < cols; i++) R[i + cols * j] = (i <= j && i < rows) ? Pm[i + rows * j] : 0.0;
}

template <class M>
__global__ void __launch_bounds__(64) k_cost_expansion(const DevProblem* __restrict__ P, DevBuffers Bf, int sq,
                                                       int al, int* fail) {
  constexpr int n = M::n, m = M::m, NQ = nq_of<M>(), PC = pcap_of<M>(), W = n > m ? n : m;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int N = P->N;
  if (t >= P->B * (long long)N) return;
  const int k = (int)(t % N);
  const long long b = t / N;
  const bool term = (k == N - 1);
  double* q = Bf.Qscr + ((size_t)b * N + k) * NQ;
  double* Qx = q;
  double* Qu = q + n;
  double* Qxx = q + n + m;
  double* Quu = Qxx + n * n;
  double* Qux = Quu + m * m;
  for (int i = 0; i < NQ; i++) q[i] = 0.0;
  const double* x = Bf.X + ((size_t)b * N + k) * n;
  const double* u = term ? nullptr : Bf.U + ((size_t)b * (N - 1) + k) * m;
  const double dt = P->dt;
  if (!term) {  // cost.jl:183-198
    const CostView C_ = cost_at<n, m>(P, k);
    for (int i = 0; i < n; i++) {
      double a = 0.0, c = 0.0;
      for (int j = 0; j < n; j++) a = fma(C_.Q[i + n * j], x[j], a);
      for (int j = 0; j < m; j++) c = fma(C_.H[j + m * i], u[j], c);
      Qx[i] = ((a + C_.q[i]) + c) * dt;
    }
    for (int i = 0; i < m; i++) {
      double a = 0.0, c = 0.0;
      for (int j = 0; j < m; j++) a = fma(C_.R[i + m * j], u[j], a);
      for (int j = 0; j < n; j++) c = fma(C_.H[i + m * j], x[j], c);
      Qu[i] = ((a + C_.r[i]) + c) * dt;
    }
    for (int i = 0; i < n * n; i++) Qxx[i] = C_.Q[i] * dt;
    for (int i = 0; i < m * m; i++) Quu[i] = C_.R[i] * dt;
    for (int i = 0; i < m * n; i++) Qux[i] = C_.H[i] * dt;
  } else {
    for (int i = 0; i < n * n; i++) Qxx[i] = P->Qf[i];
    for (int i = 0; i < n; i++) {
      double a = 0.0;
      for (int j = 0; j < n; j++) a = fma(P->Qf[i + n * j], x[j], a);
      Qx[i] = a + P->qf[i];
    }
  }
  double Wk[(W + PC) * W];  // Cholesky / QR workspace
  if (sq) {  // objective.jl:70-86
    if (!dev_chol_upper(Wk, Qxx, n)) { fail[b] = 1; return; }
    for (int i = 0; i < n * n; i++) Qxx[i] = Wk[i];
    if (!term) {
      if (!dev_chol_upper(Wk, Quu, m)) { fail[b] = 1; return; }
      for (int i = 0; i < m * m; i++) Quu[i] = Wk[i];
    }
  }
  const int p = P->knot_cnt[k];
  if (!al || p == 0) return;
  const ConRow* rows = P->rows + P->knot_off[k];
  const int pmax = P->pmax;
  const double* c = Bf.C + ((size_t)b * N + k) * pmax;
  const double* lam = Bf.lam + ((size_t)b * N + k) * pmax;
  const double* mu = Bf.mu + ((size_t)b * N + k) * pmax;
  double cx[PC * n], cu[PC * m], w[PC], ws[PC], g[PC];
  for (int i = 0; i < p * n; i++) cx[i] = 0.0;
  for (int i = 0; i < p * m; i++) cu[i] = 0.0;
  for (int r = 0; r < p; r++) {
    const ConRow row = rows[r];
    int idx[row_grad_cap<M>()];
    double v[row_grad_cap<M>()];
    const int nz = row_grad_m<M>(row, x, u, idx, v);
    for (int z = 0; z < nz; z++) {
      if (idx[z] < n) cx[r + p * idx[z]] = v[z];
      else if (!term) cu[r + p * (idx[z] - n)] = v[z];
    }
    const bool a = row_inequality(row) ? ((c[r] >= 0.0) || (lam[r] > 0.0)) : true;
    w[r] = a ? mu[r] : 0.0;
    ws[r] = a ? sqrt(mu[r]) : 0.0;
    g[r] = w[r] * c[r] + lam[r];
  }
  if (!sq) {
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++) {
        double s = 0.0;
        for (int r = 0; r < p; r++) s = fma(cx[r + p * i] * w[r], cx[r + p * j], s);
        Qxx[i + n * j] += s;
      }
    if (!term) {
      for (int j = 0; j < m; j++)
        for (int i = 0; i < m; i++) {
          double s = 0.0;
          for (int r = 0; r < p; r++) s = fma(cu[r + p * i] * w[r], cu[r + p * j], s);
          Quu[i + m * j] += s;
        }
      for (int j = 0; j < n; j++)
        for (int i = 0; i < m; i++) {
          double s = 0.0;
          for (int r = 0; r < p; r++) s = fma(cu[r + p * i] * w[r], cx[r + p * j], s);
          Qux[i + m * j] += s;
        }
    }
  } else {  // chol_plus!(Q.xx, √Iμ cx), chol_plus!(Q.uu, √Iμ cu): qr([Q; √Iμ c]).R (no ux term, A.5)
    double R[W * W];
    const int rx = n + p;
    for (int j = 0; j < n; j++) {
      for (int i = 0; i < n; i++) Wk[i + rx * j] = Qxx[i + n * j];
      for (int r = 0; r < p; r++) Wk[n + r + rx * j] = ws[r] * cx[r + p * j];
    }
    dev_qr_R(R, Wk, rx, n);
    for (int i = 0; i < n * n; i++) Qxx[i] = R[i];
    if (!term) {
      const int ru = m + p;
      for (int j = 0; j < m; j++) {
        for (int i = 0; i < m; i++) Wk[i + ru * j] = Quu[i + m * j];
        for (int r = 0; r < p; r++) Wk[m + r + ru * j] = ws[r] * cu[r + p * j];
      }
      dev_qr_R(R, Wk, ru, m);
      for (int i = 0; i < m * m; i++) Quu[i] = R[i];
    }
  }
  for (int i = 0; i < n; i++) {
    double s = 0.0;
    for (int r = 0; r < p; r++) s = fma(cx[r + p * i], g[r], s);
    Qx[i] += s;
  }
  if (!term)
    for (int i = 0; i < m; i++) {
      double s = 0.0;
      for (int r = 0; r < p; r++) s = fma(cu[r + p * i], g[r], s);
      Qu[i] += s;
    }
}

// a second stream on the handle's device and the fork/join events that overlap work on it
struct StreamPair {
  hipStream_t st2;
  hipEvent_t fork, join;
};

struct ModelOps {
  int n, m;
  int slack;  // n for an infeasible model (add_slack_controls), else 0
  int pcap;   // max constraint rows per knot of the backward kernels' LDS layout
  int has_con;  // the model defines user constraint functions (ROW_USER_*)
  int min_time; // minimum-time model (MinTime<M>): std backward pass on the LDS kernel only
  long long jws_per_lane;  // doubles of staged-Jacobian state per (knot, partial) lane (0: not staged)
  void (*slack_controls)(const DevProblem*, const DevBuffers&, long long B, int integ, hipStream_t);
  void (*cost_expansion)(const DevProblem*, const DevBuffers&, long long B, int N, int sqrt, int al, int* fail,
                         hipStream_t);
  void (*init)(const DevProblem*, const DevBuffers&, long long B, int integ, int mode, hipStream_t);
  void (*rollout_open)(const DevProblem*, const DevBuffers&, long long B, int integ, hipStream_t);
  void (*jacobian)(const DevProblem*, const DevBuffers&, long long B, int N, int integ, hipStream_t);
  void (*backward)(const DevProblem*, const DevBuffers&, long long B, int sqrt, int al, int flags, int team,
                   hipStream_t);
  // k_expand_team: the cost expansion records the team backward kernel reads (tog_bwd_team.hpp)
  void (*expand)(const DevProblem*, const DevBuffers&, long long B, int N, int pmax, int sqrt, int al, hipStream_t);
  void (*forward)(const DevProblem*, const DevBuffers&, long long B, int integ, int mode, int bookkeeping,
                  const double* Jprev, double* Jout, hipStream_t, const StreamPair* sp);
  void (*cost)(const DevProblem*, const DevBuffers&, long long B, int al, int use_bar, double* J, hipStream_t);
  void (*rollout)(const DevProblem*, const DevBuffers&, long long B, int integ, double alpha, int* ok, hipStream_t);
  void (*update_constraints)(const DevProblem*, const DevBuffers&, long long B, hipStream_t);
  // projected Newton (tog_pn.hpp): phase 0 = k_pn_begin, 1 = k_pn_project, 2 = k_pn_finish, :optimal's
  // 3 = k_pn_kkt, 4 = k_pn_ls_begin, 5 = k_pn_ls_proj, 6 = k_pn_ls_end; null for
  // the infeasible (slack) models
  void (*pn)(const DevProblem*, const DevBuffers&, const PNBuffers&, long long B, int integ, int phase, hipStream_t);
  bool implicit;                   // TOG_RK3_IMPLICIT / TOG_MIDPOINT_IMPLICIT instantiated
  int bwd_lds_bytes;
  int team_tpw;                    // trajectories per wave of k_bwd_team
  int (*team_stride)(int pmax, int sqrt);  // per-team LDS stride of k_bwd_team (doubles)
};

template <class M>
struct ModelLaunch {
  // dual partials per thread: all of them for small models, chunks of 4 otherwise (512-register
  // budget with no scratch for the quadrotor RK4 step)
#ifndef TOG_JW
#define TOG_JW 4
#endif
  // (the Kuka RBD step keeps per-joint force and mass-matrix arrays live: one partial per thread
  // holds its scratch to ~4 KB/lane against ~12 KB with 4)
  using Mb = typename ModelTraits<M>::Base;  // the differentiated model (infeasible: without slacks)
  static constexpr int JW = (Mb::n + Mb::m) <= 6 ? (Mb::n + Mb::m + (ModelTraits<M>::min_time ? 1 : 0))
                                                 : (Mb::id == TOG_MODEL_KUKA ? 1 : TOG_JW);
  static unsigned grid(long long total, int blk) { return (unsigned)((total + blk - 1) / blk); }
  // runtime integrator -> compile-time INTEG (the implicit schemes only where instantiated; tog_create
  // rejects them elsewhere)
  template <class F>
  static void with_integ(int integ, F&& f) {
    if constexpr (!ModelTraits<M>::explicit_ok) {  // KukaImplicit: the implicit schemes only
      if (integ == TOG_RK3_IMPLICIT)
        f(std::integral_constant<int, TOG_RK3_IMPLICIT>{});
      else
        f(std::integral_constant<int, TOG_MIDPOINT_IMPLICIT>{});
      return;
    }
    if (integ == TOG_RK4) {
      f(std::integral_constant<int, TOG_RK4>{});
    } else if (integ == TOG_MIDPOINT) {
      f(std::integral_constant<int, TOG_MIDPOINT>{});
    } else if (integ == TOG_RK3_IMPLICIT || integ == TOG_MIDPOINT_IMPLICIT) {
      if constexpr (ModelTraits<M>::implicit_ok) {
        if (integ == TOG_RK3_IMPLICIT)
          f(std::integral_constant<int, TOG_RK3_IMPLICIT>{});
        else
          f(std::integral_constant<int, TOG_MIDPOINT_IMPLICIT>{});
      }
    } else {
      f(std::integral_constant<int, TOG_RK3>{});
    }
  }
  static void init(const DevProblem* P, const DevBuffers& Bf, long long B, int integ, int mode, hipStream_t st) {
    with_integ(integ, [&](auto ic) {
      constexpr int I = decltype(ic)::value;
      hipLaunchKernelGGL((k_init<M, I>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf, mode);
    });
  }
  static void rollout_open(const DevProblem* P, const DevBuffers& Bf, long long B, int integ, hipStream_t st) {
    with_integ(integ, [&](auto ic) {
      constexpr int I = decltype(ic)::value;
      hipLaunchKernelGGL((k_rollout_open<M, I>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf);
    });
  }
  static void jacobian(const DevProblem* P, const DevBuffers& Bf, long long B, int N, int integ, hipStream_t st) {
    if constexpr (ModelTraits<M>::min_time) {
      using Mc = typename ModelTraits<M>::Core;
      constexpr int NCHT = (Mc::n + Mc::m + 1 + JW - 1) / JW;
      const long long total = B * (long long)(N - 1) * NCHT;
      with_integ(integ, [&](auto ic) {
        constexpr int I = decltype(ic)::value;
        hipLaunchKernelGGL((k_jacobian_mt<M, I, JW>), dim3(grid(total, 256)), dim3(256), 0, st, P, Bf, total);
      });
    } else if (Mb::id == TOG_MODEL_KUKA && integ == TOG_RK3 && Bf.jws && Bf.jac_chain) {
      if constexpr (Mb::id == TOG_MODEL_KUKA && ModelTraits<M>::explicit_ok) {  // stage-chain form (tog_kuka_jac.hpp)
        const long long total = B * (long long)(N - 1);
        hipLaunchKernelGGL((k_kuka_points<M>), dim3(grid(total, 64)), dim3(64), 0, st, P, Bf, total);
        hipLaunchKernelGGL((k_kuka_sjac<M, 0>), dim3(grid(total * 21, 256)), dim3(256), 0, st, P, Bf, total);
        hipLaunchKernelGGL((k_kuka_sjac<M, 1>), dim3(grid(total * 21, 256)), dim3(256), 0, st, P, Bf, total);
        hipLaunchKernelGGL((k_kuka_chain<M>), dim3((unsigned)total), dim3(64), 0, st, P, Bf, total);
      }
    } else if (Mb::id == TOG_MODEL_KUKA && integ == TOG_RK3 && Bf.jws) {
      if constexpr (Mb::id == TOG_MODEL_KUKA && ModelTraits<M>::explicit_ok) {  // duals through the step, one launch per RK3 stage (A/B)
        constexpr int SW = TOG_JAC_STAGE_W, NCHS = (Mb::n + Mb::m + SW - 1) / SW;
        const long long total = B * (long long)(N - 1) * NCHS;
        const dim3 g(grid(total, 256)), blk(256);
        hipLaunchKernelGGL((k_jacobian_rk3_stage<M, 0, SW>), g, blk, 0, st, P, Bf, total);
        hipLaunchKernelGGL((k_jacobian_rk3_stage<M, 1, SW>), g, blk, 0, st, P, Bf, total);
        hipLaunchKernelGGL((k_jacobian_rk3_stage<M, 2, SW>), g, blk, 0, st, P, Bf, total);
      }
    } else {
      constexpr int NCH = (Mb::n + Mb::m + JW - 1) / JW;
      const long long total = B * (long long)(N - 1) * NCH;
      with_integ(integ, [&](auto ic) {
        constexpr int I = decltype(ic)::value;
        hipLaunchKernelGGL((k_jacobian<M, I, JW>), dim3(grid(total, 256)), dim3(256), 0, st, P, Bf, total);
      });
    }
  }
  static void backward(const DevProblem* P, const DevBuffers& Bf, long long B, int sq, int al, int flags, int team,
                       hipStream_t st) {
    if constexpr (M::m <= M::n && M::n + 1 <= 16 && !ModelTraits<M>::min_time) {
    if (team) {  // column-per-lane teams, TPW trajectories per wave (tog_bwd_team.hpp)
      constexpr int TPW = TeamCfg<M>::TPW;
      const dim3 g((unsigned)((B + TPW - 1) / TPW)), blk(64);
      DevBuffers Bl = Bf;  // layout of this variant (the S-region differs between std and sqrt)
      Bl.bwd_stride = Bf.bwd_stride2[sq ? 1 : 0];
      Bl.bwd_shmem = Bf.bwd_shmem2[sq ? 1 : 0];
      const unsigned sm = (unsigned)Bl.bwd_shmem;
      // (ALI bit 1: the time-varying-Objective variants, Bf.tv)
      auto launch = [&](auto wpe_c) {
        constexpr int W = decltype(wpe_c)::value;
        if (sq) {
          if (Bf.tv) {
            if (al) hipLaunchKernelGGL((k_bwd_team<M, 1, 3, W>), g, blk, sm, st, P, Bl, flags);
            else hipLaunchKernelGGL((k_bwd_team<M, 1, 2, W>), g, blk, sm, st, P, Bl, flags);
          } else {
            if (al) hipLaunchKernelGGL((k_bwd_team<M, 1, 1, W>), g, blk, sm, st, P, Bl, flags);
            else hipLaunchKernelGGL((k_bwd_team<M, 1, 0, W>), g, blk, sm, st, P, Bl, flags);
          }
        } else {
          if (Bf.tv) {
            if (al) hipLaunchKernelGGL((k_bwd_team<M, 0, 3, W>), g, blk, sm, st, P, Bl, flags);
            else hipLaunchKernelGGL((k_bwd_team<M, 0, 2, W>), g, blk, sm, st, P, Bl, flags);
          } else {
            if (al) hipLaunchKernelGGL((k_bwd_team<M, 0, 1, W>), g, blk, sm, st, P, Bl, flags);
            else hipLaunchKernelGGL((k_bwd_team<M, 0, 0, W>), g, blk, sm, st, P, Bl, flags);
          }
        }
      };
      // TOG_BWD_TAIL: "quad" (default) or "team" (the one-wave team kernel), for A/B checks (read per
      // launch: tests switch it within one process)
      const char* tk = getenv("TOG_BWD_TAIL");
      const bool quad = !(getenv("TOG_NO_DUO") || (tk && !strcmp(tk, "team")));
      if (Bf.tail && sq && TeamCfg<M>::TEAM == 16 && quad) {
        // convergence tail, square-root pass, one trajectory per workgroup: the QRs, the side work, tmp1
        // and the downdate on four waves (tog_bwd_quad.hpp)
        if constexpr (TeamCfg<M>::TEAM == 16) {
          const dim3 gd((unsigned)B);
          if (Bf.tv) {
            if (al) hipLaunchKernelGGL((k_bwd_quad<M, 3>), gd, dim3(256), 0, st, P, Bf, flags);
            else hipLaunchKernelGGL((k_bwd_quad<M, 2>), gd, dim3(256), 0, st, P, Bf, flags);
          } else {
            if (al) hipLaunchKernelGGL((k_bwd_quad<M, 1>), gd, dim3(256), 0, st, P, Bf, flags);
            else hipLaunchKernelGGL((k_bwd_quad<M, 0>), gd, dim3(256), 0, st, P, Bf, flags);
          }
        }
      } else if (Bf.tail || (B + TPW - 1) / TPW <= Bf.simds) {
        // (a batch that gives at most one wave per SIMD, e.g. config 5's 4,096 Kuka trajectories in 1,024
        // waves, gains nothing from the 2-wave register budget and would spill under it)
        launch(std::integral_constant<int, 1>{});
      } else {
        launch(std::integral_constant<int, TOG_BWD_WAVES>{});
      }
      return;
    }
    }
    const dim3 g((unsigned)B), blk(64);
    if (sq) {
      if (al) hipLaunchKernelGGL((k_backward<M, 1, 1>), g, blk, 0, st, P, Bf, flags);
      else hipLaunchKernelGGL((k_backward<M, 1, 0>), g, blk, 0, st, P, Bf, flags);
    } else {
      if (al) hipLaunchKernelGGL((k_backward<M, 0, 1>), g, blk, 0, st, P, Bf, flags);
      else hipLaunchKernelGGL((k_backward<M, 0, 0>), g, blk, 0, st, P, Bf, flags);
    }
  }
  static void expand(const DevProblem* P, const DevBuffers& Bf, long long B, int N, int pmax, int sq, int al,
                     hipStream_t st) {
    if constexpr (M::m <= M::n && M::n + 1 <= 16 && !ModelTraits<M>::min_time) {
      constexpr int TPW = TeamCfg<M>::TPW;
      const unsigned sm = (unsigned)(sizeof(double) * TPW * expand_team_stride<M>(pmax));
      // square root, at most 4 controls, 16-lane teams: the knots with a constant Q.xx on 4-lane teams
      // (k_expand_u), the dense ones on k_expand_team (only the terminal knot when no stage knot has a
      // state row); TOG_EXPAND_QUAD=0 keeps every knot on k_expand_team, for A/B checks
      int mode = 0;
      if constexpr (M::m <= 4 && TeamCfg<M>::TEAM == 16) {
        const char* eq = getenv("TOG_EXPAND_QUAD");
        if (sq && !(eq && eq[0] == '0')) {
          const long long qteams = B * (long long)(N - 1);
          if (al) hipLaunchKernelGGL((k_expand_u<M, 1>), dim3((unsigned)((qteams + 15) / 16)), dim3(64), 0, st, P, Bf);
          else hipLaunchKernelGGL((k_expand_u<M, 0>), dim3((unsigned)((qteams + 15) / 16)), dim3(64), 0, st, P, Bf);
          mode = (al && Bf.dense_stage_knots) ? 1 : 2;
        }
      }
      const long long teams = (mode == 2) ? B : B * (long long)N;
      const dim3 g((unsigned)((teams + TPW - 1) / TPW)), blk(64);
      if (sq) {
        if (al) hipLaunchKernelGGL((k_expand_team<M, 1, 1>), g, blk, sm, st, P, Bf, mode);
        else hipLaunchKernelGGL((k_expand_team<M, 1, 0>), g, blk, sm, st, P, Bf, mode);
      } else {
        if (al) hipLaunchKernelGGL((k_expand_team<M, 0, 1>), g, blk, sm, st, P, Bf, mode);
        else hipLaunchKernelGGL((k_expand_team<M, 0, 0>), g, blk, sm, st, P, Bf, mode);
      }
    }
  }
  template <int INTEG>
  static void spec(const DevProblem* P, const DevBuffers& Bf, long long B, int mode, int lo, int cnt, const int* list,
                   const int* count, hipStream_t st) {
    // the tail kernels inline the diagonal cost only (the dense cost's run-time indexing of x, u would put
    // them in scratch); dense costs take k_ls_spec
    if (Bf.tail && Bf.cand && Bf.spec_tail2_shmem > 0 && Bf.cost_diag && !list && cnt <= SPEC_LANES) {
      hipLaunchKernelGGL((k_ls_spec_tail2<M, INTEG, 1>), dim3((unsigned)B), dim3(3 * WAVE),
                         (unsigned)Bf.spec_tail2_shmem, st, P, Bf, mode, lo, cnt);
      return;
    }
    if (Bf.tail && Bf.cand && Bf.spec_tail_shmem > 0 && Bf.cost_diag && !list && cnt <= WAVE) {
      hipLaunchKernelGGL((k_ls_spec_tail<M, INTEG, 1>), dim3((unsigned)B), dim3(WAVE), (unsigned)Bf.spec_tail_shmem, st,
                         P, Bf, mode, lo, cnt);
      return;
    }
    const unsigned gs = grid(B * (long long)cnt, 256);  // one lane per (trajectory, trial); list rounds exit early
    const unsigned rb = (mode == TOG_MODE_AL) ? (unsigned)Bf.rows_lds : 0u;
    auto launch = [&](auto cand_c, auto lrt_c, auto dc_c) {
      constexpr bool CAND = decltype(cand_c)::value, LRT = decltype(lrt_c)::value;
      constexpr int DC = decltype(dc_c)::value;
      if constexpr (M::n * M::m > 64)  // (64-lane workgroups spread the waves over every CU: 5% on the Kuka's)
        hipLaunchKernelGGL((k_ls_spec_w1<M, INTEG, CAND, LRT, DC>), dim3(grid(B * (long long)cnt, 64)), dim3(64),
                           LRT ? rb : 0u, st, P, Bf, mode, lo, cnt, list, count);
      else
        hipLaunchKernelGGL((k_ls_spec<M, INTEG, CAND, LRT, DC>), dim3(gs), dim3(256), LRT ? rb : 0u, st, P, Bf, mode,
                           lo, cnt, list, count);
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    using D0 = std::integral_constant<int, 0>;
    using D1 = std::integral_constant<int, 1>;
    if (Bf.cand) {  // (the candidate-copy line search is the default path: its kernels know the diagonal cost)
      if (rb) {
        if (Bf.cost_diag) launch(T_{}, T_{}, D1{});
        else launch(T_{}, T_{}, D0{});
      } else {
        if (Bf.cost_diag) launch(T_{}, F_{}, D1{});
        else launch(T_{}, F_{}, D0{});
      }
    } else {
      if (rb) launch(F_{}, T_{}, D0{});
      else launch(F_{}, F_{}, D0{});
    }
  }
  // candidate-copy line search: one or two speculative rounds, each followed by its decisions, then the
  // copy of the accepted rollouts and the bookkeeping (no replay rollout on the critical path)
  template <int INTEG>
  static void forward_cand(const DevProblem* P, const DevBuffers& Bf, long long B, int mode, int bk, const double* Jp,
                           double* Jo, hipStream_t st) {
    const int F = Bf.ls_first;
    (void)hipMemsetAsync(Bf.ls_count, 0, sizeof(int) * LS_COUNT_SLOTS, st);
    if (F >= Bf.nc) {
      spec<INTEG>(P, Bf, B, mode, 0, Bf.nc, nullptr, nullptr, st);
      hipLaunchKernelGGL((k_ls_decide<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, Bf.nc, bk, Jp, nullptr,
                         nullptr, nullptr, nullptr, 0);
    } else if (bk && Bf.ls_pend_ok) {
      // pending mode: one round per batch step; a trajectory the round leaves undecided continues its
      // line search in the next step's round, so no step waits on a second serial rollout chain
      spec<INTEG>(P, Bf, B, mode, 0, F, nullptr, nullptr, st);
      hipLaunchKernelGGL((k_ls_decide<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, F, bk, Jp, nullptr, nullptr,
                         nullptr, nullptr, 1);
    } else {
      spec<INTEG>(P, Bf, B, mode, 0, F, nullptr, nullptr, st);
      hipLaunchKernelGGL((k_ls_decide<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, F, bk, Jp, nullptr, nullptr,
                         Bf.ls_list, Bf.ls_count, 0);
      spec<INTEG>(P, Bf, B, mode, F, Bf.nc - F, Bf.ls_list, Bf.ls_count, st);
      hipLaunchKernelGGL((k_ls_decide<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, Bf.nc, bk, Jp, Bf.ls_list,
                         Bf.ls_count, nullptr, nullptr, 0);
    }
    const long long tot = B * (long long)Bf.nknots * cand_q<M>();
    hipLaunchKernelGGL((k_ls_apply<M>), dim3(grid(tot, 256)), dim3(256), 0, st, P, Bf, bk);
    hipLaunchKernelGGL((k_ls_fallback<M>), dim3((unsigned)B), dim3(64),
                       (unsigned)(Bf.nknots * (2 * sizeof(double) + sizeof(int))), st, P, Bf,
                       (int)(mode == TOG_MODE_AL), Bf.ls_fb, Bf.ls_count + 2);
    hipLaunchKernelGGL((k_ls_book<M, INTEG>), dim3(grid(B, 64)), dim3(64), (unsigned)Bf.rows_lds, st, P, Bf, mode,
                       bk, Jp, Jo);
    if (bk && mode == TOG_MODE_AL) {
      const unsigned sm = (unsigned)(Bf.nknots * (2 * sizeof(double) + sizeof(int)));
      hipLaunchKernelGGL((k_al_outer<M>), dim3((unsigned)B), dim3(64), sm, st, P, Bf, mode, Bf.ls_done,
                         Bf.ls_count + 1);
    }
  }
  template <int INTEG>
  static void commit(const DevProblem* P, const DevBuffers& Bf, long long B, int mode, int bk, const double* Jp,
                     double* Jo, int phase, int hi, const int* list, const int* count, hipStream_t st) {
    hipLaunchKernelGGL((k_ls_commit<M, INTEG>), dim3(grid(B, 64)), dim3(64), (unsigned)Bf.rows_lds, st, P, Bf, mode,
                       bk, Jp, Jo, phase, hi, list, count);
  }
  template <int INTEG>
  static void forward_i(const DevProblem* P, const DevBuffers& Bf, long long B, int mode, int bk, const double* Jp,
                        double* Jo, hipStream_t st, const StreamPair* sp) {
    if (Bf.cand) {
      forward_cand<INTEG>(P, Bf, B, mode, bk, Jp, Jo, st);
      return;
    }
    // speculative line search in two rounds: trials [0, 8) for every trajectory (settles ~98% of them
    // on configs 2, 3 and 5), then [8, nc) only for the trajectories the first round left undecided
    // (k_ls_compact lists them, so the second round's waves are dense). Narrower first rounds were
    // measured slower: 8 lanes sharing one trajectory's K/X/U per load is what keeps the rollouts
    // coalesced, and the Kuka's heavy lanes need the width to fill the SIMDs.
    (void)hipMemsetAsync(Bf.ls_count, 0, sizeof(int) * LS_COUNT_SLOTS, st);
    if (sp && LS_MAX_ROUNDS == 2 && Bf.nc > LS_FIRST) {
      // the decided trajectories' commit (phase 1) overlaps the second round on a second stream;
      // both kernels are latency bound at low occupancy
      spec<INTEG>(P, Bf, B, mode, 0, LS_FIRST, nullptr, nullptr, st);
      int* list = Bf.ls_list + (size_t)B;
      int* count = Bf.ls_count + 1;
      hipLaunchKernelGGL((k_ls_compact<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, LS_FIRST, bk, Jp, nullptr,
                         nullptr, list, count);
      (void)hipEventRecord(sp->fork, st);
      (void)hipStreamWaitEvent(sp->st2, sp->fork, 0);
      commit<INTEG>(P, Bf, B, mode, bk, Jp, Jo, 1, LS_FIRST, nullptr, nullptr, sp->st2);
      spec<INTEG>(P, Bf, B, mode, LS_FIRST, Bf.nc - LS_FIRST, list, count, st);
      commit<INTEG>(P, Bf, B, mode, bk, Jp, Jo, 2, LS_FIRST, list, count, st);
      (void)hipEventRecord(sp->join, sp->st2);
      (void)hipStreamWaitEvent(st, sp->join, 0);
      return;
    }
    int lo = 0, round = 0;
    const int* list = nullptr;
    const int* count = nullptr;
    while (lo < Bf.nc) {
      const int hi = (round + 1 < LS_MAX_ROUNDS) ? (lo == 0 ? LS_FIRST : 2 * lo) : Bf.nc;
      const int cnt = (hi < Bf.nc ? hi : Bf.nc) - lo;
      if (round > 0) {  // list the trajectories trials [0, lo) did not settle
        int* out = Bf.ls_list + (size_t)(round & 1) * B;
        hipLaunchKernelGGL((k_ls_compact<M>), dim3(grid(B, 256)), dim3(256), 0, st, P, Bf, lo, bk, Jp,
                           list, count, out, Bf.ls_count + round);
        list = out;
        count = Bf.ls_count + round;
      }
      spec<INTEG>(P, Bf, B, mode, lo, cnt, list, count, st);
      lo += cnt;
      round++;
    }
    commit<INTEG>(P, Bf, B, mode, bk, Jp, Jo, 0, 0, nullptr, nullptr, st);
  }
  static void forward(const DevProblem* P, const DevBuffers& Bf, long long B, int integ, int mode, int bk,
                      const double* Jp, double* Jo, hipStream_t st, const StreamPair* sp) {
    with_integ(integ, [&](auto ic) { forward_i<decltype(ic)::value>(P, Bf, B, mode, bk, Jp, Jo, st, sp); });
  }
  static void cost(const DevProblem* P, const DevBuffers& Bf, long long B, int al, int bar, double* J,
                   hipStream_t st) {
    hipLaunchKernelGGL((k_cost<M>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf, al, bar, J);
  }
  static void rollout(const DevProblem* P, const DevBuffers& Bf, long long B, int integ, double alpha, int* ok,
                      hipStream_t st) {
    with_integ(integ, [&](auto ic) {
      constexpr int I = decltype(ic)::value;
      hipLaunchKernelGGL((k_rollout<M, I>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf, alpha, ok);
    });
  }
  static void slack_controls(const DevProblem* P, const DevBuffers& Bf, long long B, int integ, hipStream_t st) {
    // (an infeasible minimum-time model takes its slacks from the infeasible problem: tog_slack_controls refuses)
    if constexpr (ModelTraits<M>::slack > 0 && !ModelTraits<M>::min_time) {
      with_integ(integ, [&](auto ic) {
        constexpr int I = decltype(ic)::value;
        hipLaunchKernelGGL((k_slack_controls<M, I>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf);
      });
    }
  }
  static void cost_expansion(const DevProblem* P, const DevBuffers& Bf, long long B, int N, int sq, int al,
                             int* fail, hipStream_t st) {
    hipLaunchKernelGGL((k_cost_expansion<M>), dim3(grid(B * (long long)N, 64)), dim3(64), 0, st, P, Bf, sq, al,
                       fail);
  }
  static void update_constraints(const DevProblem* P, const DevBuffers& Bf, long long B, hipStream_t st) {
    hipLaunchKernelGGL((k_update_constraints<M>), dim3(grid(B, 64)), dim3(64), 0, st, P, Bf);
  }
  template <int INTEG>
  static void pn_phase(const DevProblem* P, const DevBuffers& Bf, const PNBuffers& W, long long B, int phase,
                       hipStream_t st) {
    // the factoring kernels' LDS is sized by the block stride (pn_lds_bytes; up to 113 KB at SM = 64)
    const size_t lds = pn_lds_bytes(W.SM, M::n + M::m);
    auto big = [&](auto kern) {  // allow dynamic LDS above 64 KB (gfx950: 160 KB per workgroup)
      if (lds > 65536) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipGetLastError();
      }
      hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(64), lds, st, P, Bf, W);
    };
    if (phase == 0)
      hipLaunchKernelGGL((k_pn_begin<M, INTEG>), dim3((unsigned)B), dim3(64), 0, st, P, Bf, W);
    else if (phase == 1)
      big(k_pn_project<M, INTEG>);
    else if (phase == 2)
      hipLaunchKernelGGL((k_pn_finish<M, INTEG>), dim3((unsigned)B), dim3(64), 0, st, P, Bf, W);
    else {  // solve_type :optimal
      if (phase == 3)
        big(k_pn_kkt<M, INTEG>);
      else if (phase == 4)
        big(k_pn_ls_begin<M, INTEG>);
      else if (phase == 5)
        big(k_pn_ls_proj<M, INTEG>);
      else
        big(k_pn_ls_end<M, INTEG>);
    }
  }
  static void pn(const DevProblem* P, const DevBuffers& Bf, const PNBuffers& W, long long B, int integ, int phase,
                 hipStream_t st) {
    with_integ(integ, [&](auto ic) { pn_phase<decltype(ic)::value>(P, Bf, W, B, phase, st); });
  }
  static ModelOps ops() {
    ModelOps o;
    o.n = M::n;
    o.m = M::m;
    o.slack = ModelTraits<M>::slack;
    o.pcap = pcap_of<M>();
    o.has_con = HasCon<M>::value ? 1 : 0;
    o.min_time = ModelTraits<M>::min_time ? 1 : 0;
    o.jws_per_lane = (Mb::id == TOG_MODEL_KUKA && !ModelTraits<M>::min_time) ? 2LL * M::n * 2 : 0;
    o.implicit = ModelTraits<M>::implicit_ok;
    o.slack_controls = slack_controls;
    o.cost_expansion = cost_expansion;
    o.init = init;
    o.rollout_open = rollout_open;
    o.jacobian = jacobian;
    o.backward = backward;
    o.expand = expand;
    o.forward = forward;
    o.cost = cost;
    o.rollout = rollout;
    o.update_constraints = update_constraints;
    // projected Newton: every model whose [x; u] fits a wave (a lane per variable of a knot)
    if constexpr (M::n + M::m <= PN_SM_MAX)
      o.pn = pn;
    else
      o.pn = nullptr;
    o.bwd_lds_bytes = (int)sizeof(BwdLds<M, true>);
    o.team_tpw = TeamCfg<M>::TPW;
    o.team_stride = bwd_team_stride<M>;
    return o;
  }
};

}  // namespace tog
