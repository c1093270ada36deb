// tog_pn.hpp — ALTRO phase 2: the projected Newton feasible projection, batched.
//
// Reference: src/solvers/direct/projected_newton.jl:6-303 (solve!, newton_step!, projection_solve!,
// _projection_solve!, _projection_linesearch!, reg_solve) with ProjectedNewtonSolverOptions
// (direct_solvers.jl:14-30), solve_type :feasible. The CPU restatement is oracle/tog_oracle_pn.c;
// every value here is produced with its operations in its order, so the two agree
// bit for bit.
//
// Mapping (MI355X): one wave (64-thread block) per trajectory. The dual vector is ordered as the
// reference's (direct_solvers.jl:80-105): G_0 = x_1 - x0, G_b = [f(x_b,u_b) - x_{b+1}; active C_b],
// G_N = active C_N. S = Y H⁻¹ Yᵀ is then block tridiagonal with blocks of n + p_active rows: the
// blocks are sized by the rows *active* at a knot, not by every row it carries (the quadrotor maze's
// infeasible problem has 69 rows a knot, of which 13-16 are active), with a stride of
// SM = min(n + pmax, PN_SM_MAX) rows. A block larger than the stride (more than 64 - n active rows)
// stops that trajectory with TOG_TRAJ_PN_ERROR | TOG_TRAJ_PN_BLOCK; nothing is written past it.
// The blocks are built in parallel over their entries (a lane per entry), the block Cholesky of
// S + 1e-2 I sweeps the knots with the current and previous factor staged in LDS (a lane per row
// for the off-diagonal solves, a lane per entry for the Schur updates), and the substitutions run a
// row per lane with the pivot broadcast from lane to lane (__shfl). Factors and S live in a
// per-trajectory HBM workspace (PNBuffers); the trial point goes to X̄, Ū.
#pragma once

namespace tog {

constexpr int PN_SM_MAX = 64;  // largest block (n + active rows): a row per lane of the wave

struct PNState {
  double viol, c_max, J;
  int count;     // _projection_solve! calls of the current projection_solve!
  int finished;  // no further newton step (c_max <= tol after a step, or an error)
  int error;     // TOG_TRAJ_PN_ERROR path
  int steps, projections, linesearches, refinements;
  int active0;   // the solver's own active flag, restored by k_pn_finish (k_jacobian gates on it)
  int over;      // a block outgrew the stride SM (TOG_TRAJ_PN_BLOCK)
  // solve_type :optimal
  int has_S;     // a _projection_solve! has set solver.stats[:S] (its factor in Ld, Lo, block sizes in szS)
  int ls;        // line search stage: 0 none, 1 begin pending, 2 projecting the trial, 3 trial projected
  int ls_count, pcount;  // line search trials, projection! iterations of the current trial
  double alpha, res0;
};

struct PNBuffers {
  double *Sd, *So, *Ld, *Lo;        // (B, nb, SM, SM): S diagonal / sub-diagonal blocks, their factors
  double *yv, *xv, *rv, *wv, *dv;   // (B, nb, SM)
  double* yd;                       // (B, N, n) dynamics rows
  double* Xs;                       // (B, N, n) the point S and H⁻¹Yᵀ were formed at (_projection_solve! start)
  int *act, *na, *sz;               // (B, N, pmax) active rows, (B, N) counts, (B, nb) block sizes
  PNState* st;                      // (B)
  double* wt;                       // (B, N n + (N-1) m) H⁻¹ diagonal of a minimum-time problem, per newton step
  // solve_type :optimal (allocated by the first such call)
  double *Ld2, *Lo2;                // (B, nb, SM, SM) factor of Y Yᵀ / of S without regularization
  double *lb, *tb;                  // (B, nb, SM) active duals in block order, scratch
  double *g, *rz, *dz;              // (B, N (n+m)) cost gradient, g + Yᵀλ, δz (knot j at j (n+m))
  double *nu, *dnu, *nut;           // (B, N, n) dynamics-row duals of solver.V, of δV, of the trial V_
  double *lc, *dlc, *lct;           // (B, N, pmax) constraint-row duals (every row, active or not)
  double *Xv, *Uv;                  // solver.V's primals while the line search moves X, U
  int* szS;                         // (B, nb) block sizes of the factor in Ld, Lo
  int optimal;                      // this call's solve_type is :optimal
  int SM, nb;
  double atol, eps;                 // active_set_tolerance, feasibility_tolerance
};

// per-trajectory views of the workspace
struct PNView {
  double *Sd, *So, *Ld, *Lo, *yv, *xv, *rv, *wv, *dv, *yd, *Xs, *wt;
  double *Ld2, *Lo2, *lb, *tb, *g, *rz, *dz, *nu, *dnu, *nut, *lc, *dlc, *lct, *Xv, *Uv;
  int *act, *na, *sz, *szS;
  int SM;
  __device__ double* M(double* A, int b) const { return A + (size_t)b * SM * SM; }
  __device__ double* V(double* v, int b) const { return v + (size_t)b * SM; }
};

__device__ __forceinline__ PNView pn_view(const PNBuffers& W, const DevProblem* P, long long b) {
  PNView v;
  const size_t blk = (size_t)W.nb * W.SM * W.SM, vec = (size_t)W.nb * W.SM;
  v.Sd = W.Sd + b * blk;
  v.So = W.So + b * blk;
  v.Ld = W.Ld + b * blk;
  v.Lo = W.Lo + b * blk;
  v.yv = W.yv + b * vec;
  v.xv = W.xv + b * vec;
  v.rv = W.rv + b * vec;
  v.wv = W.wv + b * vec;
  v.dv = W.dv + b * vec;
  v.yd = W.yd + (size_t)b * P->N * P->n;
  v.Xs = W.Xs + (size_t)b * P->N * P->n;
  v.wt = W.wt ? W.wt + (size_t)b * (P->N * P->n + (P->N - 1) * P->m) : nullptr;
  v.act = W.act + (size_t)b * P->N * P->pmax;
  v.na = W.na + (size_t)b * P->N;
  v.sz = W.sz + (size_t)b * W.nb;
  v.SM = W.SM;
  if (W.optimal) {
    const size_t nz = (size_t)P->N * (P->n + P->m), nx = (size_t)P->N * P->n, nc = (size_t)P->N * (P->pmax > 0 ? P->pmax : 1);
    v.Ld2 = W.Ld2 + b * blk;
    v.Lo2 = W.Lo2 + b * blk;
    v.lb = W.lb + b * vec;
    v.tb = W.tb + b * vec;
    v.g = W.g + b * nz;
    v.rz = W.rz + b * nz;
    v.dz = W.dz + b * nz;
    v.nu = W.nu + b * nx;
    v.dnu = W.dnu + b * nx;
    v.nut = W.nut + b * nx;
    v.lc = W.lc + b * nc;
    v.dlc = W.dlc + b * nc;
    v.lct = W.lct + b * nc;
    v.Xv = W.Xv + b * nx;
    v.Uv = W.Uv + b * (size_t)(P->N - 1) * P->m;
    v.szS = W.szS + (size_t)b * W.nb;
  }
  return v;
}

__device__ __forceinline__ void pn_sync() { __syncthreads(); }  // one-wave blocks: orders LDS traffic

// H⁻¹ diagonal (Diagonal(solver.H): Q·dt, R·dt, terminal Qf; cost.jl:214-228). A minimum-time problem's
// depends on the newton step's X, U (MinTimeCost's hessian!, minimum_time.jl:238-280): k_pn_begin writes it
// to the view's wt (pn_weights_min_time).
template <class M>
__device__ __forceinline__ double pn_wx(const DevProblem* P, const PNView& w, int k, int i) {
  if constexpr (ModelTraits<M>::min_time) {
    return w.wt[(size_t)k * M::n + i];
  } else {
    const int n = P->n;
    if (k == P->N - 1) return 1.0 / P->Qf[i + n * i];
    const double* Q = P->kc ? P->kc + (size_t)k * P->kc_stride : P->Q;  // a time-varying Objective's knot k
    return 1.0 / (Q[i + n * i] * P->dt);
  }
}
template <class M>
__device__ __forceinline__ double pn_wu(const DevProblem* P, const PNView& w, int k, int i) {
  if constexpr (ModelTraits<M>::min_time) {
    return w.wt[(size_t)P->N * M::n + (size_t)k * M::m + i];
  } else {
    const double* R = P->kc ? P->kc + (size_t)k * P->kc_stride + P->n * P->n : P->R;
    return 1.0 / (R[i + P->m * i] * P->dt);
  }
}
// update!'s cost_expansion! of a minimum-time problem (projected_newton.jl:122-148) at X, U, on the diagonal:
// Q·h² and R·h² for the model's states and controls (dt = h² = u[end]²), R_min_time for τ, 2 ℓ(x, u) +
// R_min_time for h (ℓ the quadratic stage cost without dt), terminal Qf and R_min_time. A lane per knot.
template <class M>
__device__ void pn_weights_min_time(const DevProblem* P, const PNView& w, const double* X, const double* U, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N;
  for (int k = lane; k < N; k += WAVE) {
    double* wx = w.wt + (size_t)k * n;
    if (k < N - 1) {
      double* wu = w.wt + (size_t)N * n + (size_t)k * m;
      const double* x = X + (size_t)k * n;
      const double* u = U + (size_t)k * m;
      const CostView C_ = cost_at<n, m>(P, k);
      const double h = u[m - 1], dt = h * h;
      for (int i = 0; i < n - 1; i++) wx[i] = 1.0 / (C_.Q[i + n * i] * dt);
      wx[n - 1] = 1.0 / P->R_min_time;
      for (int i = 0; i < m - 1; i++) wu[i] = 1.0 / (C_.R[i + m * i] * dt);
      const double l1 = stage_cost_dt<n, m>(P, k, x, u, 1.0);
      wu[m - 1] = 1.0 / (2.0 * l1 + P->R_min_time);
    } else {
      for (int i = 0; i < n - 1; i++) wx[i] = 1.0 / P->Qf[i + n * i];
      wx[n - 1] = 1.0 / P->R_min_time;
    }
  }
  pn_sync();
}

// dynamics_constraints! + update_constraints! at (X, U): dynamics rows into yd, constraint values
// into C (projected_newton.jl:36-44,67-73). A lane per knot.
template <class M, int INTEG>
__device__ void pn_eval(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                        const double* U, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  double* C = Bf.C + (size_t)b * N * pmax;
  const double* x0 = Bf.x0 + (size_t)b * n;
  for (int k = lane; k < N; k += WAVE) {
    const double* xk = X + (size_t)k * n;
    if (k == 0)
      for (int i = 0; i < n; i++) w.yd[i] = xk[i] - x0[i];
    if (k < N - 1) {
      double xn[n];
      discrete_step<M, INTEG>(xn, xk, U + (size_t)k * m, P->dt);
      for (int i = 0; i < n; i++) w.yd[(size_t)(k + 1) * n + i] = xn[i] - X[(size_t)(k + 1) * n + i];
    }
    const int cnt = P->knot_cnt[k];
    const ConRow* rows = P->rows + P->knot_off[k];
    for (int r = 0; r < cnt; r++) C[(size_t)k * pmax + r] = row_value_m<M>(rows[r], xk, k < N - 1 ? U + (size_t)k * m : nullptr);
  }
  pn_sync();
}

// active_set! (projected_newton.jl:75-93) and the block sizes. A lane per knot.
// Returns (to every lane) whether a block outgrew the stride SM; the caller then stops the trajectory.
__device__ int pn_active_set(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, double tol,
                             int nb, int lane) {
  const int N = P->N, pmax = P->pmax, n = P->n;
  const double* C = Bf.C + (size_t)b * N * pmax;
  for (int k = lane; k < N; k += WAVE) {
    const ConRow* rows = P->rows + P->knot_off[k];
    int c = 0;
    for (int i = 0; i < P->knot_cnt[k]; i++)
      if (!row_inequality(rows[i]) || C[(size_t)k * pmax + i] >= -tol) w.act[k * pmax + c++] = i;
    w.na[k] = c;
  }
  pn_sync();
  int over = 0;
  for (int bb = lane; bb < nb; bb += WAVE) {
    w.sz[bb] = (bb < N ? n : 0) + (bb >= 1 ? w.na[bb - 1] : 0);
    over |= w.sz[bb] > w.SM;
  }
  return __syncthreads_or(over);
}

// y[a] into yv (block order) and its Inf norm (NaN propagates); every lane returns it
__device__ double pn_gather_y(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, int nb,
                              int lane) {
  const int N = P->N, pmax = P->pmax, n = P->n;
  const double* C = Bf.C + (size_t)b * N * pmax;
  double viol = 0.0;
  for (int bb = lane; bb < nb; bb += WAVE) {
    double* y = w.V(w.yv, bb);
    int r = 0;
    if (bb < N)
      for (int i = 0; i < n; i++) y[r++] = w.yd[(size_t)bb * n + i];
    if (bb >= 1) {
      const int k = bb - 1;
      for (int q = 0; q < w.na[k]; q++) y[r++] = C[(size_t)k * pmax + w.act[k * pmax + q]];
    }
    for (int i = 0; i < r; i++) viol = tog_jlmax(viol, fabs(y[i]));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) viol = tog_jlmax(viol, __shfl_xor(viol, off, WAVE));
  pn_sync();
  return viol;
}

// rows of block bb on its own variables z_j = (x_j, u_j), j = bb-1, dense into LDS Yz (SM x (n+m))
template <class M>
__device__ void pn_block_rows(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, int bb,
                              const double* X, double* Yz, int lane) {
  constexpr int n = M::n, m = M::m, L = n + m;
  const int N = P->N, pmax = P->pmax, SM = w.SM, j = bb - 1;
  for (int e = lane; e < SM * L; e += WAVE) Yz[e] = 0.0;
  pn_sync();
  const int rb = (bb < N) ? n : 0;
  if (bb < N) {
    const double* AB = Bf.AB + ((size_t)b * (N - 1) + j) * n * L;
    for (int e = lane; e < n * L; e += WAVE) Yz[(e % n) + SM * (e / n)] = AB[e];
  }
  if (lane < w.na[j]) {
    const ConRow r = P->rows[P->knot_off[j] + w.act[j * pmax + lane]];
    int idx[row_grad_cap<M>()];
    double v[row_grad_cap<M>()];
    const int nz = row_grad_m<M>(r, X + (size_t)j * n, j < N - 1 ? Bf.U + ((size_t)b * (N - 1) + j) * m : nullptr, idx, v);
    for (int z = 0; z < nz; z++) Yz[(rb + lane) + SM * idx[z]] = v[z];
  }
  pn_sync();
}

// S = Y H⁻¹ Yᵀ by blocks (projected_newton.jl:233-234; structure of _buildShurCompliment!, :728-757);
// UNIT: Y Yᵀ (multiplier_projection!)
template <class M, bool UNIT = false>
__device__ void pn_build_S(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                           double* Yz, int nb, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, SM = w.SM;
  {
    double* S0 = w.M(w.Sd, 0);
    for (int e = lane; e < SM * SM; e += WAVE)
      S0[e] = ((e % SM) == (e / SM) && (e % SM) < n) ? (UNIT ? 1.0 : pn_wx<M>(P, w, 0, e % SM)) : 0.0;
  }
  for (int bb = 1; bb < nb; bb++) {
    const int j = bb - 1, sb = w.sz[bb], sp = w.sz[bb - 1], nv = (bb < N) ? n + m : n;
    pn_block_rows<M>(P, Bf, b, w, bb, X, Yz, lane);
    double* Sd = w.M(w.Sd, bb);
    for (int e = lane; e < sb * sb; e += WAVE) {
      const int i = e % sb, l = e / sb;
      double acc = 0.0;
      for (int v = 0; v < nv; v++) {
        const double wv = UNIT ? 1.0 : v < n ? pn_wx<M>(P, w, j, v) : pn_wu<M>(P, w, j, v - n);
        acc = fma(Yz[i + SM * v], wv * Yz[l + SM * v], acc);
      }
      if (bb < N && i < n && i == l) acc = acc + (UNIT ? 1.0 : pn_wx<M>(P, w, j + 1, i));
      Sd[i + SM * l] = acc;
    }
    const double sg = (bb - 1 == 0) ? 1.0 : -1.0;
    double* So = w.M(w.So, bb);
    for (int e = lane; e < sb * sp; e += WAVE) {
      const int i = e % sb, c = e / sb;
      So[i + SM * c] = (c < n) ? Yz[i + SM * c] * (sg * (UNIT ? 1.0 : pn_wx<M>(P, w, j, c))) : 0.0;
    }
    pn_sync();
  }
}

// block Cholesky of S + ρI; Lp/Lc: LDS (SM x SM each), LoL: LDS (SM x SM). Returns 0 or a failure.
__device__ int pn_factor(const PNView& w, int nb, double rho, double* Lp, double* Lc, double* LoL, int lane) {
  const int SM = w.SM;
  for (int bb = 0; bb < nb; bb++) {
    const int sb = w.sz[bb];
    const int sp = bb >= 1 ? w.sz[bb - 1] : 0;
    if (bb >= 1 && lane < sb) {  // Lo_b = So_b Lp^{-T}: lane i solves Lp y = So_b[i, :]ᵀ
      const double* So = w.M(w.So, bb);
      for (int l = 0; l < sp; l++) {
        double t = So[lane + SM * l];
        for (int q = 0; q < l; q++) t = fma(-Lp[l + SM * q], LoL[lane + SM * q], t);
        LoL[lane + SM * l] = t / Lp[l + SM * l];
      }
    }
    pn_sync();
    const double* Sd = w.M(w.Sd, bb);
    for (int e = lane; e < sb * sb; e += WAVE) {
      const int i = e % sb, l = e / sb;
      if (i < l) continue;
      double t = Sd[i + SM * l];
      if (i == l) t = t + rho;
      for (int q = 0; q < sp; q++) t = fma(-LoL[i + SM * q], LoL[l + SM * q], t);
      Lc[i + SM * l] = t;
    }
    pn_sync();
    for (int j = 0; j < sb; j++) {  // right-looking Cholesky (oracle pn_chol)
      const double a = Lc[j + SM * j];
      if (!(a > 0.0)) return bb + 1;
      const double d = sqrt(a);
      pn_sync();
      if (lane == j) Lc[j + SM * j] = d;
      if (lane > j && lane < sb) Lc[lane + SM * j] = Lc[lane + SM * j] / d;
      pn_sync();
      const int t = sb - j - 1;
      for (int e = lane; e < t * t; e += WAVE) {
        const int i = j + 1 + e % t, l = j + 1 + e / t;
        if (i >= l) Lc[i + SM * l] = fma(-Lc[i + SM * j], Lc[l + SM * j], Lc[i + SM * l]);
      }
      pn_sync();
    }
    double* Ld = w.M(w.Ld, bb);
    double* Lo = w.M(w.Lo, bb);
    for (int e = lane; e < SM * SM; e += WAVE) {
      Ld[e] = Lc[e];
      Lp[e] = Lc[e];
      if (bb >= 1) Lo[e] = LoL[e];
    }
    pn_sync();
  }
  return 0;
}

// x = (S + ρI)⁻¹ r through the block factor (a row per lane, pivots broadcast by __shfl).
// T1, T2: LDS staging (SM x SM) of the blocks being used; xn: LDS (SM) previous block's solution.
__device__ void pn_fsolve(const PNView& w, int nb, const double* r, double* x, double* T1, double* T2, double* xn,
                          int lane) {
  const int SM = w.SM;
  for (int bb = 0; bb < nb; bb++) {  // forward
    const int sb = w.sz[bb], sp = bb >= 1 ? w.sz[bb - 1] : 0;
    const double* Ld = w.M(w.Ld, bb);
    const double* Lo = w.M(w.Lo, bb);
    for (int e = lane; e < SM * SM; e += WAVE) {
      T1[e] = Ld[e];
      if (bb >= 1) T2[e] = Lo[e];
    }
    pn_sync();
    double t = 0.0;
    if (lane < sb) {
      t = w.V(const_cast<double*>(r), bb)[lane];
      for (int q = 0; q < sp; q++) t = fma(-T2[lane + SM * q], xn[q], t);
    }
    double* wb = w.V(w.wv, bb);
    const double dl = (lane < sb) ? T1[lane + SM * lane] : 1.0;  // this lane's pivot L[i,i]
    for (int l = 0; l < sb; l++) {
      const double wl = __shfl(t / dl, l, WAVE);
      if (lane == l) wb[l] = wl;
      if (lane > l && lane < sb) t = fma(-T1[lane + SM * l], wl, t);
    }
    pn_sync();
    if (lane < sb) xn[lane] = wb[lane];
    pn_sync();
  }
  for (int bb = nb - 1; bb >= 0; bb--) {  // backward
    const int sb = w.sz[bb], sn = bb + 1 < nb ? w.sz[bb + 1] : 0;
    const double* Ld = w.M(w.Ld, bb);
    for (int e = lane; e < SM * SM; e += WAVE) {
      T1[e] = Ld[e];
      if (bb + 1 < nb) T2[e] = w.M(w.Lo, bb + 1)[e];
    }
    pn_sync();
    double t = 0.0;
    if (lane < sb) {
      t = w.V(w.wv, bb)[lane];
      for (int q = 0; q < sn; q++) t = fma(-T2[q + SM * lane], xn[q], t);
    }
    double* xb = w.V(x, bb);
    const double dl = (lane < sb) ? T1[lane + SM * lane] : 1.0;
    for (int l = sb - 1; l >= 0; l--) {
      const double xl = __shfl(t / dl, l, WAVE);
      if (lane == l) xb[l] = xl;
      if (lane < l) t = fma(-T1[l + SM * lane], xl, t);
    }
    pn_sync();
    if (lane < sb) xn[lane] = xb[lane];
    pn_sync();
  }
}

// r = y - S x (a row per lane); |r|₂ with the oracle's sequential sum (lane 0), returned to all lanes
__device__ double pn_residual(const PNView& w, int nb, const double* y, const double* x, double* r, double* rl,
                              int lane) {
  const int SM = w.SM;
  double ss = 0.0;
  for (int bb = 0; bb < nb; bb++) {
    const int sb = w.sz[bb];
    if (lane < sb) {
      const int i = lane;
      const double* Sd = w.M(w.Sd, bb);
      const double* xb = w.V(const_cast<double*>(x), bb);
      double t = 0.0;
      for (int q = 0; q < sb; q++) t = fma(Sd[i + SM * q], xb[q], t);
      if (bb >= 1) {
        const double* So = w.M(w.So, bb);
        const double* xp = w.V(const_cast<double*>(x), bb - 1);
        for (int q = 0; q < w.sz[bb - 1]; q++) t = fma(So[i + SM * q], xp[q], t);
      }
      if (bb + 1 < nb) {
        const double* So1 = w.M(w.So, bb + 1);
        const double* xq = w.V(const_cast<double*>(x), bb + 1);
        for (int q = 0; q < w.sz[bb + 1]; q++) t = fma(So1[q + SM * i], xq[q], t);
      }
      const double ri = w.V(const_cast<double*>(y), bb)[i] - t;
      w.V(r, bb)[i] = ri;
      rl[i] = ri;
    }
    pn_sync();
    if (lane == 0)
      for (int i = 0; i < sb; i++) ss = fma(rl[i], rl[i], ss);
    pn_sync();
  }
  return sqrt(__shfl(ss, 0, WAVE));
}

// LDS of the kernels that factor and solve (dynamic, sized by the stride SM and L = n + m): three SM x SM
// blocks, the rows of one block on its knot's variables (SM x L), two vectors. 113 KB at SM = 64, L = 30.
struct PNLds {
  double *A, *Bm, *Cm, *Yz, *vec, *vec2;
};
__host__ __device__ constexpr size_t pn_lds_bytes(int SM, int L) {
  return sizeof(double) * ((size_t)3 * SM * SM + (size_t)SM * L + 2 * (size_t)SM);
}
__device__ __forceinline__ PNLds pn_lds(int SM, int L) {
  extern __shared__ double pn_smem[];
  PNLds s;
  s.A = pn_smem;
  s.Bm = s.A + SM * SM;
  s.Cm = s.Bm + SM * SM;
  s.Yz = s.Cm + SM * SM;
  s.vec = s.Yz + SM * L;
  s.vec2 = s.vec + SM;
  return s;
}

// reg_solve(S, y, Sreg, 1e-8, 25) into xv (projected_newton.jl:286-303)
__device__ void pn_reg_solve(const PNView& w, int nb, PNLds& sh, PNState& s, int lane) {
  pn_fsolve(w, nb, w.yv, w.xv, sh.A, sh.Bm, sh.vec, lane);
  for (int cnt = 0; cnt < 25; cnt++) {
    const double nr = pn_residual(w, nb, w.yv, w.xv, w.rv, sh.vec2, lane);
    if (nr < 1e-8) break;
    pn_fsolve(w, nb, w.rv, w.dv, sh.A, sh.Bm, sh.vec, lane);
    for (int bb = 0; bb < nb; bb++)
      if (lane < w.sz[bb]) w.V(w.xv, bb)[lane] = w.V(w.xv, bb)[lane] + w.V(w.dv, bb)[lane];
    pn_sync();
    s.refinements++;
  }
}

// trial point Z_ = Z + α δZ, δZ = -H⁻¹ Yᵀ δλ, into X̄, Ū (a variable per lane)
template <class M>
__device__ void pn_trial(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, double* Yz,
                         double alpha, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, SM = w.SM;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  double* Xt = Bf.Xb + (size_t)b * N * n;
  double* Ut = Bf.Ub + (size_t)b * (N - 1) * m;
  for (int j = 0; j < N; j++) {
    const int bb = j + 1, nv = (j < N - 1) ? n + m : n;
    pn_block_rows<M>(P, Bf, b, w, bb, w.Xs, Yz, lane);  // H⁻¹Yᵀ of _projection_solve!: Jacobians at its start
    if (lane < nv) {
      const int v = lane;
      double t = 0.0;
      if (v < n) t = (j == 0) ? w.V(w.xv, 0)[v] : -w.V(w.xv, j)[v];
      const double* lb = w.V(w.xv, bb);
      for (int i = 0; i < w.sz[bb]; i++) t = fma(Yz[i + SM * v], lb[i], t);
      const double wv = v < n ? pn_wx<M>(P, w, j, v) : pn_wu<M>(P, w, j, v - n);
      const double dz = -(wv * t);
      if (v < n)
        Xt[(size_t)j * n + v] = X[(size_t)j * n + v] + alpha * dz;
      else
        Ut[(size_t)j * m + (v - n)] = U[(size_t)j * m + (v - n)] + alpha * dz;
    }
    pn_sync();
  }
}

// newton_step! prologue (update!: active set at V) and projection_solve!'s first viol
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_begin(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNState& s = W.st[b];
  if (s.finished) return;
  const PNView w = pn_view(W, P, b);
  const int N = P->N;
  if (W.optimal && s.steps > 0) {  // :optimal: every newton step starts from solver.V, not from the returned V_
    for (int e = lane; e < N * M::n; e += WAVE) Bf.X[(size_t)b * N * M::n + e] = w.Xv[e];
    for (int e = lane; e < (N - 1) * M::m; e += WAVE) Bf.U[(size_t)b * (N - 1) * M::m + e] = w.Uv[e];
    pn_sync();
  }
  if constexpr (ModelTraits<M>::min_time)
    pn_weights_min_time<M>(P, w, Bf.X + (size_t)b * N * M::n, Bf.U + (size_t)b * (N - 1) * M::m, lane);
  pn_eval<M, INTEG>(P, Bf, b, w, Bf.X + (size_t)b * N * M::n, Bf.U + (size_t)b * (N - 1) * M::m, lane);
  if (pn_active_set(P, Bf, b, w, W.atol, W.nb, lane)) {
    if (lane == 0) {
      s.active0 = Bf.st[b].active;
      s.error = s.over = 1;
      s.viol = NAN;
      Bf.st[b].active = 0;
    }
    return;
  }
  const double viol = pn_gather_y(P, Bf, b, w, W.nb, lane);
  if (W.optimal) {  // update!'s Jacobians at V: the first k_jacobian of the projection loop, for every trajectory
    for (int e = lane; e < N * M::n; e += WAVE) w.Xs[e] = Bf.X[(size_t)b * N * M::n + e];
    pn_sync();
  }
  if (lane == 0) {
    s.viol = viol;
    s.count = 0;
    // k_jacobian runs only for active trajectories: a converged AL solve left them inactive
    s.active0 = Bf.st[b].active;
    Bf.st[b].active = (W.optimal || viol > W.eps) ? 1 : 0;
  }
}

// a block outgrew the stride: stop the trajectory (k_pn_finish flags it)
__device__ __forceinline__ void pn_stop_over(PNState& s, PNState* dst, TrajState& ts, int lane) {
  if (lane == 0) {
    s.error = s.over = 1;
    *dst = s;
    ts.active = 0;
  }
}

// one pass of projection_solve!'s loop: _projection_solve! (Jacobians from k_jacobian at X, U)
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_project(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNLds sh = pn_lds(W.SM, M::n + M::m);
  PNState s = W.st[b];
  if (s.finished || s.error || s.count >= 10 || !(s.viol > W.eps)) {  // while count < 10 && viol > eps
    if (W.optimal && lane == 0 && !s.finished) Bf.st[b].active = 0;     // (:optimal: Jacobians at V are kept)
    return;
  }
  constexpr int n = M::n, m = M::m;
  const int N = P->N, nb = W.nb;
  const PNView w = pn_view(W, P, b);
  double* X = Bf.X + (size_t)b * N * n;
  double* U = Bf.U + (size_t)b * (N - 1) * m;
  s.count++;
  s.projections++;
  for (int e = lane; e < N * n; e += WAVE) w.Xs[e] = X[e];
  pn_eval<M, INTEG>(P, Bf, b, w, X, U, lane);
  if (pn_active_set(P, Bf, b, w, W.atol, nb, lane)) return pn_stop_over(s, &W.st[b], Bf.st[b], lane);
  const double viol0 = pn_gather_y(P, Bf, b, w, nb, lane);
  pn_build_S<M>(P, Bf, b, w, X, sh.Yz, nb, lane);
  double viol = viol0;
  if (pn_factor(w, nb, 1e-2, sh.A, sh.Bm, sh.Cm, lane)) {
    s.error = 1;  // PosDefException in cholesky
  } else {
    s.has_S = 1;  // solver.stats[:S] = Sreg
    if (W.optimal && lane < nb) {
      for (int bb = lane; bb < nb; bb += WAVE) w.szS[bb] = w.sz[bb];
    }
    double viol_prev = viol0;
    for (int count = 0; count < 10; count++) {
      // _projection_linesearch!: y at the current point (last evaluation), δλ, trial, y at the trial
      const double vls0 = pn_gather_y(P, Bf, b, w, nb, lane);
      s.linesearches++;
      pn_reg_solve(w, nb, sh, s, lane);
      pn_trial<M>(P, Bf, b, w, sh.Yz, 1.0, lane);
      double* Xt = Bf.Xb + (size_t)b * N * n;
      double* Ut = Bf.Ub + (size_t)b * (N - 1) * m;
      pn_eval<M, INTEG>(P, Bf, b, w, Xt, Ut, lane);
      viol = pn_gather_y(P, Bf, b, w, nb, lane);
      if (!(viol < vls0)) {  // `count += a` (MethodError) in the reference
        s.error = 1;
        break;
      }
      for (int e = lane; e < N * n; e += WAVE) X[e] = Xt[e];
      for (int e = lane; e < (N - 1) * m; e += WAVE) U[e] = Ut[e];
      pn_sync();
      const double rate = log10(viol) / log10(viol_prev);
      viol_prev = viol;
      if (rate < 1.1 || viol < W.eps) break;
    }
    if (!s.error) viol = viol_prev;
  }
  s.viol = viol;
  if (lane == 0) {
    W.st[b] = s;
    if (s.error || s.count >= 10 || !(s.viol > W.eps)) Bf.st[b].active = 0;  // no further Jacobians
  }
}

// record_iteration!: J = cost(prob), c_max = max_violation(prob) at X, U; the solve! loop's break
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_finish(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNState s = W.st[b];
  if (s.finished) return;
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pmax = P->pmax;
  const double* X = Bf.X + (size_t)b * N * n;
  const double* U = Bf.U + (size_t)b * (N - 1) * m;
  double* C = Bf.C + (size_t)b * N * pmax;
  for (int k = lane; k < N; k += WAVE) {
    const int cnt = P->knot_cnt[k];
    const ConRow* rows = P->rows + P->knot_off[k];
    for (int r = 0; r < cnt; r++)
      C[(size_t)k * pmax + r] = row_value_m<M>(rows[r], X + (size_t)k * n, k < N - 1 ? U + (size_t)k * m : nullptr);
  }
  pn_sync();
  if (lane != 0) return;
  Bf.st[b].active = s.active0;
  s.steps++;
  s.c_max = traj_max_violation(P, Bf, b);
  s.J = traj_cost<M>(P, Bf, b, X, U, false, nullptr);
  if (s.error || s.c_max <= W.eps) s.finished = 1;
  if (s.error) Bf.st[b].flags |= TOG_TRAJ_PN_ERROR | (s.over ? TOG_TRAJ_PN_BLOCK : 0);
  W.st[b] = s;
}

// ---------------------------------------------------------------------------------------------------------
// solve_type :optimal: newton_step! after the projection (projected_newton.jl:522-546). The oracle's
// pn_grad / pn_form_r / pn_multiplier_projection / pn_kkt / pn_line_search (oracle/tog_oracle_pn.c) with the
// same operations in the same order. Kernels: k_pn_kkt (cost_expansion!, multiplier_projection!,
// solveKKT_Shur at solver.V), k_pn_ls_begin (line_search's update! and res0, first trial),
// k_pn_ls_proj (one projection! iteration at the trial, after k_jacobian there), k_pn_ls_end
// (multiplier_projection! at the projected trial, the acceptance test, the next trial).
// ---------------------------------------------------------------------------------------------------------

// the objective's gradient (cost_expansion!'s gradient!, :139-148) at X, U into w.g; a lane per knot. A
// minimum-time problem's is MinTimeCost's gradient! (minimum_time.jl:201-237): the padded quadratic cost's at
// dt = h², R_min_time τ for τ, τ (2 ℓ(x, u) + R_min_time) for h, terminal Qf x + qf and R_min_time τ
template <class M>
__device__ void pn_grad(const DevProblem* P, const PNView& w, const double* X, const double* U, int lane) {
  constexpr int n = M::n, m = M::m;
  constexpr bool MT = ModelTraits<M>::min_time;
  const int N = P->N;
  for (int k = lane; k < N; k += WAVE) {
    const double* x = X + (size_t)k * n;
    double* q = w.g + (size_t)k * (n + m);
    if (k < N - 1) {
      const double* u = U + (size_t)k * m;
      const CostView C_ = cost_at<n, m>(P, k);
      const double dt = MT ? u[m - 1] * u[m - 1] : P->dt;
      for (int i = 0; i < n; i++) {
        double a = 0.0, c = 0.0;
        for (int j = 0; j < n; j++) a = fma(C_.Q[i + n * j], x[j], a);
        for (int j = 0; j < m; j++) c = fma(C_.H[j + m * i], u[j], c);
        q[i] = ((a + C_.q[i]) + c) * dt;
      }
      for (int i = 0; i < m; i++) {
        double a = 0.0, c = 0.0;
        for (int j = 0; j < m; j++) a = fma(C_.R[i + m * j], u[j], a);
        for (int j = 0; j < n; j++) c = fma(C_.H[i + m * j], x[j], c);
        q[n + i] = ((a + C_.r[i]) + c) * dt;
      }
      if constexpr (MT) {
        const double l1 = stage_cost_dt<n, m>(P, k, x, u, 1.0);
        q[n + m - 1] = u[m - 1] * (2.0 * l1 + P->R_min_time);
        q[n - 1] = P->R_min_time * x[n - 1];
      }
    } else {
      for (int i = 0; i < n; i++) {
        double a = 0.0;
        for (int j = 0; j < n; j++) a = fma(P->Qf[i + n * j], x[j], a);
        q[i] = a + P->qf[i];
      }
      if constexpr (MT) q[n - 1] = P->R_min_time * x[n - 1];
    }
  }
  pn_sync();
}

// duals (full layout) <-> the active duals in block order; a lane per block
__device__ void pn_gather_duals(const DevProblem* P, const PNView& w, const double* nu, const double* lc, double* lb,
                                int nb, int lane) {
  const int N = P->N, pmax = P->pmax, n = P->n;
  for (int bb = lane; bb < nb; bb += WAVE) {
    double* l = lb + (size_t)bb * w.SM;
    int r = 0;
    if (bb < N)
      for (int i = 0; i < n; i++) l[r++] = nu[(size_t)bb * n + i];
    if (bb >= 1)
      for (int q = 0; q < w.na[bb - 1]; q++) l[r++] = lc[(size_t)(bb - 1) * pmax + w.act[(bb - 1) * pmax + q]];
  }
  pn_sync();
}
__device__ void pn_scatter_duals(const DevProblem* P, const PNView& w, const double* lb, double* nu, double* lc,
                                 int nb, int lane) {
  const int N = P->N, pmax = P->pmax, n = P->n;
  for (int bb = lane; bb < nb; bb += WAVE) {
    const double* l = lb + (size_t)bb * w.SM;
    int r = 0;
    if (bb < N)
      for (int i = 0; i < n; i++) nu[(size_t)bb * n + i] = l[r++];
    if (bb >= 1)
      for (int q = 0; q < w.na[bb - 1]; q++) lc[(size_t)(bb - 1) * pmax + w.act[(bb - 1) * pmax + q]] = l[r++];
  }
  pn_sync();
}

// out = Yᵀ l: column z_j gets ±l_j (+I initial condition, -I dynamics of block j), then block j+1's rows
template <class M>
__device__ void pn_yt(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                      const double* l, double* out, double* Yz, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, SM = w.SM;
  for (int j = 0; j < N; j++) {
    const int bb = j + 1, nv = (j < N - 1) ? n + m : n;
    pn_block_rows<M>(P, Bf, b, w, bb, X, Yz, lane);
    if (lane < nv) {
      const int v = lane;
      double t = (v < n) ? ((j == 0) ? l[v] : -l[(size_t)j * SM + v]) : 0.0;
      const double* lbb = l + (size_t)bb * SM;
      for (int i = 0; i < w.sz[bb]; i++) t = fma(Yz[i + SM * v], lbb[i], t);
      out[(size_t)j * (n + m) + v] = t;
    }
    pn_sync();
  }
}

// out = Y z (block order): row i of block bb from its ±I term, then block bb's own variables z_{bb-1}
template <class M>
__device__ void pn_ymul(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                        const double* z, double* out, double* Yz, int nb, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, SM = w.SM;
  for (int bb = 0; bb < nb; bb++) {
    const int j = bb - 1, nv = (j < N - 1) ? n + m : n;
    if (bb >= 1) pn_block_rows<M>(P, Bf, b, w, bb, X, Yz, lane);
    if (lane < w.sz[bb]) {
      const int i = lane;
      double t = (bb < N && i < n) ? ((bb == 0) ? z[i] : -z[(size_t)bb * (n + m) + i]) : 0.0;
      if (bb >= 1)
        for (int v = 0; v < nv; v++) t = fma(Yz[i + SM * v], z[(size_t)j * (n + m) + v], t);
      out[(size_t)bb * SM + i] = t;
    }
    pn_sync();
  }
}

// |[g + Yᵀλ; y]|₂ with rz = g + Yᵀλ formed: the oracle's sequential sum of squares (lane 0)
__device__ double pn_res_norm(const DevProblem* P, const PNView& w, int nb, int lane) {
  double ss = 0.0;
  if (lane == 0) {
    const int n = P->n, m = P->m, N = P->N;
    for (int j = 0; j < N; j++)
      for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) {
        const double r = w.rz[(size_t)j * (n + m) + v];
        ss = fma(r, r, ss);
      }
    for (int bb = 0; bb < nb; bb++)
      for (int i = 0; i < w.sz[bb]; i++) {
        const double y = w.yv[(size_t)bb * w.SM + i];
        ss = fma(y, y, ss);
      }
  }
  return sqrt(__shfl(ss, 0, WAVE));
}

// rz = g + Yᵀλ, λ the active rows of (nu, lc)
template <class M>
__device__ void pn_form_r(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                          const double* nu, const double* lc, double* Yz, int nb, int lane) {
  constexpr int n = M::n, m = M::m;
  pn_gather_duals(P, w, nu, lc, w.lb, nb, lane);
  pn_yt<M>(P, Bf, b, w, X, w.lb, w.rz, Yz, lane);
  for (int e = lane; e < P->N * (n + m); e += WAVE) w.rz[e] = w.g[e] + w.rz[e];
  pn_sync();
}

// multiplier_projection! (:407-420): λ += -(Y Yᵀ) \ (Y (g + Yᵀλ)); returns the residual norm after it
template <class M>
__device__ double pn_multiplier_projection(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w,
                                           const double* X, double* nu, double* lc, PNLds& sh, int nb, int lane,
                                           int& err) {
  pn_form_r<M>(P, Bf, b, w, X, nu, lc, sh.Yz, nb, lane);
  pn_ymul<M>(P, Bf, b, w, X, w.rz, w.tb, sh.Yz, nb, lane);
  pn_build_S<M, true>(P, Bf, b, w, X, sh.Yz, nb, lane);
  PNView w2 = w;
  w2.Ld = w.Ld2;
  w2.Lo = w.Lo2;
  if (pn_factor(w2, nb, 0.0, sh.A, sh.Bm, sh.Cm, lane)) {
    err = 1;  // Y Yᵀ not positive definite
    return NAN;
  }
  pn_fsolve(w2, nb, w.tb, w.xv, sh.A, sh.Bm, sh.vec, lane);
  for (int bb = 0; bb < nb; bb++)
    if (lane < w.sz[bb]) w.lb[(size_t)bb * w.SM + lane] = w.lb[(size_t)bb * w.SM + lane] + -w.xv[(size_t)bb * w.SM + lane];
  pn_sync();
  pn_scatter_duals(P, w, w.lb, nu, lc, nb, lane);
  pn_form_r<M>(P, Bf, b, w, X, nu, lc, sh.Yz, nb, lane);
  return pn_res_norm(P, w, nb, lane);
}

// solveKKT_Shur (:436-452): δλ = L \ (y - Y H⁻¹ r) with stats[:S]'s factor, δz = -H⁻¹ (r + Yᵀδλ)
template <class M>
__device__ void pn_kkt(const DevProblem* P, const DevBuffers& Bf, long long b, const PNView& w, const double* X,
                       PNLds& sh, int nb, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N;
  for (int e = lane; e < N * (n + m); e += WAVE) {
    const int j = e / (n + m), v = e % (n + m);
    if (j == N - 1 && v >= n) continue;
    const double wv = v < n ? pn_wx<M>(P, w, j, v) : pn_wu<M>(P, w, j, v - n);
    w.dz[e] = wv * w.rz[e];
  }
  pn_sync();
  pn_ymul<M>(P, Bf, b, w, X, w.dz, w.tb, sh.Yz, nb, lane);
  for (int bb = 0; bb < nb; bb++)
    if (lane < w.sz[bb]) w.tb[(size_t)bb * w.SM + lane] = w.yv[(size_t)bb * w.SM + lane] - w.tb[(size_t)bb * w.SM + lane];
  pn_sync();
  pn_fsolve(w, nb, w.tb, w.xv, sh.A, sh.Bm, sh.vec, lane);
  pn_yt<M>(P, Bf, b, w, X, w.xv, w.dz, sh.Yz, lane);
  for (int e = lane; e < N * (n + m); e += WAVE) {
    const int j = e / (n + m), v = e % (n + m);
    if (j == N - 1 && v >= n) continue;
    const double wv = v < n ? pn_wx<M>(P, w, j, v) : pn_wu<M>(P, w, j, v - n);
    w.dz[e] = -(wv * (w.rz[e] + w.dz[e]));
  }
  for (int e = lane; e < N * n; e += WAVE) w.dnu[e] = 0.0;
  for (int e = lane; e < N * P->pmax; e += WAVE) w.dlc[e] = 0.0;
  pn_sync();
  pn_scatter_duals(P, w, w.xv, w.dnu, w.dlc, nb, lane);
}

// V_ = solver.V + α δV into X, U and the trial duals
template <class M>
__device__ void pn_ls_trial(const DevProblem* P, const PNView& w, double* X, double* U, double alpha, int lane) {
  constexpr int n = M::n, m = M::m;
  const int N = P->N, pm = P->pmax;
  for (int e = lane; e < N * n; e += WAVE) X[e] = w.Xv[e] + alpha * w.dz[(size_t)(e / n) * (n + m) + e % n];
  for (int e = lane; e < (N - 1) * m; e += WAVE) U[e] = w.Uv[e] + alpha * w.dz[(size_t)(e / m) * (n + m) + n + e % m];
  for (int e = lane; e < N * n; e += WAVE) w.nut[e] = w.nu[e] + alpha * w.dnu[e];
  for (int e = lane; e < N * pm; e += WAVE) w.lct[e] = w.lc[e] + alpha * w.dlc[e];
  pn_sync();
}

// line_search's failure: return solver.V
template <class M>
__device__ void pn_ls_restore(const DevProblem* P, const PNView& w, double* X, double* U, int lane) {
  const int N = P->N;
  for (int e = lane; e < N * M::n; e += WAVE) X[e] = w.Xv[e];
  for (int e = lane; e < (N - 1) * M::m; e += WAVE) U[e] = w.Uv[e];
  pn_sync();
}

// after projection_solve! (k_jacobian left Jacobians at w.Xs in AB): cost_expansion!, multiplier_projection!,
// solveKKT_Shur at solver.V
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_kkt(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNLds sh = pn_lds(W.SM, M::n + M::m);
  PNState s = W.st[b];
  if (!W.optimal || s.finished || s.error) return;
  const int N = P->N, nb = W.nb;
  const PNView w = pn_view(W, P, b);
  // stats[:S] must exist (KeyError) and, when this step did not project, match the active set's blocks
  int mismatch = 0;
  if (s.has_S && s.count == 0)
    for (int bb = lane; bb < nb; bb += WAVE) mismatch |= (w.szS[bb] != w.sz[bb]);
  mismatch = __syncthreads_or(mismatch);
  int err = (!s.has_S || mismatch) ? 1 : 0;
  if (!err) {
    pn_grad<M>(P, w, Bf.X + (size_t)b * N * M::n, Bf.U + (size_t)b * (N - 1) * M::m, lane);
    pn_multiplier_projection<M>(P, Bf, b, w, w.Xs, w.nu, w.lc, sh, nb, lane, err);
  }
  if (!err) pn_kkt<M>(P, Bf, b, w, w.Xs, sh, nb, lane);
  if (lane == 0) {
    if (err) {
      s.error = 1;
    } else {
      s.ls = 1;
      Bf.st[b].active = 1;  // line_search's update!: Jacobians at solver.V
    }
    W.st[b] = s;
  }
}

// line_search (:463-472): update! at solver.V, res0, the first trial V_ = V + δV
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_ls_begin(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNLds sh = pn_lds(W.SM, M::n + M::m);
  PNState s = W.st[b];
  if (!W.optimal || s.finished || s.error || s.ls != 1) return;
  const int N = P->N, nb = W.nb;
  const PNView w = pn_view(W, P, b);
  double* X = Bf.X + (size_t)b * N * M::n;
  double* U = Bf.U + (size_t)b * (N - 1) * M::m;
  for (int e = lane; e < N * M::n; e += WAVE) w.Xv[e] = X[e];
  for (int e = lane; e < (N - 1) * M::m; e += WAVE) w.Uv[e] = U[e];
  // update!'s cost_expansion! at solver.V: a minimum-time problem's H for the first trial's projection!
  if constexpr (ModelTraits<M>::min_time) pn_weights_min_time<M>(P, w, X, U, lane);
  pn_eval<M, INTEG>(P, Bf, b, w, X, U, lane);
  if (pn_active_set(P, Bf, b, w, W.atol, nb, lane)) return pn_stop_over(s, &W.st[b], Bf.st[b], lane);
  pn_gather_y(P, Bf, b, w, nb, lane);
  pn_grad<M>(P, w, X, U, lane);
  pn_form_r<M>(P, Bf, b, w, X, w.nu, w.lc, sh.Yz, nb, lane);
  const double res0 = pn_res_norm(P, w, nb, lane);
  pn_ls_trial<M>(P, w, X, U, 1.0, lane);
  if (lane == 0) {
    s.res0 = res0;
    s.alpha = 1.0;
    s.ls_count = 0;
    s.pcount = 0;
    s.ls = 2;
    W.st[b] = s;  // k_jacobian stays on: the trial's Jacobians
  }
}

// one pass of projection! (:328-357) at the trial (Jacobians from k_jacobian there): stop on viol < eps or
// after 11 Newton steps, else δZ = -H⁻¹Yᵀ (Y H⁻¹ Yᵀ) \ y
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_ls_proj(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNLds sh = pn_lds(W.SM, M::n + M::m);
  PNState s = W.st[b];
  if (!W.optimal || s.finished || s.error || s.ls != 2) return;
  constexpr int n = M::n, m = M::m;
  const int N = P->N, nb = W.nb;
  const PNView w = pn_view(W, P, b);
  double* X = Bf.X + (size_t)b * N * n;
  double* U = Bf.U + (size_t)b * (N - 1) * m;
  pn_eval<M, INTEG>(P, Bf, b, w, X, U, lane);
  if (pn_active_set(P, Bf, b, w, W.atol, nb, lane)) return pn_stop_over(s, &W.st[b], Bf.st[b], lane);
  const double viol = pn_gather_y(P, Bf, b, w, nb, lane);
  if (viol < W.eps || s.pcount > 10) {
    if (lane == 0) {
      s.ls = 3;
      Bf.st[b].active = 0;  // AB keeps the Jacobians at the projected trial
      W.st[b] = s;
    }
    return;
  }
  pn_build_S<M>(P, Bf, b, w, X, sh.Yz, nb, lane);
  PNView w2 = w;
  w2.Ld = w.Ld2;
  w2.Lo = w.Lo2;
  if (pn_factor(w2, nb, 0.0, sh.A, sh.Bm, sh.Cm, lane)) {
    if (lane == 0) {  // the trial is rejected (oracle pn_line_search: more active rows than free variables)
      s.ls = 4;
      Bf.st[b].active = 0;
      W.st[b] = s;
    }
    return;
  }
  pn_fsolve(w2, nb, w.yv, w.xv, sh.A, sh.Bm, sh.vec, lane);
  pn_yt<M>(P, Bf, b, w, X, w.xv, w.rz, sh.Yz, lane);
  for (int e = lane; e < N * (n + m); e += WAVE) {
    const int j = e / (n + m), v = e % (n + m);
    if (j == N - 1 && v >= n) continue;
    const double wv = v < n ? pn_wx<M>(P, w, j, v) : pn_wu<M>(P, w, j, v - n);
    const double dz = -(wv * w.rz[e]);
    if (v < n)
      X[(size_t)j * n + v] = X[(size_t)j * n + v] + dz;
    else
      U[(size_t)j * m + (v - n)] = U[(size_t)j * m + (v - n)] + dz;
  }
  if (lane == 0) {
    s.pcount++;
    W.st[b] = s;
  }
}

// line_search (:478-494) after projection!: cost_expansion! and multiplier_projection! at V_, the test
// res < (1 - 0.01 α) res0, else α /= 2 and the next trial; after 10 trials solver.V. A trial whose
// Y H⁻¹ Yᵀ or Y Yᵀ does not factor is rejected (the oracle's pn_line_search).
template <class M, int INTEG>
__global__ void __launch_bounds__(64) k_pn_ls_end(const DevProblem* __restrict__ P, DevBuffers Bf, PNBuffers W) {
  const long long b = blockIdx.x;
  const int lane = threadIdx.x;
  PNLds sh = pn_lds(W.SM, M::n + M::m);
  PNState s = W.st[b];
  if (!W.optimal || s.finished || s.error || (s.ls != 3 && s.ls != 4)) return;
  const int N = P->N, nb = W.nb;
  const PNView w = pn_view(W, P, b);
  double* X = Bf.X + (size_t)b * N * M::n;
  double* U = Bf.U + (size_t)b * (N - 1) * M::m;
  int rejected = s.ls == 4;  // projection!'s Y H⁻¹ Yᵀ did not factor
  double res = NAN;
  if (!rejected) {
    pn_grad<M>(P, w, X, U, lane);
    // cost_expansion!(prob, solver, V_): a minimum-time problem's H at the trial, the next trial's projection!'s
    if constexpr (ModelTraits<M>::min_time) pn_weights_min_time<M>(P, w, X, U, lane);
    res = pn_multiplier_projection<M>(P, Bf, b, w, X, w.nut, w.lct, sh, nb, lane, rejected);
  }
  int next = 0;
  if (!rejected && res < (1.0 - s.alpha * 0.01) * s.res0) {
    s.ls = 0;  // V_ accepted: prob = V_
  } else {
    s.alpha /= 2.0;
    s.ls_count++;
    if (s.ls_count >= 10) {
      pn_ls_restore<M>(P, w, X, U, lane);
      s.ls = 0;
    } else {
      pn_ls_trial<M>(P, w, X, U, s.alpha, lane);
      s.pcount = 0;
      s.ls = 2;
      next = 1;
    }
  }
  if (lane == 0) {
    if (next) Bf.st[b].active = 1;
    W.st[b] = s;
  }
}

}  // namespace tog
