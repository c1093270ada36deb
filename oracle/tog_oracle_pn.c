/* tog_oracle_pn.c — CPU oracle of ALTRO phase 2, the projected Newton feasible projection.
 * TEST INFRASTRUCTURE ONLY (included by tog_oracle.c; see its header).
 *
 * Restates src/solvers/direct/projected_newton.jl:6-303 for solve_type = :feasible (the default of
 * ProjectedNewtonSolverOptions, src/solvers/direct/direct_solvers.jl:14-30):
 *   solve!            :6-20    n_steps newton steps, record_iteration!, break on c_max <= tol
 *   newton_step!      :484-501 update!, projection_solve!, return (feasible)
 *   projection_solve! :198-210 while count < 10 && viol > eps: _projection_solve!
 *   _projection_solve!:213-254 Jacobians at V, active set, S = Y H⁻¹ Yᵀ, Sreg = cholesky(S + 1e-2 I),
 *                              up to 10 line searches, stop on log10 rate < 1.1 or viol < eps
 *   _projection_linesearch! :256-284 δλ = reg_solve(S, y, Sreg, 1e-8, 25), δZ = -H⁻¹Yᵀδλ
 *   reg_solve         :286-303 iterative refinement of Sreg \ y towards S \ y
 * Dual ordering (direct_solvers.jl:80-105, primals.jl:175-184): blocks G_0 = x_1 - x0 (n rows),
 * G_b = [f(x_b,u_b) - x_{b+1}; active C_b] for b = 1..N-1 (1-based knots), G_N = active C_N. In this
 * order S is block tridiagonal; the reference hands the same matrix to CHOLMOD, this restatement
 * (and the device kernel, bit for bit) factors it block by block:
 *   L_00 = chol(S_00 + ρI); Lo_b = S_{b,b-1} L_{b-1}^{-T}; L_bb = chol(S_bb + ρI - Lo_b Lo_bᵀ).
 * reg_solve refines towards S⁻¹y to |r|₂ < 1e-8, so the two factorizations reach the same δλ to that
 * tolerance.
 *
 * Arithmetic contract with k_pn_solve (tog_pn.hpp): every entry is one sequential fma chain in the
 * index order written here; H⁻¹ is applied as w = 1/h (h = Q_ii·dt, R_ii·dt, Qf_ii: the diagonal of
 * solver.H, cost.jl:214-228). */

typedef struct {
  int n, m, N, SM, nb;        /* SM = n + pmax (largest block); nb = N + 1 blocks */
  int* sz;                    /* block sizes */
  int* act;                   /* active constraint rows per knot: act[k*pmax + r] = row index */
  int* na;                    /* active count per knot */
  double *Sd, *So, *Ld, *Lo;  /* (nb, SM, SM) each, column-major SM x SM */
  double *yv, *xv, *rv, *wv, *dv; /* (nb, SM) */
  double *yd;                 /* dynamics rows (N, n): yd[0] = x_1 - x0, yd[k+1] = f(x_k,u_k) - x_{k+1} */
  double *Cv;                 /* constraint values (N, pmax) */
  double *Xt, *Ut;            /* trial point */
  double *Xs, *Us;            /* the point S and HinvY were formed at (fixed through the line searches) */
  double *wx, *wu;            /* H⁻¹ diagonal: wx (N, n), wu (N-1, m) */
  int refinements, linesearches, projections, error;
  /* solve_type :optimal (newton_step!'s KKT step, projected_newton.jl:501-547) */
  double *Ld2, *Lo2;          /* (nb, SM, SM) factor of Y Yᵀ / of S without regularization */
  double *lb, *tb;            /* (nb, SM) active duals in block order, scratch */
  int* szS;                   /* block sizes of the factor in Ld, Lo (solver.stats[:S]) */
  int has_S;                  /* a _projection_solve! has set solver.stats[:S] */
  double *g, *rz, *dz;        /* (N, n+m): cost gradient, g + Yᵀλ, δz */
  double *nu, *lc;            /* duals of solver.V: dynamics rows (N, n), constraint rows (N, P) */
  double *dnu, *dlc;          /* δV's duals (zero off the KKT step's active set) */
  double *nut, *lct;          /* duals of the line search's V_ */
  double *Xv, *Uv;            /* solver.V's primals while the line search moves the current point */
} pn_ws;

#define PNM(A, b, i, j) ((A)[((size_t)(b) * ws->SM + (j)) * ws->SM + (i)])
#define PNV(v, b, i) ((v)[(size_t)(b) * ws->SM + (i)])

/* dynamics_constraints! + update_constraints! (projected_newton.jl:36-44,67-73) at (X, U) */
static void pn_eval(oc_solver* s, pn_ws* ws, const double* X, const double* U) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  for (int i = 0; i < n; i++) ws->yd[i] = X[i] - s->x0[i];
  for (int k = 0; k < N - 1; k++) {
    double xn[16];
    traj_f(s, xn, X + (size_t)k * n, U + (size_t)k * m);
    for (int i = 0; i < n; i++) ws->yd[(size_t)(k + 1) * n + i] = xn[i] - X[(size_t)(k + 1) * n + i];
  }
  for (int k = 0; k < N; k++)
    if (s->p[k]) set_eval(s, k, X + (size_t)k * n, k < N - 1 ? U + (size_t)k * m : NULL, ws->Cv + (size_t)k * P, NULL,
                          NULL, NULL);
}

/* the active residual vector y[a] in block order, and its Inf norm (NaN propagates) */
static double pn_gather_y(oc_solver* s, pn_ws* ws) {
  int n = s->n, N = s->N, P = s->pmax;
  double viol = 0.0;
  for (int b = 0; b <= N; b++) {
    int r = 0;
    if (b < N)
      for (int i = 0; i < n; i++) PNV(ws->yv, b, r++) = ws->yd[(size_t)b * n + i];
    if (b >= 1) {
      int k = b - 1;
      for (int q = 0; q < ws->na[k]; q++) PNV(ws->yv, b, r++) = ws->Cv[(size_t)k * P + ws->act[k * P + q]];
    }
    for (int i = 0; i < ws->sz[b]; i++) viol = tog_jlmax(viol, fabs(PNV(ws->yv, b, i)));
  }
  return viol;
}

/* active_set! (projected_newton.jl:75-93): equality rows, and inequality rows with c >= -tol */
static void pn_active_set(oc_solver* s, pn_ws* ws, double tol) {
  int n = s->n, N = s->N, P = s->pmax;
  for (int k = 0; k < N; k++) {
    int c = 0;
    for (int i = 0; i < s->p[k]; i++) {
      size_t j = (size_t)k * P + i;
      if (!s->ineq[j] || ws->Cv[j] >= -tol) ws->act[k * P + c++] = i;
    }
    ws->na[k] = c;
  }
  for (int b = 0; b <= N; b++) ws->sz[b] = (b < N ? n : 0) + (b >= 1 ? ws->na[b - 1] : 0);
}

/* rows of block b on its own variables z = (x_j, u_j), j = b-1 (dense s x (n+m), ld SM):
   dynamics rows [A_j B_j], active constraint rows [Cx_j Cu_j]; b = N: terminal rows [Cx]. */
static void pn_block_rows(oc_solver* s, pn_ws* ws, int b, const double* X, const double* U, double* Yz) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax, SM = ws->SM, L = n + m + 1;
  int j = b - 1, r = 0;
  for (int e = 0; e < SM * (n + m); e++) Yz[e] = 0.0;
  if (b < N) {
    const double* F = s->F + (size_t)j * n * L;
    for (int i = 0; i < n; i++, r++)
      for (int v = 0; v < n + m; v++) Yz[r + SM * v] = F[i + n * v];
  }
  if (ws->na[j]) {
    double c[256], Jx[256 * 16], Ju[256 * OM];
    int p = set_eval(s, j, X + (size_t)j * n, j < N - 1 ? U + (size_t)j * m : NULL, c, Jx, j < N - 1 ? Ju : NULL, NULL);
    for (int q = 0; q < ws->na[j]; q++, r++) {
      int row = ws->act[j * P + q];
      for (int v = 0; v < n; v++) Yz[r + SM * v] = Jx[row + p * v];
      if (j < N - 1)
        for (int v = 0; v < m; v++) Yz[r + SM * (n + v)] = Ju[row + p * v];
    }
  }
}

/* S blocks (projected_newton.jl:233-234 with the block structure of _buildShurCompliment!,
   :728-757): Sd_b = Y_b W Y_bᵀ (+ W_{x_{j+1}} on the dynamics diagonal), So_b = S_{b,b-1}. */
static void pn_build_S(oc_solver* s, pn_ws* ws, const double* X, const double* U, int unit) {
  int n = s->n, m = s->m, N = s->N, SM = ws->SM;
  double* Yz = malloc(sizeof(double) * SM * (n + m));
  /* b = 0: S_00 = W_{x_0} */
  for (int e = 0; e < SM * SM; e++) PNM(ws->Sd, 0, e % SM, e / SM) = 0.0;
  for (int i = 0; i < n; i++) PNM(ws->Sd, 0, i, i) = unit ? 1.0 : ws->wx[i];
  for (int b = 1; b <= N; b++) {
    int j = b - 1, sb = ws->sz[b], nv = (b < N) ? n + m : n;
    const double* wxj = ws->wx + (size_t)j * n;
    pn_block_rows(s, ws, b, X, U, Yz);
    for (int l = 0; l < sb; l++)
      for (int i = 0; i < sb; i++) {
        double acc = 0.0;
        for (int v = 0; v < nv; v++) {
          double w = unit ? 1.0 : v < n ? wxj[v] : ws->wu[(size_t)j * m + (v - n)];
          acc = fma(Yz[i + SM * v], w * Yz[l + SM * v], acc);
        }
        if (b < N && i < n && i == l) acc = acc + (unit ? 1.0 : ws->wx[(size_t)(j + 1) * n + i]);
        PNM(ws->Sd, b, i, l) = acc;
      }
    /* So_b[i, c] = Y_b[i, x_j c] · (±w_{x_j c}) for the first n columns of G_{b-1} (+ for the initial
       condition block, - for a dynamics block), 0 on its constraint columns */
    double sg = (b - 1 == 0) ? 1.0 : -1.0;
    int sp = ws->sz[b - 1];
    for (int c = 0; c < sp; c++)
      for (int i = 0; i < sb; i++) PNM(ws->So, b, i, c) = (c < n) ? Yz[i + SM * c] * (sg * (unit ? 1.0 : wxj[c])) : 0.0;
  }
  free(Yz);
}

/* in-place lower Cholesky (right-looking; column j: sqrt, divide, trailing fma updates) */
static int pn_chol(double* M, int s, int ld) {
  for (int j = 0; j < s; j++) {
    double a = M[j + ld * j];
    if (!(a > 0.0)) return j + 1;
    double d = sqrt(a);
    M[j + ld * j] = d;
    for (int i = j + 1; i < s; i++) M[i + ld * j] = M[i + ld * j] / d;
    for (int l = j + 1; l < s; l++)
      for (int i = l; i < s; i++) M[i + ld * l] = fma(-M[i + ld * j], M[l + ld * j], M[i + ld * l]);
  }
  return 0;
}

/* block Cholesky of S + ρI into (Ldf, Lof) */
static int pn_factor_into(pn_ws* ws, double rho, double* Ldf, double* Lof) {
  int SM = ws->SM;
  for (int b = 0; b < ws->nb; b++) {
    int sb = ws->sz[b];
    double* Ld = &PNM(Ldf, b, 0, 0);
    if (b >= 1) {
      int sp = ws->sz[b - 1];
      const double* Lp = &PNM(Ldf, b - 1, 0, 0);
      /* Lo_b = So_b Lp^{-T}: row i solves Lp y = So_b[i, :]ᵀ */
      for (int i = 0; i < sb; i++)
        for (int l = 0; l < sp; l++) {
          double t = PNM(ws->So, b, i, l);
          for (int q = 0; q < l; q++) t = fma(-Lp[l + SM * q], PNM(Lof, b, i, q), t);
          PNM(Lof, b, i, l) = t / Lp[l + SM * l];
        }
    }
    for (int l = 0; l < sb; l++)
      for (int i = l; i < sb; i++) {
        double t = PNM(ws->Sd, b, i, l);
        if (i == l) t = t + rho;
        if (b >= 1)
          for (int q = 0; q < ws->sz[b - 1]; q++) t = fma(-PNM(Lof, b, i, q), PNM(Lof, b, l, q), t);
        Ld[i + SM * l] = t;
      }
    if (pn_chol(Ld, sb, SM)) return b + 1;
  }
  return 0;
}
static int pn_factor(pn_ws* ws, double rho) { return pn_factor_into(ws, rho, ws->Ld, ws->Lo); }

/* x = (S + ρI)⁻¹ r through the block factor (Ldf, Lof) */
static void pn_fsolve_with(pn_ws* ws, const double* Ldf, const double* Lof, const double* r, double* x) {
  for (int b = 0; b < ws->nb; b++) { /* forward: w_b = L_bb⁻¹ (r_b - Lo_b w_{b-1}) */
    int sb = ws->sz[b];
    double t[512];
    for (int i = 0; i < sb; i++) {
      double a = PNV(r, b, i);
      if (b >= 1)
        for (int q = 0; q < ws->sz[b - 1]; q++) a = fma(-PNM(Lof, b, i, q), PNV(ws->wv, b - 1, q), a);
      t[i] = a;
    }
    for (int l = 0; l < sb; l++) {
      double wl = t[l] / PNM(Ldf, b, l, l);
      PNV(ws->wv, b, l) = wl;
      for (int i = l + 1; i < sb; i++) t[i] = fma(-PNM(Ldf, b, i, l), wl, t[i]);
    }
  }
  for (int b = ws->nb - 1; b >= 0; b--) { /* backward: x_b = L_bbᵀ⁻¹ (w_b - Lo_{b+1}ᵀ x_{b+1}) */
    int sb = ws->sz[b];
    double t[512];
    for (int i = 0; i < sb; i++) {
      double a = PNV(ws->wv, b, i);
      if (b + 1 < ws->nb)
        for (int q = 0; q < ws->sz[b + 1]; q++) a = fma(-PNM(Lof, b + 1, q, i), PNV(x, b + 1, q), a);
      t[i] = a;
    }
    for (int l = sb - 1; l >= 0; l--) {
      double xl = t[l] / PNM(Ldf, b, l, l);
      PNV(x, b, l) = xl;
      for (int i = 0; i < l; i++) t[i] = fma(-PNM(Ldf, b, l, i), xl, t[i]);
    }
  }
}
static void pn_fsolve(pn_ws* ws, const double* r, double* x) { pn_fsolve_with(ws, ws->Ld, ws->Lo, r, x); }

/* r = y - S x; returns |r|₂ (sequential sum of squares in block/row order, then sqrt) */
static double pn_residual(pn_ws* ws, const double* y, const double* x, double* r) {
  double ss = 0.0;
  for (int b = 0; b < ws->nb; b++)
    for (int i = 0; i < ws->sz[b]; i++) {
      double t = 0.0;
      for (int q = 0; q < ws->sz[b]; q++) t = fma(PNM(ws->Sd, b, i, q), PNV(x, b, q), t);
      if (b >= 1)
        for (int q = 0; q < ws->sz[b - 1]; q++) t = fma(PNM(ws->So, b, i, q), PNV(x, b - 1, q), t);
      if (b + 1 < ws->nb)
        for (int q = 0; q < ws->sz[b + 1]; q++) t = fma(PNM(ws->So, b + 1, q, i), PNV(x, b + 1, q), t);
      double ri = PNV(y, b, i) - t;
      PNV(r, b, i) = ri;
      ss = fma(ri, ri, ss);
    }
  return sqrt(ss);
}

/* reg_solve(S, y, Sreg, 1e-8, 25) (projected_newton.jl:286-303) into ws->xv */
static void pn_reg_solve(pn_ws* ws) {
  pn_fsolve(ws, ws->yv, ws->xv);
  for (int cnt = 0; cnt < 25; cnt++) {
    double nr = pn_residual(ws, ws->yv, ws->xv, ws->rv);
    if (nr < 1e-8) break;
    pn_fsolve(ws, ws->rv, ws->dv);
    for (int b = 0; b < ws->nb; b++)
      for (int i = 0; i < ws->sz[b]; i++) PNV(ws->xv, b, i) = PNV(ws->xv, b, i) + PNV(ws->dv, b, i);
    ws->refinements++;
  }
}

/* trial point Z_ = Z + α δZ, δZ = -H⁻¹ Yᵀ δλ (δλ = ws->xv) */
static void pn_trial(oc_solver* s, pn_ws* ws, double alpha) {
  int n = s->n, m = s->m, N = s->N, SM = ws->SM;
  double* Yz = malloc(sizeof(double) * SM * (n + m));
  for (int j = 0; j < N; j++) {
    int b = j + 1; /* the block whose own variables are z_j */
    pn_block_rows(s, ws, b, ws->Xs, ws->Us, Yz); /* HinvY of _projection_solve!: Jacobians at its start */
    int nv = (j < N - 1) ? n + m : n;
    for (int v = 0; v < nv; v++) {
      double t;
      if (v < n) /* x_j in block j: +I (initial condition) or -I (dynamics of knot j-1) */
        t = (j == 0) ? PNV(ws->xv, 0, v) : -PNV(ws->xv, j, v);
      else
        t = 0.0;
      for (int i = 0; i < ws->sz[b]; i++) t = fma(Yz[i + SM * v], PNV(ws->xv, b, i), t);
      double w = v < n ? ws->wx[(size_t)j * n + v] : ws->wu[(size_t)j * m + (v - n)];
      double dz = -(w * t);
      if (v < n)
        ws->Xt[(size_t)j * n + v] = s->X[(size_t)j * n + v] + alpha * dz;
      else
        ws->Ut[(size_t)j * m + (v - n)] = s->U[(size_t)j * m + (v - n)] + alpha * dz;
    }
  }
  free(Yz);
}

/* _projection_linesearch! (projected_newton.jl:256-284); returns viol, sets ws->error */
static double pn_linesearch(oc_solver* s, pn_ws* ws) {
  int n = s->n, m = s->m, N = s->N;
  double viol0 = pn_gather_y(s, ws);
  ws->linesearches++;
  pn_reg_solve(ws);
  pn_trial(s, ws, 1.0);
  pn_eval(s, ws, ws->Xt, ws->Ut);
  double viol = pn_gather_y(s, ws);
  if (!(viol < viol0)) {
    /* `count += a` with a::BitVector: MethodError in the reference */
    ws->error = 1;
    return viol;
  }
  memcpy(s->X, ws->Xt, sizeof(double) * n * N);
  memcpy(s->U, ws->Ut, sizeof(double) * m * (N - 1));
  return viol;
}

/* _projection_solve! (projected_newton.jl:213-254) */
static double pn_projection_solve(oc_solver* s, pn_ws* ws, double tol_active, double eps) {
  ws->projections++;
  memcpy(ws->Xs, s->X, sizeof(double) * s->n * s->N);
  memcpy(ws->Us, s->U, sizeof(double) * s->m * (s->N - 1));
  pn_eval(s, ws, s->X, s->U);
  oc_jacobians(s);
  pn_active_set(s, ws, tol_active);
  double viol0 = pn_gather_y(s, ws);
  pn_build_S(s, ws, s->X, s->U, 0);
  if (pn_factor(ws, 1e-2)) {
    ws->error = 1; /* PosDefException in cholesky */
    return viol0;
  }
  ws->has_S = 1; /* solver.stats[:S] = Sreg */
  memcpy(ws->szS, ws->sz, sizeof(int) * ws->nb);
  double viol_prev = viol0;
  for (int count = 0; count < 10; count++) {
    double viol = pn_linesearch(s, ws);
    if (ws->error) return viol;
    double rate = log10(viol) / log10(viol_prev);
    viol_prev = viol;
    if (rate < 1.1 || viol < eps) break;
  }
  return viol_prev;
}

/* ---------------------------------------------------------------------------------------------------
 * solve_type :optimal: newton_step! after the projection (projected_newton.jl:522-546): cost_expansion!,
 * multiplier_projection! (:407-420), solveKKT_Shur (:436-452) with solver.stats[:S] (the last
 * _projection_solve!'s cholesky(S + 1e-2 I)), line_search (:463-496) with projection! (:328-357) at each
 * trial. The primal vector is indexed z[j (n+m) + v] (knot j, v < n state, v >= n control); duals keep
 * the reference's full layout (every constraint row, active or not; PrimalDual, primals.jl:158-192).
 * Solves of Y Yᵀ and Y H⁻¹ Yᵀ (the reference's sparse backslash) go through the same block Cholesky
 * without regularization; norms are the sequential sum of squares (the reference's BLAS nrm2 agrees to
 * rounding: unpinned at the last bit).
 * ------------------------------------------------------------------------------------------------- */
#define PNZ(j) ((size_t)(j) * (n + m))

/* the cost gradient g (cost_expansion!'s gradient!, :139-148) at (X, U): the plain objective's Q.x, Q.u */
static void pn_grad(oc_solver* s, pn_ws* ws, double* X, double* U) {
  int n = s->n, m = s->m, N = s->N;
  double *sx = s->X, *su = s->U;
  s->X = X;
  s->U = U;
  for (int k = 0; k < N - 1; k++) expansion_stage(s, k);
  expansion_terminal(s);
  s->X = sx;
  s->U = su;
  for (int j = 0; j < N; j++) {
    for (int v = 0; v < n; v++) ws->g[PNZ(j) + v] = s->Qx[(size_t)j * n + v];
    if (j < N - 1)
      for (int v = 0; v < m; v++) ws->g[PNZ(j) + n + v] = s->Qu[(size_t)j * m + v];
  }
}

/* duals (full layout) -> active duals in block order (lb), and back */
static void pn_gather_duals(oc_solver* s, pn_ws* ws, const double* nu, const double* lc, double* lb) {
  int n = s->n, N = s->N, P = s->pmax;
  for (int b = 0; b <= N; b++) {
    int r = 0;
    if (b < N)
      for (int i = 0; i < n; i++) PNV(lb, b, r++) = nu[(size_t)b * n + i];
    if (b >= 1)
      for (int q = 0; q < ws->na[b - 1]; q++) PNV(lb, b, r++) = lc[(size_t)(b - 1) * P + ws->act[(b - 1) * P + q]];
  }
}
static void pn_scatter_duals(oc_solver* s, pn_ws* ws, const double* lb, double* nu, double* lc) {
  int n = s->n, N = s->N, P = s->pmax;
  for (int b = 0; b <= N; b++) {
    int r = 0;
    if (b < N)
      for (int i = 0; i < n; i++) nu[(size_t)b * n + i] = PNV(lb, b, r++);
    if (b >= 1)
      for (int q = 0; q < ws->na[b - 1]; q++) lc[(size_t)(b - 1) * P + ws->act[(b - 1) * P + q]] = PNV(lb, b, r++);
  }
}

/* out = Yᵀ l (l active duals in block order): column z_j gets ±l_j (initial condition +I, dynamics -I of
   block j) and then block j+1's rows on its own variables, in row order */
static void pn_yt(oc_solver* s, pn_ws* ws, const double* X, const double* U, const double* l, double* out) {
  int n = s->n, m = s->m, N = s->N, SM = ws->SM;
  double* Yz = malloc(sizeof(double) * SM * (n + m));
  for (int j = 0; j < N; j++) {
    int b = j + 1, nv = (j < N - 1) ? n + m : n;
    pn_block_rows(s, ws, b, X, U, Yz);
    for (int v = 0; v < nv; v++) {
      double t = (v < n) ? ((j == 0) ? PNV(l, 0, v) : -PNV(l, j, v)) : 0.0;
      for (int i = 0; i < ws->sz[b]; i++) t = fma(Yz[i + SM * v], PNV(l, b, i), t);
      out[PNZ(j) + v] = t;
    }
  }
  free(Yz);
}

/* out = Y z (block order): row i of block b starts from its ±I term, then block b's own variables z_{b-1} */
static void pn_ymul(oc_solver* s, pn_ws* ws, const double* X, const double* U, const double* z, double* out) {
  int n = s->n, m = s->m, N = s->N, SM = ws->SM;
  double* Yz = malloc(sizeof(double) * SM * (n + m));
  for (int b = 0; b <= N; b++) {
    int j = b - 1, nv = (j < N - 1) ? n + m : n;
    if (b >= 1) pn_block_rows(s, ws, b, X, U, Yz);
    for (int i = 0; i < ws->sz[b]; i++) {
      double t = (b < N && i < n) ? ((b == 0) ? z[i] : -z[PNZ(b) + i]) : 0.0;
      if (b >= 1)
        for (int v = 0; v < nv; v++) t = fma(Yz[i + SM * v], z[PNZ(j) + v], t);
      PNV(out, b, i) = t;
    }
  }
  free(Yz);
}

/* |[g + Yᵀλ; y]|₂ (residual, :454-460) with rz = g + Yᵀλ already formed */
static double pn_res_norm(oc_solver* s, pn_ws* ws) {
  int n = s->n, m = s->m, N = s->N;
  double ss = 0.0;
  for (int j = 0; j < N; j++)
    for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) ss = fma(ws->rz[PNZ(j) + v], ws->rz[PNZ(j) + v], ss);
  for (int b = 0; b <= N; b++)
    for (int i = 0; i < ws->sz[b]; i++) ss = fma(PNV(ws->yv, b, i), PNV(ws->yv, b, i), ss);
  return sqrt(ss);
}

/* rz = g + Yᵀλ at the current point (Jacobians s->F, constraint rows at X, U), λ the duals' active rows */
static void pn_form_r(oc_solver* s, pn_ws* ws, const double* X, const double* U, const double* nu, const double* lc) {
  int n = s->n, m = s->m, N = s->N;
  pn_gather_duals(s, ws, nu, lc, ws->lb);
  pn_yt(s, ws, X, U, ws->lb, ws->rz);
  for (int j = 0; j < N; j++)
    for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) ws->rz[PNZ(j) + v] = ws->g[PNZ(j) + v] + ws->rz[PNZ(j) + v];
}

/* multiplier_projection! (:407-420): δλ = -(Y Yᵀ) \ (Y (g + Yᵀλ)), λ += δλ on the active rows; returns the
   residual norm after it, or NaN with *fail set when Y Yᵀ does not factor (rank-deficient active rows) */
static double pn_multiplier_projection(oc_solver* s, pn_ws* ws, const double* X, const double* U, double* nu, double* lc,
                                       int* fail) {
  pn_form_r(s, ws, X, U, nu, lc);
  pn_ymul(s, ws, X, U, ws->rz, ws->tb);
  pn_build_S(s, ws, X, U, 1);
  if (pn_factor_into(ws, 0.0, ws->Ld2, ws->Lo2)) {
    *fail = 1;
    return NAN;
  }
  pn_fsolve_with(ws, ws->Ld2, ws->Lo2, ws->tb, ws->xv);
  for (int b = 0; b < ws->nb; b++)
    for (int i = 0; i < ws->sz[b]; i++) PNV(ws->lb, b, i) = PNV(ws->lb, b, i) + -PNV(ws->xv, b, i);
  pn_scatter_duals(s, ws, ws->lb, nu, lc);
  pn_form_r(s, ws, X, U, nu, lc);
  return pn_res_norm(s, ws);
}

/* solveKKT_Shur (:436-452) at the current point: r = g + Yᵀλ, δλ = L \ (y - Y H⁻¹ r), δz = -H⁻¹ (r + Yᵀδλ);
   δλ is scattered to the duals' full layout (zero off the active set) */
static void pn_kkt(oc_solver* s, pn_ws* ws, const double* X, const double* U) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  double* hz = ws->dz; /* H⁻¹ r, overwritten by δz below */
  for (int j = 0; j < N; j++)
    for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) {
      double w = v < n ? ws->wx[(size_t)j * n + v] : ws->wu[(size_t)j * m + (v - n)];
      hz[PNZ(j) + v] = w * ws->rz[PNZ(j) + v];
    }
  pn_ymul(s, ws, X, U, hz, ws->tb);
  for (int b = 0; b < ws->nb; b++)
    for (int i = 0; i < ws->sz[b]; i++) PNV(ws->tb, b, i) = PNV(ws->yv, b, i) - PNV(ws->tb, b, i);
  pn_fsolve(ws, ws->tb, ws->xv); /* L \ : the factor of stats[:S] */
  pn_yt(s, ws, X, U, ws->xv, ws->dz);
  for (int j = 0; j < N; j++)
    for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) {
      double w = v < n ? ws->wx[(size_t)j * n + v] : ws->wu[(size_t)j * m + (v - n)];
      ws->dz[PNZ(j) + v] = -(w * (ws->rz[PNZ(j) + v] + ws->dz[PNZ(j) + v]));
    }
  memset(ws->dnu, 0, sizeof(double) * (size_t)N * n);
  memset(ws->dlc, 0, sizeof(double) * (size_t)N * P);
  pn_scatter_duals(s, ws, ws->xv, ws->dnu, ws->dlc);
}

/* update! at the current point (s->X, s->U): dynamics and constraint values, Jacobians, active set, y */
static double pn_update(oc_solver* s, pn_ws* ws, double atol) {
  pn_eval(s, ws, s->X, s->U);
  oc_jacobians(s);
  memcpy(ws->Xs, s->X, sizeof(double) * s->n * s->N);
  memcpy(ws->Us, s->U, sizeof(double) * s->m * (s->N - 1));
  pn_active_set(s, ws, atol);
  return pn_gather_y(s, ws);
}

static void pn_weights_min_time(const oc_solver* s, pn_ws* ws);

/* line_search (:463-496) from solver.V (s->X, s->U, ws->nu, ws->lc) along (δz, δλ); leaves the returned
   V_ (or solver.V) in s->X, s->U and solver.V in ws->Xv, ws->Uv. A trial whose Y H⁻¹ Yᵀ or Y Yᵀ does not
   factor (a KKT step so long that the active rows outnumber the free variables: the reference's sparse
   backslash then returns a useless or non-finite solve) is rejected like one whose residual did not fall. */
static void pn_line_search(oc_solver* s, pn_ws* ws, double atol, double eps) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  const size_t nx = (size_t)N * n, nu_ = (size_t)(N - 1) * m;
  memcpy(ws->Xv, s->X, sizeof(double) * nx);
  memcpy(ws->Uv, s->U, sizeof(double) * nu_);
  pn_update(s, ws, atol);
  /* update!'s cost_expansion! at solver.V: a minimum-time problem's H (MinTimeCost's hessian!) moves with V, and
     projection! of the first trial uses it (H = Diagonal(solver.H), :328-333) */
  if (s->mt) pn_weights_min_time(s, ws);
  pn_grad(s, ws, s->X, s->U);
  pn_form_r(s, ws, s->X, s->U, ws->nu, ws->lc);
  const double res0 = pn_res_norm(s, ws);
  double alpha = 1.0;
  for (int count = 0; count < 10; count++) {
    /* V_ = solver.V + α δV */
    for (int k = 0; k < N; k++)
      for (int i = 0; i < n; i++) s->X[(size_t)k * n + i] = ws->Xv[(size_t)k * n + i] + alpha * ws->dz[PNZ(k) + i];
    for (int k = 0; k < N - 1; k++)
      for (int i = 0; i < m; i++) s->U[(size_t)k * m + i] = ws->Uv[(size_t)k * m + i] + alpha * ws->dz[PNZ(k) + n + i];
    for (size_t e = 0; e < nx; e++) ws->nut[e] = ws->nu[e] + alpha * ws->dnu[e];
    for (size_t e = 0; e < (size_t)N * P; e++) ws->lct[e] = ws->lc[e] + alpha * ws->dlc[e];
    /* projection!: Newton steps onto the active constraints with S = Y H⁻¹ Yᵀ (no regularization) */
    for (int pc = 0;; pc++) {
      double viol = pn_update(s, ws, atol);
      if (viol < eps || pc > 10) break;
      pn_build_S(s, ws, s->X, s->U, 0);
      if (pn_factor_into(ws, 0.0, ws->Ld2, ws->Lo2)) goto reject;
      pn_fsolve_with(ws, ws->Ld2, ws->Lo2, ws->yv, ws->xv);
      pn_yt(s, ws, s->X, s->U, ws->xv, ws->rz);
      for (int j = 0; j < N; j++)
        for (int v = 0; v < ((j < N - 1) ? n + m : n); v++) {
          double w = v < n ? ws->wx[(size_t)j * n + v] : ws->wu[(size_t)j * m + (v - n)];
          double dz = -(w * ws->rz[PNZ(j) + v]);
          if (v < n)
            s->X[(size_t)j * n + v] = s->X[(size_t)j * n + v] + dz;
          else
            s->U[(size_t)j * m + (v - n)] = s->U[(size_t)j * m + (v - n)] + dz;
        }
    }
    pn_grad(s, ws, s->X, s->U);
    if (s->mt) pn_weights_min_time(s, ws); /* cost_expansion!(prob, solver, V_): the next trial's projection! H */
    int fail = 0;
    double res = pn_multiplier_projection(s, ws, s->X, s->U, ws->nut, ws->lct, &fail);
    if (!fail && res < (1.0 - alpha * 0.01) * res0) return;
  reject:
    alpha /= 2.0;
  }
  memcpy(s->X, ws->Xv, sizeof(double) * nx);
  memcpy(s->U, ws->Uv, sizeof(double) * nu_);
}
#undef PNZ

OC_EXPORT void oc_default_pn_options(tog_pn_options* o) {
  o->n_steps = 1;
  o->solve_type = 0;
  o->active_set_tolerance = 1e-3;
  o->feasibility_tolerance = 1e-6;
}

/* H of a minimum-time problem (update!'s cost_expansion!, projected_newton.jl:122-148, at the newton step's
   X, U): MinTimeCost's hessian! (minimum_time.jl:238-280) on the diagonal: Q·h² and R·h² for the model's
   states and controls (dt = h² = u[end]²), R_min_time for τ, 2 ℓ(x, u) + R_min_time for h (ℓ the quadratic
   stage cost without dt), terminal Qf and R_min_time. */
static void pn_weights_min_time(const oc_solver* s, pn_ws* ws) {
  const int n = s->n, m = s->m, N = s->N;
  for (int k = 0; k < N - 1; k++) {
    const double* x = s->X + (size_t)k * n;
    const double* u = s->U + (size_t)k * m;
    const double h = u[m - 1], dt = h * h;
    for (int i = 0; i < n - 1; i++) ws->wx[(size_t)k * n + i] = 1.0 / (kQ(s, k)[IDX(i, i, n)] * dt);
    ws->wx[(size_t)k * n + n - 1] = 1.0 / s->R_mt;
    for (int i = 0; i < m - 1; i++) ws->wu[(size_t)k * m + i] = 1.0 / (kR(s, k)[IDX(i, i, m)] * dt);
    const double l1 = stage_cost(s, k, x, u, 1.0);
    ws->wu[(size_t)k * m + m - 1] = 1.0 / (2.0 * l1 + s->R_mt);
  }
  for (int i = 0; i < n - 1; i++) ws->wx[(size_t)(N - 1) * n + i] = 1.0 / s->Qf[IDX(i, i, n)];
  ws->wx[(size_t)(N - 1) * n + n - 1] = 1.0 / s->R_mt;
}

/* solve!(prob, ProjectedNewtonSolver) (projected_newton.jl:6-20); out: TOG_PN_NSTATS doubles. Returns 0, or
   -4 for an unknown solve_type. A minimum-time problem's H (MinTimeCost's hessian!, its diagonal) is formed at
   each newton step's V (update!) and, under :optimal, again wherever the reference calls cost_expansion!: at
   solver.V when the line search starts and at each projected trial V_ (pn_line_search); solveKKT_Shur keeps the
   newton step's Hinv (:501-547). */
OC_EXPORT int oc_solve_pn(oc_solver* s, const tog_pn_options* o, double* out) {
  const int optimal = o->solve_type == 1;
  if (o->solve_type != 0 && !optimal) return -4;
  int n = s->n, m = s->m, N = s->N, P = s->pmax > 0 ? s->pmax : 1;
  pn_ws W, *ws = &W;
  memset(ws, 0, sizeof(W));
  ws->n = n;
  ws->m = m;
  ws->N = N;
  ws->SM = n + s->pmax;
  ws->nb = N + 1;
  size_t blk = (size_t)ws->nb * ws->SM * ws->SM, vec = (size_t)ws->nb * ws->SM;
  ws->sz = calloc(ws->nb, sizeof(int));
  ws->act = calloc((size_t)N * P, sizeof(int));
  ws->na = calloc(N, sizeof(int));
  ws->Sd = calloc(blk, sizeof(double));
  ws->So = calloc(blk, sizeof(double));
  ws->Ld = calloc(blk, sizeof(double));
  ws->Lo = calloc(blk, sizeof(double));
  ws->yv = calloc(vec, sizeof(double));
  ws->xv = calloc(vec, sizeof(double));
  ws->rv = calloc(vec, sizeof(double));
  ws->wv = calloc(vec, sizeof(double));
  ws->dv = calloc(vec, sizeof(double));
  ws->yd = calloc((size_t)N * n, sizeof(double));
  ws->Cv = calloc((size_t)N * P, sizeof(double));
  ws->Xt = calloc((size_t)N * n, sizeof(double));
  ws->Ut = calloc((size_t)(N - 1) * m, sizeof(double));
  ws->Xs = calloc((size_t)N * n, sizeof(double));
  ws->Us = calloc((size_t)(N - 1) * m, sizeof(double));
  ws->wx = calloc((size_t)N * n, sizeof(double));
  ws->wu = calloc((size_t)(N - 1) * m, sizeof(double));
  ws->Ld2 = calloc(blk, sizeof(double));
  ws->Lo2 = calloc(blk, sizeof(double));
  ws->lb = calloc(vec, sizeof(double));
  ws->tb = calloc(vec, sizeof(double));
  ws->szS = calloc(ws->nb, sizeof(int));
  const size_t nz = (size_t)N * (n + m);
  ws->g = calloc(nz, sizeof(double));
  ws->rz = calloc(nz, sizeof(double));
  ws->dz = calloc(nz, sizeof(double));
  ws->nu = calloc((size_t)N * n, sizeof(double)); /* PrimalDual(prob): zero duals */
  ws->dnu = calloc((size_t)N * n, sizeof(double));
  ws->nut = calloc((size_t)N * n, sizeof(double));
  ws->lc = calloc((size_t)N * P, sizeof(double));
  ws->dlc = calloc((size_t)N * P, sizeof(double));
  ws->lct = calloc((size_t)N * P, sizeof(double));
  ws->Xv = calloc((size_t)N * n, sizeof(double));
  ws->Uv = calloc((size_t)(N - 1) * m, sizeof(double));
  /* H = Diagonal(solver.H): stage Q·dt, R·dt (cost.jl:214-223), terminal Qf (:225-228); per knot (a
     time-varying Objective) */
  for (int k = 0; k < N; k++)
    for (int i = 0; i < n; i++)
      ws->wx[(size_t)k * n + i] = 1.0 / (k < N - 1 ? kQ(s, k)[IDX(i, i, n)] * s->dt : s->Qf[IDX(i, i, n)]);
  for (int k = 0; k < N - 1; k++)
    for (int i = 0; i < m; i++) ws->wu[(size_t)k * m + i] = 1.0 / (kR(s, k)[IDX(i, i, m)] * s->dt);
  double viol = 0.0, c_max = 0.0, J = 0.0;
  int steps = 0;
  s->hpn_n = 0;
  for (int it = 0; it < o->n_steps; it++) {
    if (s->mt) pn_weights_min_time(s, ws);
    /* newton_step!: update! (active set at V), then projection_solve!. :optimal starts every step from
       solver.V, which solve! never moves to the returned V_ (it only copies V_ into prob) */
    if (optimal && it > 0) {
      memcpy(s->X, ws->Xv, sizeof(double) * (size_t)n * N);
      memcpy(s->U, ws->Uv, sizeof(double) * (size_t)m * (N - 1));
    }
    if (optimal) {
      viol = pn_update(s, ws, o->active_set_tolerance);
    } else {
      pn_eval(s, ws, s->X, s->U);
      pn_active_set(s, ws, o->active_set_tolerance);
      viol = pn_gather_y(s, ws);
    }
    int projected = 0;
    for (int count = 0; count < 10 && viol > o->feasibility_tolerance && !ws->error; count++, projected++)
      viol = pn_projection_solve(s, ws, o->active_set_tolerance, o->feasibility_tolerance);
    if (optimal && !ws->error) {
      /* stats[:S] must exist (KeyError otherwise) and match the current active set's blocks (a factor of a
         different layout: DimensionMismatch, or a silently mismatched solve, in the reference) */
      if (!ws->has_S || (!projected && memcmp(ws->szS, ws->sz, sizeof(int) * ws->nb))) ws->error = 1;
    }
    if (optimal && !ws->error) {
      pn_grad(s, ws, s->X, s->U);
      int fail = 0;
      pn_multiplier_projection(s, ws, ws->Xs, ws->Us, ws->nu, ws->lc, &fail);
      if (fail) ws->error = 1; /* Y Yᵀ at solver.V does not factor */
      if (!ws->error) {
        pn_kkt(s, ws, ws->Xs, ws->Us);
        pn_line_search(s, ws, o->active_set_tolerance, o->feasibility_tolerance);
      }
    }
    steps++;
    /* record_iteration!: J = cost(prob), c_max = max_violation(prob) */
    update_constraints(s, s->X, s->U);
    c_max = max_violation(s);
    J = obj_cost(s, s->X, s->U);
    const double rec[2] = {J, c_max};
    hist_push(&s->hpn, &s->hpn_n, &s->hpn_cap, 2, rec);
    if (ws->error || c_max <= o->feasibility_tolerance) break;
  }
  if (ws->error) s->flags |= TOG_TRAJ_PN_ERROR;
  if (out) {
    out[TOG_PN_VIOL] = viol;
    out[TOG_PN_C_MAX] = c_max;
    out[TOG_PN_J] = J;
    out[TOG_PN_PROJECTIONS] = ws->projections;
    out[TOG_PN_LINESEARCHES] = ws->linesearches;
    out[TOG_PN_REFINEMENTS] = ws->refinements;
    out[TOG_PN_STEPS] = steps;
  }
  free(ws->sz); free(ws->act); free(ws->na); free(ws->Sd); free(ws->So); free(ws->Ld); free(ws->Lo);
  free(ws->yv); free(ws->xv); free(ws->rv); free(ws->wv); free(ws->dv); free(ws->yd); free(ws->Cv);
  free(ws->Xt); free(ws->Ut); free(ws->Xs); free(ws->Us); free(ws->wx); free(ws->wu);
  free(ws->Ld2); free(ws->Lo2); free(ws->lb); free(ws->tb); free(ws->szS); free(ws->g); free(ws->rz); free(ws->dz);
  free(ws->nu); free(ws->dnu); free(ws->nut); free(ws->lc); free(ws->dlc); free(ws->lct); free(ws->Xv); free(ws->Uv);
  return 0;
}
#undef PNM
#undef PNV
