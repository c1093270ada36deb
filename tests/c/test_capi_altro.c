/*
 * test_capi_altro.c — a plain C caller of tog_solve_altro (include/tog.h): the reference's quadrotor_maze
 * ALTRO case (problems/quadrotor_maze.jl:1-114, test/infeasible_tests.jl:57-76: an initial state guess,
 * so altro_problem makes it an infeasible-start solve) described exactly as integration/julia/libtog.jl's
 * tog_desc marshals that Problem and tog_altro_options its ALTROSolverOptions:
 *   model  rk3(Dynamics.quadrotor) -> TOG_MODEL_QUADROTOR, TOG_RK3; N = 101, dt = tf/(N-1), tf = 5
 *   obj    LQRObjective(Q, R, Qf, xf, N), Q = 1e-3 I with 1e-2 on the quaternion, R = 1e-4 I, Qf = 1000 I
 *   cons   knot 1: bnd1 (u in [0, 50]); knots 2..N-1: [bnd2, maze] (the 44 cylinders, r + r_quad);
 *          knot N: bnd_xf (the terminal box). Knots sharing a ConstraintSet object share one entry.
 *   opts   ALTROSolverOptions(resolve_feasible_problem=false, R_inf=0.001, opts_al =
 *          AugmentedLagrangianSolverOptions(iterations=40, cost_tolerance=1e-5,
 *          cost_tolerance_intermediate=1e-4, constraint_tolerance=1e-3, penalty_scaling=10, penalty_initial=1))
 * The state guess comes from the caller (initial_states!, src/problem.jl:153-154), as the Julia user would
 * pass it.
 *   test_capi_altro <in.bin> <out.bin>  in: int64 B, x0 (13, B), U0 (4, 100, B), X0 (13, 101, B);
 *                                       out: X (13, 101, B), U (4, 100, B), stats (TOG_NSTATS, B),
 *                                       hist_count (2, B), hist_outer (4, 41, B), hist_inner (3, 12041, B)
 * tests/test_c_caller.py compares out.bin with the Python path (solve_b with ALTROSolverOptions) bit for bit,
 * the iteration histories of tog_solve_altro_ex included.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tog.h"

enum { n = 13, m = 4, N = 101, NCYL = 44 };

static int fail_rc(const char* what, int rc) {
  fprintf(stderr, "%s failed: %d (%s)\n", what, rc, tog_last_error());
  return 1;
}

/* numpy.linspace(a, b, k): a + i (b - a)/(k - 1), the last point exactly b */
static void linspace(double* out, double a, double b, int k) {
  const double step = (b - a) / (k - 1);
  for (int i = 0; i < k; i++) out[i] = (i == k - 1) ? b : i * step + a;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s <in.bin> <out.bin>\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return fail_rc("open input", -1);
  int64_t B = 0;
  if (fread(&B, sizeof(B), 1, f) != 1 || B < 1) return fail_rc("read B", -1);
  const size_t nx0 = (size_t)n * B, nU = (size_t)m * (N - 1) * B, nX = (size_t)n * N * B;
  double* x0 = malloc(sizeof(double) * nx0);
  double* U = malloc(sizeof(double) * nU);
  double* X = malloc(sizeof(double) * nX);
  if (fread(x0, sizeof(double), nx0, f) != nx0 || fread(U, sizeof(double), nU, f) != nU ||
      fread(X, sizeof(double), nX, f) != nX)
    return fail_rc("read x0/U0/X0", -1);
  fclose(f);

  /* LQRObjective(Q, R, Qf, xf, N) (src/objective.jl:102-114) */
  double Q[n * n] = {0}, R[m * m] = {0}, H[m * n] = {0}, q[n], r[m] = {0}, Qf[n * n] = {0}, qf[n], xf[n] = {0};
  for (int i = 0; i < n; i++) Q[i + n * i] = (i >= 3 && i < 7) ? 1e-2 : 1e-3, Qf[i + n * i] = 1000.0;
  for (int i = 0; i < m; i++) R[i + m * i] = 1e-4;
  xf[1] = 60.0;
  xf[2] = 10.0;
  xf[3] = 1.0;
  double c = 0.0, cf = 0.0;
  for (int i = 0; i < n; i++) { /* (-Q) xf and (0.5 xf' Q) xf, left to right as Julia evaluates them */
    double t = 0.0, tf = 0.0;
    for (int j = 0; j < n; j++) {
      t += (-Q[i + n * j]) * xf[j];
      tf += (-Qf[i + n * j]) * xf[j];
    }
    q[i] = t;
    qf[i] = tf;
  }
  {
    double hx[n], hxf[n];
    for (int j = 0; j < n; j++) {
      double t = 0.0, tf = 0.0;
      for (int i = 0; i < n; i++) {
        t += (0.5 * xf[i]) * Q[i + n * j];
        tf += (0.5 * xf[i]) * Qf[i + n * j];
      }
      hx[j] = t;
      hxf[j] = tf;
    }
    for (int j = 0; j < n; j++) {
      c += hx[j] * xf[j];
      cf += hxf[j] * xf[j];
    }
  }
  /* the maze: 44 cylinders (x, y, r_cyl + r_quad) in problems/quadrotor_maze.jl's order */
  const double r_quad = 2.0, r_cyl = 2.0;
  double cyl[3 * NCYL], t[10];
  int nc = 0;
  struct { double a, b; int k; int along_x; double fixed; } rows[7] = {
      {-25, -10, 5, 1, 10.0}, {10, 25, 5, 1, 10.0}, {-5, 5, 4, 1, 30.0}, {-25, -10, 5, 1, 50.0},
      {10, 25, 5, 1, 50.0}, {10 + 2 * r_cyl, 50 - 2 * r_cyl, 10, 0, -25.0}, {10 + 2 * r_cyl, 50 - 2 * r_cyl, 10, 0, 25.0}};
  for (int g = 0; g < 7; g++) {
    linspace(t, rows[g].a, rows[g].b, rows[g].k);
    for (int i = 0; i < rows[g].k; i++, nc++) {
      cyl[3 * nc] = rows[g].along_x ? t[i] : rows[g].fixed;
      cyl[3 * nc + 1] = rows[g].along_x ? rows[g].fixed : t[i];
      cyl[3 * nc + 2] = r_cyl + r_quad;
    }
  }
  /* BoundConstraints: data [x_max; x_min; u_max; u_min] */
  double bnd1[2 * n + 2 * m], bnd2[2 * n + 2 * m], bxf[2 * n + 2 * m];
  for (int i = 0; i < n; i++) {
    bnd1[i] = INFINITY, bnd1[n + i] = -INFINITY;
    bnd2[i] = INFINITY, bnd2[n + i] = -INFINITY;
    bxf[i] = xf[i], bxf[n + i] = xf[i];
  }
  bnd2[0] = 25.0, bnd2[2] = 20.0, bnd2[n + 0] = -25.0, bnd2[n + 2] = 0.0;
  for (int i = 3; i < 7; i++) bxf[i] = INFINITY, bxf[n + i] = -INFINITY;
  for (int i = 7; i < 10; i++) bxf[i] = 0.0, bxf[n + i] = 0.0;
  for (int i = 0; i < m; i++) {
    bnd1[2 * n + i] = 50.0, bnd1[2 * n + m + i] = 0.0;
    bnd2[2 * n + i] = 50.0, bnd2[2 * n + m + i] = 0.0;
    bxf[2 * n + i] = INFINITY, bxf[2 * n + m + i] = -INFINITY;
  }
  tog_constraint c_first[1] = {{TOG_CON_BOUND, 0, bnd1}};
  tog_constraint c_stage[2] = {{TOG_CON_BOUND, 0, bnd2}, {TOG_CON_CIRCLES, NCYL, cyl}};
  tog_constraint c_term[1] = {{TOG_CON_BOUND, 0, bxf}};
  tog_constraint_set sets[3] = {{1, c_first}, {2, c_stage}, {1, c_term}};
  int32_t knot_set[N];
  for (int k = 0; k < N; k++) knot_set[k] = (k == 0) ? 0 : (k == N - 1 ? 2 : 1);
  tog_problem_desc d;
  memset(&d, 0, sizeof(d));
  d.model = TOG_MODEL_QUADROTOR;
  d.integrator = TOG_RK3;
  d.n = n;
  d.m = m;
  d.N = N;
  d.flags = 0;
  d.batch = B;
  d.dt = 5.0 / (N - 1);
  d.Q = Q, d.R = R, d.H = H, d.q = q, d.r = r, d.c = c;
  d.Qf = Qf, d.qf = qf, d.cf = cf;
  d.n_sets = 3;
  d.sets = sets;
  d.knot_set = knot_set;

  tog_altro_options a;
  tog_default_altro_options(&a);
  a.opts_al.iterations = 300;
  a.opts_al.al_iterations = 40;
  a.opts_al.al_cost_tolerance = 1e-5;
  a.opts_al.al_cost_tolerance_intermediate = 1e-4;
  a.opts_al.constraint_tolerance = 1e-3;
  a.opts_al.penalty_scaling = 10.0;
  a.opts_al.penalty_initial = 1.0;
  a.resolve_feasible_problem = 0;
  a.R_inf = 0.001;

  /* the solver the reference returns (altro_methods.jl:40-52): solver_al.stats with its per-iteration
     vectors (every inner record of the AL phase: al_iterations x (iterations + 1) at most) */
  const int cap = a.opts_al.al_iterations * (a.opts_al.iterations + 1) + 1, ocap = a.opts_al.al_iterations + 1;
  double* St = malloc(sizeof(double) * TOG_NSTATS * B);
  double* Hin = malloc(sizeof(double) * 3 * (size_t)cap * B);
  double* Hout = malloc(sizeof(double) * 4 * (size_t)ocap * B);
  double* Hcnt = malloc(sizeof(double) * 2 * B);
  tog_altro_result res;
  memset(&res, 0, sizeof(res));
  res.inner_capacity = cap;
  res.stats = St;
  res.hist_inner = Hin;
  res.hist_outer = Hout;
  res.hist_count = Hcnt;
  int rc = tog_solve_altro_ex(&d, &a, 0, x0, X, U, NULL, &res);
  if (rc) return fail_rc("tog_solve_altro_ex", rc);
  if (!(res.time >= res.time_al && res.time_al > 0.0 && res.time_pn == 0.0 && res.handle == NULL))
    return fail_rc("tog_altro_result times / handle", -1);
  f = fopen(argv[2], "wb");
  if (!f) return fail_rc("open output", -1);
  fwrite(X, sizeof(double), nX, f);
  fwrite(U, sizeof(double), nU, f);
  fwrite(St, sizeof(double), (size_t)TOG_NSTATS * B, f);
  fwrite(Hcnt, sizeof(double), 2 * (size_t)B, f);
  fwrite(Hout, sizeof(double), 4 * (size_t)ocap * B, f);
  fwrite(Hin, sizeof(double), 3 * (size_t)cap * B, f);
  fclose(f);
  printf("ok B=%lld\n", (long long)B);
  free(x0), free(U), free(X), free(St), free(Hin), free(Hout), free(Hcnt);
  return 0;
}
