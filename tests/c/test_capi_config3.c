/*
 * test_capi_config3.c — a plain C caller of libtog's ABI (include/tog.h): BASELINE config 3 (the
 * quadrotor point-to-point AL-iLQR problem of test/quadrotor_tests.jl:4-60, square-root backward pass)
 * described exactly as integration/julia/libtog.jl's tog_desc marshals that Problem:
 *   model  Dynamics.quadrotor -> TOG_MODEL_QUADROTOR, info[:integration] = :rk4 -> TOG_RK4
 *   obj    LQRObjective(Q, R, Qf, xf, N): q = -Q xf, c = 0.5 xf'Q xf, qf = -Qf xf, cf = 0.5 xf'Qf xf
 *          (src/objective.jl:102-114), H = 0, r = 0
 *   cons   Constraints([bnd, goal], N): every knot holds its own copy of the set (constraint_sets.jl:162-165),
 *          bnd = BoundConstraint(n, m, u_min=0, u_max=15) -> TOG_CON_BOUND [x_max; x_min; u_max; u_min],
 *          goal = goal_constraint(xf) -> TOG_CON_GOAL (xf read from the closure)
 *   opts   AugmentedLagrangianSolverOptions(opts_uncon = iLQRSolverOptions(cost_tolerance=1e-5,
 *          square_root=true), constraint_tolerance=1e-3, cost_tolerance=1e-5, cost_tolerance_intermediate=1e-4)
 * then tog_create -> tog_set_state -> tog_solve (AL, default budget) -> tog_get.
 *
 *   test_capi_config3 --version           prints tog_version() (links the library, no device needed)
 *   test_capi_config3 <in.bin> <out.bin>  in: int64 B, x0 (13, B), U0 (4, 100, B); out: X (13, 101, B),
 *                                         U (4, 100, B), stats (TOG_NSTATS, B)   (column-major doubles)
 * tests/test_c_caller.py compares out.bin with the Python (ctypes) path bit for bit.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tog.h"

enum { n = 13, m = 4, N = 101 };

static int fail_rc(const char* what, int rc) {
  fprintf(stderr, "%s failed: %d (%s)\n", what, rc, tog_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc == 2 && strcmp(argv[1], "--version") == 0) {
    printf("%d\n", (int)tog_version());
    return tog_version() == TOG_ABI_VERSION ? 0 : 1;
  }
  if (argc != 3) {
    fprintf(stderr, "usage: %s <in.bin> <out.bin> | --version\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return fail_rc("open input", -1);
  int64_t B = 0;
  if (fread(&B, sizeof(B), 1, f) != 1 || B < 1) return fail_rc("read B", -1);
  double* x0 = malloc(sizeof(double) * n * B);
  double* U = malloc(sizeof(double) * m * (N - 1) * B);
  if (fread(x0, sizeof(double), (size_t)(n * B), f) != (size_t)(n * B) ||
      fread(U, sizeof(double), (size_t)(m * (N - 1) * B), f) != (size_t)(m * (N - 1) * B))
    return fail_rc("read x0/U0", -1);
  fclose(f);

  /* LQRObjective(Q, R, Qf, xf, N) */
  double Q[n * n] = {0}, R[m * m] = {0}, H[m * n] = {0}, q[n], r[m] = {0}, Qf[n * n] = {0}, qf[n], xf[n] = {0};
  for (int i = 0; i < n; i++) Q[i + n * i] = 1e-2, Qf[i + n * i] = 1000.0;
  for (int i = 0; i < m; i++) R[i + m * i] = 1e-2;
  xf[1] = 50.0;
  xf[3] = 1.0;
  double c = 0.0, cf = 0.0;
  for (int i = 0; i < n; i++) {  /* (-Q) xf and (0.5 xf' Q) xf, left to right as Julia evaluates them */
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
  /* Constraints([bnd, goal], N): one copy of the set per knot */
  double bnd[2 * n + 2 * m];
  for (int i = 0; i < n; i++) bnd[i] = INFINITY, bnd[n + i] = -INFINITY;
  for (int i = 0; i < m; i++) bnd[2 * n + i] = 15.0, bnd[2 * n + m + i] = 0.0;
  tog_constraint cons[2] = {{TOG_CON_BOUND, 0, bnd}, {TOG_CON_GOAL, n, xf}};
  tog_constraint_set sets[N];
  int32_t knot_set[N];
  for (int k = 0; k < N; k++) {
    sets[k].n_con = 2;
    sets[k].con = cons;
    knot_set[k] = k;
  }
  tog_problem_desc d;
  memset(&d, 0, sizeof(d));
  d.model = TOG_MODEL_QUADROTOR;
  d.integrator = TOG_RK4;
  d.n = n;
  d.m = m;
  d.N = N;
  d.flags = 0;
  d.batch = B;
  d.dt = 0.05;
  d.Q = Q, d.R = R, d.H = H, d.q = q, d.r = r, d.c = c;
  d.Qf = Qf, d.qf = qf, d.cf = cf;
  d.n_sets = N;
  d.sets = sets;
  d.knot_set = knot_set;
  d.user_model = NULL;
  d.R_min_time = 0.0;

  tog_options o;
  tog_default_options(&o);
  o.cost_tolerance = 1e-5;
  o.square_root = 1;
  o.al_cost_tolerance = 1e-5;
  o.al_cost_tolerance_intermediate = 1e-4;
  o.constraint_tolerance = 1e-3;

  tog_handle* h = NULL;
  int rc = tog_create(&d, &o, 0, &h);
  if (rc) return fail_rc("tog_create", rc);
  if ((rc = tog_set_state(h, x0, U, NULL))) return fail_rc("tog_set_state", rc);
  if ((rc = tog_solve(h, TOG_MODE_AL, 0))) return fail_rc("tog_solve", rc);  /* 0: tog_solve_budget */
  double* X = malloc(sizeof(double) * n * N * B);
  double* St = malloc(sizeof(double) * TOG_NSTATS * B);
  if ((rc = tog_get(h, TOG_FIELD_X, X)) || (rc = tog_get(h, TOG_FIELD_U, U)) || (rc = tog_get(h, TOG_FIELD_STATS, St)))
    return fail_rc("tog_get", rc);
  tog_destroy(h);
  f = fopen(argv[2], "wb");
  if (!f) return fail_rc("open output", -1);
  fwrite(X, sizeof(double), (size_t)(n * N * B), f);
  fwrite(U, sizeof(double), (size_t)(m * (N - 1) * B), f);
  fwrite(St, sizeof(double), (size_t)(TOG_NSTATS * B), f);
  fclose(f);
  printf("ok B=%lld\n", (long long)B);
  free(x0), free(U), free(X), free(St);
  return 0;
}
