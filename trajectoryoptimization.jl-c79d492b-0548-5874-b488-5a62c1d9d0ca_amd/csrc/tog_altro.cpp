// tog_altro.cpp — solve!(prob, ALTROSolverOptions) behind the C ABI (include/tog.h tog_solve_altro).
//
// The ALTRO driver of src/solvers/altro/altro_methods.jl:2-124, host side of the ABI so that every
// caller (the Julia binding, C, the Python package) reaches the same flow:
//   altro_problem (:98-124): a given initial state trajectory makes the problem an infeasible-start one
//     (infeasible_problem, src/solvers/altro/infeasible.jl:2-33); tf = 0 makes it a minimum-time one
//     (minimum_time_problem, src/solvers/altro/minimum_time.jl:2-34). Both are descriptor transforms here;
//   the AL solve (augmented_lagrangian_methods.jl:2-31; iLQR when unconstrained, :33-36) on a libtog handle;
//   projected Newton (:31-39) on the same device buffers when requested;
//   process_results! (:56-95): the model states and controls go back to the caller's X, U (the time steps
//     of a minimum-time solve to h), and with resolve_feasible_problem the feasible problem is solved again
//     from the infeasible solve's controls (from the open-loop rollout of projection!'s trajectory when
//     dynamically_feasible_projection).
// Plain C++ over the public entry points (tog_create / tog_set_state / tog_slack_controls / tog_solve /
// tog_get / tog_solve_pn): no device code of its own.
#include <math.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/tog.h"

extern "C" int32_t tog__fail(int32_t code, const char* msg);  // tog_runtime.cpp: sets tog_last_error

namespace {

// A transformed tog_problem_desc and every array it points into.
struct Desc {
  tog_problem_desc d{};
  std::vector<double> Q, R, H, q, r, Qf, qf;
  std::vector<std::vector<double>> data;          // one per constraint
  std::vector<std::vector<tog_constraint>> cons;  // one per set
  std::vector<tog_constraint_set> sets;
  std::vector<int32_t> knot_set;

  int add_set(std::vector<tog_constraint> cs, std::vector<std::vector<double>> ds) {
    for (size_t i = 0; i < cs.size(); i++) {
      data.push_back(std::move(ds[i]));
      cs[i].data = nullptr;  // wired in finalize
    }
    cons.push_back(std::move(cs));
    return (int)cons.size() - 1;
  }
  void finalize() {
    size_t di = 0;
    sets.resize(cons.size());
    for (size_t s = 0; s < cons.size(); s++) {
      for (auto& c : cons[s]) {
        const std::vector<double>& v = data[di++];
        c.data = v.empty() ? nullptr : v.data();
      }
      sets[s].n_con = (int32_t)cons[s].size();
      sets[s].con = cons[s].data();
    }
    d.Q = Q.data();
    d.R = R.data();
    d.H = H.data();
    d.q = q.data();
    d.r = r.data();
    d.Qf = Qf.data();
    d.qf = qf.data();
    d.n_sets = (int32_t)sets.size();
    d.sets = sets.empty() ? nullptr : sets.data();
    d.knot_set = knot_set.data();
  }
};

int con_len(const tog_constraint& c, int n, int m) {  // doubles of a constraint's data
  switch (c.type) {
    case TOG_CON_BOUND: return 2 * n + 2 * m;
    case TOG_CON_GOAL: return c.count > 0 ? c.count : n;
    case TOG_CON_CIRCLES: return 3 * c.count;
    case TOG_CON_SPHERES: return 4 * c.count;
    case TOG_CON_USER: return 3;
    default: return 0;
  }
}

std::vector<double> copy_data(const tog_constraint& c, int n, int m) {
  const int L = con_len(c, n, m);
  return c.data && L > 0 ? std::vector<double>(c.data, c.data + L) : std::vector<double>();
}

bool is_constrained(const tog_problem_desc* d) {
  for (int k = 0; k < d->N; k++) {
    const int si = d->knot_set ? d->knot_set[k] : -1;
    if (si >= 0 && si < d->n_sets && d->sets[si].n_con > 0) return true;
  }
  return false;
}

// infeasible_problem(prob, R_inf) (infeasible.jl:2-33): model add_slack_controls (m -> m + n), stage cost
// R = blockdiag(R, R_inf I/dt), H = [H; 0], r = [r; 0]; every stage constraint set in
// update_constraint_set_jacobians' order (the non-bound constraints, then the bounds, constraint_sets.jl:
// 135-150) followed by infeasible_constraints (u_slack = 0); the terminal set is kept.
int infeasible_desc(const tog_problem_desc* s, double R_inf, Desc& o) {
  const int n = s->n, m = s->m, N = s->N, mi = m + n;
  o.d = *s;
  o.d.m = mi;
  o.d.flags = s->flags | TOG_PROB_INFEASIBLE;
  o.Q.assign(s->Q, s->Q + n * n);
  o.q.assign(s->q, s->q + n);
  o.Qf.assign(s->Qf, s->Qf + n * n);
  o.qf.assign(s->qf, s->qf + n);
  o.R.assign((size_t)mi * mi, 0.0);
  o.H.assign((size_t)mi * n, 0.0);
  o.r.assign(mi, 0.0);
  for (int j = 0; j < m; j++)
    for (int i = 0; i < m; i++) o.R[i + mi * j] = s->R[i + m * j];
  for (int i = 0; i < n; i++) o.R[(m + i) + mi * (m + i)] = R_inf * 1.0 / s->dt;
  for (int j = 0; j < n; j++)
    for (int i = 0; i < m; i++) o.H[i + mi * j] = s->H[i + m * j];
  for (int i = 0; i < m; i++) o.r[i] = s->r[i];
  std::vector<int> memo(s->n_sets + 1, -1);  // stage set per source set (index n_sets: the empty set)
  o.knot_set.assign(N, -1);
  for (int k = 0; k < N; k++) {
    const int si = s->knot_set ? s->knot_set[k] : -1;
    if (k == N - 1) {  // terminal: the problem's own set
      if (si < 0) continue;
      const tog_constraint_set& set = s->sets[si];
      std::vector<tog_constraint> cs(set.con, set.con + set.n_con);
      std::vector<std::vector<double>> ds;
      for (auto& c : cs) ds.push_back(copy_data(c, n, m));
      o.knot_set[k] = o.add_set(std::move(cs), std::move(ds));
      continue;
    }
    const int key = si < 0 ? s->n_sets : si;
    if (memo[key] < 0) {
      std::vector<tog_constraint> cs;
      std::vector<std::vector<double>> ds;
      if (si >= 0) {
        const tog_constraint_set& set = s->sets[si];
        for (int pass = 0; pass < 2; pass++)
          for (int c = 0; c < set.n_con; c++) {
            const tog_constraint& con = set.con[c];
            if ((con.type == TOG_CON_BOUND) != (pass == 1)) continue;
            if (con.type == TOG_CON_BOUND) {
              if (con.count == 1) return tog__fail(TOG_ERR_UNSUPPORTED, "trim=false bounds on an infeasible-start problem");
              // [x_max; x_min; u_max; u_min] over the augmented controls: the slack entries are unbounded
              std::vector<double> b(2 * n + 2 * mi);
              for (int i = 0; i < 2 * n; i++) b[i] = con.data[i];
              for (int i = 0; i < mi; i++) {
                b[2 * n + i] = i < m ? con.data[2 * n + i] : INFINITY;
                b[2 * n + mi + i] = i < m ? con.data[2 * n + m + i] : -INFINITY;
              }
              cs.push_back({TOG_CON_BOUND, 0, nullptr});
              ds.push_back(std::move(b));
            } else {
              if (con.type == TOG_CON_USER) return tog__fail(TOG_ERR_UNSUPPORTED, "user constraint rows in tog_solve_altro");
              cs.push_back(con);
              ds.push_back(copy_data(con, n, m));
            }
          }
      }
      cs.push_back({TOG_CON_INFEASIBLE, 0, nullptr});
      ds.push_back({});
      memo[key] = o.add_set(std::move(cs), std::move(ds));
    }
    o.knot_set[k] = memo[key];
  }
  o.finalize();
  return TOG_OK;
}

// minimum_time_problem(prob, R_min_time, dt_max, dt_min) (minimum_time.jl:2-34): model
// add_min_time_controls (x = [x; τ], u = [u; h]), MinTimeCost over the zero-padded quadratic cost, and
// mintime_constraints (:125-141): at every knot the non-bound constraints, then the bounds combined with
// √dt_min <= h <= √dt_max (τ unbounded; a knot without bounds gets them alone), then h_k = τ_k at the
// knots 1 < k < N.
int min_time_desc(const tog_problem_desc* s, double R_min_time, double dt_max, double dt_min, Desc& o) {
  const int n = s->n, m = s->m, N = s->N, nt = n + 1, mt = m + 1;
  o.d = *s;
  o.d.n = nt;
  o.d.m = mt;
  o.d.flags = (s->flags & ~TOG_PROB_TF_MIN) | TOG_PROB_MIN_TIME;
  o.d.R_min_time = R_min_time;
  auto pad = [](const double* A, int r, int c, int R, int Cc) {
    std::vector<double> out((size_t)R * Cc, 0.0);
    for (int j = 0; j < c; j++)
      for (int i = 0; i < r; i++) out[i + (size_t)R * j] = A[i + (size_t)r * j];
    return out;
  };
  o.Q = pad(s->Q, n, n, nt, nt);
  o.R = pad(s->R, m, m, mt, mt);
  o.H = pad(s->H, m, n, mt, nt);
  o.q = pad(s->q, n, 1, nt, 1);
  o.r = pad(s->r, m, 1, mt, 1);
  o.Qf = pad(s->Qf, n, n, nt, nt);
  o.qf = pad(s->qf, n, 1, nt, 1);
  o.knot_set.assign(N, -1);
  std::vector<int> memo(3 * (s->n_sets + 1), -1);
  for (int k = 0; k < N; k++) {
    const int si = s->knot_set ? s->knot_set[k] : -1;
    const int pos = (k == 0) ? 0 : (k == N - 1 ? 1 : 2);
    const int key = 3 * (si < 0 ? s->n_sets : si) + pos;
    if (memo[key] < 0) {
      std::vector<tog_constraint> cs;
      std::vector<std::vector<double>> ds;
      const tog_constraint* bnd = nullptr;
      if (si >= 0) {
        const tog_constraint_set& set = s->sets[si];
        for (int c = 0; c < set.n_con; c++) {
          const tog_constraint& con = set.con[c];
          if (con.type == TOG_CON_BOUND) {
            if (!bnd) bnd = &con;
            continue;
          }
          if (con.type == TOG_CON_USER || con.type == TOG_CON_INFEASIBLE)
            return tog__fail(TOG_ERR_UNSUPPORTED, "minimum time with user or slack constraint rows");
          tog_constraint cc = con;
          if (cc.type == TOG_CON_GOAL && cc.count == 0) cc.count = n;  // the goal stays on x[1:n]
          cs.push_back(cc);
          ds.push_back(copy_data(con, n, m));
        }
      }
      std::vector<double> b(2 * nt + 2 * mt);
      for (int i = 0; i < n; i++) {
        b[i] = bnd ? bnd->data[i] : INFINITY;
        b[nt + i] = bnd ? bnd->data[n + i] : -INFINITY;
      }
      b[n] = INFINITY;
      b[nt + n] = -INFINITY;
      for (int i = 0; i < m; i++) {
        b[2 * nt + i] = bnd ? bnd->data[2 * n + i] : INFINITY;
        b[2 * nt + mt + i] = bnd ? bnd->data[2 * n + m + i] : -INFINITY;
      }
      b[2 * nt + m] = sqrt(dt_max);
      b[2 * nt + mt + m] = sqrt(dt_min);
      cs.push_back({TOG_CON_BOUND, 0, nullptr});
      ds.push_back(std::move(b));
      if (pos == 2) {
        cs.push_back({TOG_CON_MIN_TIME_EQ, 0, nullptr});
        ds.push_back({});
      }
      memo[key] = o.add_set(std::move(cs), std::move(ds));
    }
    o.knot_set[k] = memo[key];
  }
  o.finalize();
  return TOG_OK;
}

struct Handle {
  tog_handle* h = nullptr;
  ~Handle() {
    if (h) tog_destroy(h);
  }
};

// create, set the state, (slack controls), solve to completion with the default step budget
int run(const tog_problem_desc* d, const tog_options* o, int32_t device, const double* x0, const double* U,
        const double* X, bool slack, int mode, Handle& H) {
  int rc = tog_create(d, o, device, &H.h);
  if (rc) return rc;
  if ((rc = tog_set_state(H.h, x0, U, X))) return rc;
  if (slack && (rc = tog_slack_controls(H.h))) return rc;
  return tog_solve(H.h, mode, 0);
}

}  // namespace

extern "C" {

void tog_default_altro_options(tog_altro_options* a) {
  memset(a, 0, sizeof(*a));
  tog_default_options(&a->opts_al);
  a->R_inf = 1.0;
  a->R_minimum_time = 1.0;
  a->dt_max = 1.0;
  a->dt_min = 1.0e-3;
  a->projected_newton_tolerance = 1.0e-3;
  a->dynamically_feasible_projection = 1;
  a->resolve_feasible_problem = 1;
  a->projected_newton = 0;
  tog_default_pn_options(&a->opts_pn);
}

int32_t tog_solve_altro(const tog_problem_desc* desc, const tog_altro_options* opts, int32_t device,
                        const double* x0, double* X, double* U, double* h_out, double* stats,
                        double* stats_resolve, double* stats_pn) {
  if (!desc || !opts || !x0 || !U) return tog__fail(TOG_ERR_ARG, "tog_solve_altro: null argument");
  if (desc->flags & (TOG_PROB_INFEASIBLE | TOG_PROB_MIN_TIME))
    return tog__fail(TOG_ERR_ARG, "tog_solve_altro takes the original problem (altro_problem transforms it)");
  const int n = desc->n, m = desc->m, N = desc->N;
  const long long B = desc->batch;
  // altro_problem (altro_methods.jl:101): an initial state trajectory that is not all NaN
  long long given = 0;
  if (X)
    for (long long b = 0; b < B; b++) {
      bool all_nan = true;
      for (int i = 0; i < n; i++) all_nan = all_nan && isnan(X[i + (size_t)n * N * b]);
      given += all_nan ? 0 : 1;
    }
  if (given != 0 && given != B)
    return tog__fail(TOG_ERR_ARG, "infeasible start: X must be given for every trajectory of the batch or for none");
  const bool infeasible = given == B && B > 0;
  const bool min_time = (desc->flags & TOG_PROB_TF_MIN) != 0;
  if (infeasible && min_time) return tog__fail(TOG_ERR_UNSUPPORTED, "infeasible start + minimum time");
  if (opts->projected_newton && (infeasible || min_time))
    return tog__fail(TOG_ERR_UNSUPPORTED, "projected Newton on the infeasible-start or minimum-time problem");
  tog_options oal = opts->opts_al;
  if (opts->projected_newton) {  // altro_methods.jl:5-13
    if (opts->projected_newton_tolerance >= 0) {
      oal.constraint_tolerance = opts->projected_newton_tolerance;
    } else {
      oal.constraint_tolerance = 0.0;
      oal.kickout_max_penalty = 1;
    }
  }
  int rc;
  const size_t nU = (size_t)m * (N - 1), nX = (size_t)n * N;
  if (infeasible) {
    Desc di;
    if ((rc = infeasible_desc(desc, opts->R_inf, di))) return rc;
    const int mi = m + n;
    std::vector<double> Ui((size_t)mi * (N - 1) * B, 0.0);
    for (long long b = 0; b < B; b++)
      for (int k = 0; k < N - 1; k++)
        for (int i = 0; i < m; i++) Ui[i + mi * (k + (size_t)(N - 1) * b)] = U[i + m * (k + (size_t)(N - 1) * b)];
    {
      Handle H;
      if ((rc = run(&di.d, &oal, device, x0, Ui.data(), X, true, TOG_MODE_AL, H))) return rc;
      std::vector<double> Xi(nX * B);
      if ((rc = tog_get(H.h, TOG_FIELD_X, Xi.data())) || (rc = tog_get(H.h, TOG_FIELD_U, Ui.data()))) return rc;
      if (stats && (rc = tog_get(H.h, TOG_FIELD_STATS, stats))) return rc;
      // process_results!: X and the model controls U[1:m]
      memcpy(X, Xi.data(), sizeof(double) * nX * B);
      for (long long b = 0; b < B; b++)
        for (int k = 0; k < N - 1; k++)
          for (int i = 0; i < m; i++) U[i + m * (k + (size_t)(N - 1) * b)] = Ui[i + mi * (k + (size_t)(N - 1) * b)];
    }
    if (opts->resolve_feasible_problem) {
      // the feasible problem from the infeasible solve's controls; projection! (ilqr_methods.jl:179-190)
      // leaves the open-loop rollout of U from x0: X = NaN
      const bool con = is_constrained(desc);
      tog_options ores = oal;
      Handle H;
      if ((rc = run(desc, &ores, device, x0, U, opts->dynamically_feasible_projection ? nullptr : X, false,
                    con ? TOG_MODE_AL : TOG_MODE_ILQR, H)))
        return rc;
      if ((rc = tog_get(H.h, TOG_FIELD_X, X)) || (rc = tog_get(H.h, TOG_FIELD_U, U))) return rc;
      if (stats_resolve && (rc = tog_get(H.h, TOG_FIELD_STATS, stats_resolve))) return rc;
    }
    return TOG_OK;
  }
  if (min_time) {
    Desc dm;
    if ((rc = min_time_desc(desc, opts->R_minimum_time, opts->dt_max, opts->dt_min, dm))) return rc;
    const int nt = n + 1, mt = m + 1;
    const double h0 = sqrt(desc->dt);
    std::vector<double> x0t((size_t)nt * B), Ut((size_t)mt * (N - 1) * B), Xt((size_t)nt * N * B);
    for (long long b = 0; b < B; b++) {
      for (int i = 0; i < n; i++) x0t[i + (size_t)nt * b] = x0[i + (size_t)n * b];
      x0t[n + (size_t)nt * b] = 0.0;
      for (int k = 0; k < N - 1; k++) {
        for (int i = 0; i < m; i++) Ut[i + mt * (k + (size_t)(N - 1) * b)] = U[i + m * (k + (size_t)(N - 1) * b)];
        Ut[m + mt * (k + (size_t)(N - 1) * b)] = h0;
      }
    }
    Handle H;
    if ((rc = run(&dm.d, &oal, device, x0t.data(), Ut.data(), nullptr, false, TOG_MODE_AL, H))) return rc;
    if ((rc = tog_get(H.h, TOG_FIELD_X, Xt.data())) || (rc = tog_get(H.h, TOG_FIELD_U, Ut.data()))) return rc;
    if (stats && (rc = tog_get(H.h, TOG_FIELD_STATS, stats))) return rc;
    for (long long b = 0; b < B; b++) {  // process_results!: X[1:n], U[1:m]; h separately
      if (X)
        for (int k = 0; k < N; k++)
          for (int i = 0; i < n; i++) X[i + n * (k + (size_t)N * b)] = Xt[i + nt * (k + (size_t)N * b)];
      for (int k = 0; k < N - 1; k++) {
        for (int i = 0; i < m; i++) U[i + m * (k + (size_t)(N - 1) * b)] = Ut[i + mt * (k + (size_t)(N - 1) * b)];
        if (h_out) h_out[k + (size_t)(N - 1) * b] = Ut[m + mt * (k + (size_t)(N - 1) * b)];
      }
    }
    return TOG_OK;
  }
  // feasible start, fixed time: solve!(prob_altro, solver.solver_al), the AL solver itself (an unconstrained
  // problem too: the solver-level solve! has no iLQR fallback), then projected Newton
  tog_options o = oal;
  Handle H;
  if ((rc = run(desc, &o, device, x0, U, nullptr, false, TOG_MODE_AL, H))) return rc;
  if (opts->projected_newton) {
    std::vector<double> pn((size_t)TOG_PN_NSTATS * B);
    if ((rc = tog_solve_pn(H.h, &opts->opts_pn, pn.data()))) return rc;
    if (stats_pn) memcpy(stats_pn, pn.data(), sizeof(double) * pn.size());
  }
  std::vector<double> Xs(nX * B);
  if ((rc = tog_get(H.h, TOG_FIELD_X, Xs.data())) || (rc = tog_get(H.h, TOG_FIELD_U, U))) return rc;
  if (X) memcpy(X, Xs.data(), sizeof(double) * nX * B);
  if (stats && (rc = tog_get(H.h, TOG_FIELD_STATS, stats))) return rc;
  (void)nU;
  return TOG_OK;
}

}  // extern "C"
