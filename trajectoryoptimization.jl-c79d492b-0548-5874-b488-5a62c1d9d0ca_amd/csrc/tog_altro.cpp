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

#include <chrono>
#include <string>
#include <vector>

#include "../../include/tog.h"
#include "tog_altro_desc.hpp"

namespace {
using namespace tog_altro;

struct Handle {
  tog_handle* h = nullptr;
  ~Handle() {
    if (h) tog_destroy(h);
  }
  tog_handle* release() {
    tog_handle* r = h;
    h = nullptr;
    return r;
  }
};

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// create, set the state, (slack controls), (histories), solve to completion within max_steps batch steps
// (0: the tog_solve_budget default)
int run(const tog_problem_desc* d, const tog_options* o, int32_t device, const double* x0, const double* U,
        const double* X, bool slack, int mode, Handle& H, int max_steps, int hcap) {
  int rc = tog_create(d, o, device, &H.h);
  if (rc) return rc;
  if ((rc = tog_set_state(H.h, x0, U, X))) return rc;
  if (slack && (rc = tog_slack_controls(H.h))) return rc;
  if (hcap > 0 && (rc = tog_history_enable(H.h, hcap))) return rc;
  return tog_solve(H.h, mode, max_steps);
}

// solver_al.stats of the AL phase: the summary rows and the iteration histories
int read_al(tog_handle* h, tog_altro_result* r) {
  int rc;
  if (r->stats && (rc = tog_get(h, TOG_FIELD_STATS, r->stats))) return rc;
  if (r->inner_capacity > 0) {
    if (r->hist_inner && (rc = tog_get(h, TOG_FIELD_HIST_INNER, r->hist_inner))) return rc;
    if (r->hist_outer && (rc = tog_get(h, TOG_FIELD_HIST_OUTER, r->hist_outer))) return rc;
    if (r->hist_count && (rc = tog_get(h, TOG_FIELD_HIST_COUNT, r->hist_count))) return rc;
  }
  return TOG_OK;
}

// trajectories whose AL phase ended with one of the reference's exceptions: forward_pass.jl:80-82's
// error("Cost increased") and lowrankdowndate!'s PosDefException (backward_pass.jl:186-192)
std::vector<char> raised(tog_handle* h, long long B, int& rc) {
  std::vector<int32_t> f(B);
  std::vector<char> out(B, 0);
  rc = tog_status(h, f.data());
  for (long long b = 0; b < B && !rc; b++) out[b] = (f[b] & (TOG_TRAJ_COST_INCREASED | TOG_TRAJ_SQRT_PD_FAIL)) != 0;
  return out;
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
  a->max_steps = 0;
  tog_default_pn_options(&a->opts_pn);
}

int32_t tog_solve_altro(const tog_problem_desc* desc, const tog_altro_options* opts, int32_t device,
                        const double* x0, double* X, double* U, double* h_out, double* stats,
                        double* stats_resolve, double* stats_pn) {
  tog_altro_result r;
  memset(&r, 0, sizeof(r));
  r.stats = stats;
  r.stats_resolve = stats_resolve;
  r.stats_pn = stats_pn;
  return tog_solve_altro_ex(desc, opts, device, x0, X, U, h_out, &r);
}

int32_t tog_solve_altro_ex(const tog_problem_desc* desc, const tog_altro_options* opts, int32_t device,
                           const double* x0, double* X, double* U, double* h_out, tog_altro_result* res) {
  const double t0 = now_s();
  if (!desc || !opts || !x0 || !U) return tog__fail(TOG_ERR_ARG, "tog_solve_altro: null argument");
  if (desc->flags & (TOG_PROB_INFEASIBLE | TOG_PROB_MIN_TIME))
    return tog__fail(TOG_ERR_ARG, "tog_solve_altro takes the original problem (altro_problem transforms it)");
  tog_altro_result local;
  memset(&local, 0, sizeof(local));
  tog_altro_result* R = res ? res : &local;
  R->handle = nullptr;
  R->time = R->time_al = R->time_pn = 0.0;
  if (R->inner_capacity < 0) return tog__fail(TOG_ERR_ARG, "inner_capacity must be >= 0");
  const int hcap = R->inner_capacity;
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
  if (opts->max_steps < 0) return tog__fail(TOG_ERR_ARG, "max_steps must be >= 0");
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
  const size_t nX = (size_t)n * N;
  auto finish = [&](Handle& H) {
    if (R->keep_handle) R->handle = H.release();
    R->time = now_s() - t0;
    return TOG_OK;
  };
  // solve!(prob_altro, solver.solver_pn) (altro_methods.jl:31-39) on the AL phase's handle, before
  // process_results!; a trajectory whose AL phase raised never gets there (its statistics zero, its history NaN)
  auto phase2 = [&](Handle& H, const std::vector<char>& err) {
    std::vector<double> pn((size_t)TOG_PN_NSTATS * B);
    const double tp = now_s();
    int rc2;
    if ((rc2 = tog_solve_pn(H.h, &opts->opts_pn, pn.data()))) return rc2;
    R->time_pn = now_s() - tp;
    if (R->hist_pn && (rc2 = tog_get_pn_history(H.h, R->hist_pn, nullptr))) return rc2;
    const size_t np = 2 * (size_t)opts->opts_pn.n_steps;
    for (long long b = 0; b < B; b++) {
      if (!err[b]) continue;
      memset(pn.data() + (size_t)TOG_PN_NSTATS * b, 0, sizeof(double) * TOG_PN_NSTATS);
      if (R->hist_pn)
        for (size_t i = 0; i < np; i++) R->hist_pn[np * b + i] = NAN;
    }
    if (R->stats_pn) memcpy(R->stats_pn, pn.data(), sizeof(double) * pn.size());
    return (int)TOG_OK;
  };
  if (infeasible && min_time) {
    // minimum_time_problem(infeasible_problem(prob)) (altro_methods.jl:98-124). The slacks come from
    // slack_controls on the infeasible problem (infeasible.jl:63-80, the model at prob.dt), on a handle of
    // its own, before the time step becomes a control
    const int mi = m + n, nt = n + 1, mt = mi + 1;
    const double h0 = sqrt(desc->dt);
    std::vector<double> Ui((size_t)mi * (N - 1) * B, 0.0);
    for (long long b = 0; b < B; b++)
      for (int k = 0; k < N - 1; k++)
        for (int i = 0; i < m; i++) Ui[i + mi * (k + (size_t)(N - 1) * b)] = U[i + m * (k + (size_t)(N - 1) * b)];
    {
      Desc di;
      if ((rc = infeasible_desc(desc, opts->R_inf, di))) return rc;
      Handle Hs;
      if ((rc = tog_create(&di.d, &oal, device, &Hs.h)) || (rc = tog_set_state(Hs.h, x0, Ui.data(), X)) ||
          (rc = tog_slack_controls(Hs.h)) || (rc = tog_get(Hs.h, TOG_FIELD_U, Ui.data())))
        return rc;
    }
    Desc dmi;
    if ((rc = infeasible_min_time_desc(desc, opts->R_inf, opts->R_minimum_time, opts->dt_max, opts->dt_min, dmi)))
      return rc;
    // U = [U; s; √dt], X = [X; √dt], x0 = [x0; 0] (minimum_time.jl:30-33)
    std::vector<double> x0t((size_t)nt * B), Ut((size_t)mt * (N - 1) * B), Xt((size_t)nt * N * B);
    for (long long b = 0; b < B; b++) {
      for (int i = 0; i < n; i++) x0t[i + (size_t)nt * b] = x0[i + (size_t)n * b];
      x0t[n + (size_t)nt * b] = 0.0;
      for (int k = 0; k < N - 1; k++) {
        for (int i = 0; i < mi; i++) Ut[i + mt * (k + (size_t)(N - 1) * b)] = Ui[i + mi * (k + (size_t)(N - 1) * b)];
        Ut[mi + mt * (k + (size_t)(N - 1) * b)] = h0;
      }
      for (int k = 0; k < N; k++) {
        for (int i = 0; i < n; i++) Xt[i + nt * (k + (size_t)N * b)] = X[i + n * (k + (size_t)N * b)];
        Xt[n + nt * (k + (size_t)N * b)] = h0;
      }
    }
    const std::vector<double> X_in(X, X + nX * B), U_in(U, U + (size_t)m * (N - 1) * B);
    Handle H1;
    const double ta = now_s();
    if ((rc = run(&dmi.d, &oal, device, x0t.data(), Ut.data(), Xt.data(), false, TOG_MODE_AL, H1, opts->max_steps,
                  hcap)))
      return rc;
    R->time_al = now_s() - ta;
    const std::vector<char> err = raised(H1.h, B, rc);
    if (rc) return rc;
    if (opts->projected_newton && (rc = phase2(H1, err))) return rc;
    if ((rc = tog_get(H1.h, TOG_FIELD_X, Xt.data())) || (rc = tog_get(H1.h, TOG_FIELD_U, Ut.data()))) return rc;
    if ((rc = read_al(H1.h, R))) return rc;
    // process_results!: X[1:n], U[1:m]; then infeasible_to_feasible_problem (infeasible.jl:37-58): the feasible
    // minimum-time problem from them, h and τ from the infeasible solve (τ_1 = 0); projection! leaves the
    // open-loop rollout (X = NaN)
    std::vector<double> Uf((size_t)(m + 1) * (N - 1) * B), Xf((size_t)nt * N * B), hf((size_t)(N - 1) * B);
    for (long long b = 0; b < B; b++) {
      for (int k = 0; k < N; k++) {
        for (int i = 0; i < n; i++) X[i + n * (k + (size_t)N * b)] = Xt[i + nt * (k + (size_t)N * b)];
        for (int i = 0; i < n; i++) Xf[i + nt * (k + (size_t)N * b)] = Xt[i + nt * (k + (size_t)N * b)];
        Xf[n + nt * (k + (size_t)N * b)] = k == 0 ? 0.0 : Xt[n + nt * (k + (size_t)N * b)];
      }
      for (int k = 0; k < N - 1; k++) {
        for (int i = 0; i < m; i++) {
          U[i + m * (k + (size_t)(N - 1) * b)] = Ut[i + mt * (k + (size_t)(N - 1) * b)];
          Uf[i + (m + 1) * (k + (size_t)(N - 1) * b)] = Ut[i + mt * (k + (size_t)(N - 1) * b)];
        }
        const double hk = Ut[mi + mt * (k + (size_t)(N - 1) * b)];
        Uf[m + (m + 1) * (k + (size_t)(N - 1) * b)] = hk;
        hf[k + (size_t)(N - 1) * b] = hk;
      }
    }
    if (opts->resolve_feasible_problem) {
      Desc dm;
      if ((rc = min_time_desc(desc, opts->R_minimum_time, opts->dt_max, opts->dt_min, dm))) return rc;
      Handle H2;
      if ((rc = run(&dm.d, &oal, device, x0t.data(), Uf.data(), opts->dynamically_feasible_projection ? nullptr : Xf.data(),
                    false, TOG_MODE_AL, H2, opts->max_steps, 0)))
        return rc;
      std::vector<double> X2((size_t)nt * N * B);
      if ((rc = tog_get(H2.h, TOG_FIELD_X, X2.data())) || (rc = tog_get(H2.h, TOG_FIELD_U, Uf.data()))) return rc;
      if (R->stats_resolve && (rc = tog_get(H2.h, TOG_FIELD_STATS, R->stats_resolve))) return rc;
      for (long long b = 0; b < B; b++) {
        for (int k = 0; k < N; k++)
          for (int i = 0; i < n; i++) X[i + n * (k + (size_t)N * b)] = X2[i + nt * (k + (size_t)N * b)];
        for (int k = 0; k < N - 1; k++) {
          for (int i = 0; i < m; i++) U[i + m * (k + (size_t)(N - 1) * b)] = Uf[i + (m + 1) * (k + (size_t)(N - 1) * b)];
          hf[k + (size_t)(N - 1) * b] = Uf[m + (m + 1) * (k + (size_t)(N - 1) * b)];
        }
      }
    }
    for (long long b = 0; b < B; b++) {
      if (err[b]) {  // the exception left prob untouched: no process_results!, no resolve
        memcpy(X + nX * b, X_in.data() + nX * b, sizeof(double) * nX);
        memcpy(U + (size_t)m * (N - 1) * b, U_in.data() + (size_t)m * (N - 1) * b, sizeof(double) * m * (N - 1));
        if (R->stats_resolve) memset(R->stats_resolve + (size_t)TOG_NSTATS * b, 0, sizeof(double) * TOG_NSTATS);
        continue;
      }
      if (h_out) memcpy(h_out + (size_t)(N - 1) * b, hf.data() + (size_t)(N - 1) * b, sizeof(double) * (N - 1));
    }
    return finish(H1);
  }
  if (infeasible) {
    Desc di;
    if ((rc = infeasible_desc(desc, opts->R_inf, di))) return rc;
    const int mi = m + n;
    std::vector<double> Ui((size_t)mi * (N - 1) * B, 0.0);
    for (long long b = 0; b < B; b++)
      for (int k = 0; k < N - 1; k++)
        for (int i = 0; i < m; i++) Ui[i + mi * (k + (size_t)(N - 1) * b)] = U[i + m * (k + (size_t)(N - 1) * b)];
    // the caller's X, U: what a raised trajectory keeps (its solve ran on infeasible_problem's copy)
    const std::vector<double> X_in(X, X + nX * B), U_in(U, U + (size_t)m * (N - 1) * B);
    Handle H1;
    const double ta = now_s();
    if ((rc = run(&di.d, &oal, device, x0, Ui.data(), X, true, TOG_MODE_AL, H1, opts->max_steps, hcap))) return rc;
    R->time_al = now_s() - ta;
    const std::vector<char> err = raised(H1.h, B, rc);
    if (rc) return rc;
    // (on the infeasible problem; a raised trajectory's X, U go back to the caller's below)
    if (opts->projected_newton && (rc = phase2(H1, err))) return rc;
    std::vector<double> Xi(nX * B);
    if ((rc = tog_get(H1.h, TOG_FIELD_X, Xi.data())) || (rc = tog_get(H1.h, TOG_FIELD_U, Ui.data()))) return rc;
    // (the statistics rows after projected Newton: its TOG_TRAJ_PN_ERROR lands in the flags)
    if ((rc = read_al(H1.h, R))) return rc;
    // process_results!: X and the model controls U[1:m]
    memcpy(X, Xi.data(), sizeof(double) * nX * B);
    for (long long b = 0; b < B; b++)
      for (int k = 0; k < N - 1; k++)
        for (int i = 0; i < m; i++) U[i + m * (k + (size_t)(N - 1) * b)] = Ui[i + mi * (k + (size_t)(N - 1) * b)];
    if (opts->resolve_feasible_problem) {
      // the feasible problem from the infeasible solve's controls; projection! (ilqr_methods.jl:179-190)
      // leaves the open-loop rollout of U from x0: X = NaN
      const bool con = is_constrained(desc);
      tog_options ores = oal;
      Handle H2;
      if ((rc = run(desc, &ores, device, x0, U, opts->dynamically_feasible_projection ? nullptr : X, false,
                    con ? TOG_MODE_AL : TOG_MODE_ILQR, H2, opts->max_steps, 0)))
        return rc;
      if ((rc = tog_get(H2.h, TOG_FIELD_X, X)) || (rc = tog_get(H2.h, TOG_FIELD_U, U))) return rc;
      if (R->stats_resolve && (rc = tog_get(H2.h, TOG_FIELD_STATS, R->stats_resolve))) return rc;
    }
    for (long long b = 0; b < B; b++) {
      if (!err[b]) continue;  // the exception left prob untouched: no process_results!, no resolve
      memcpy(X + nX * b, X_in.data() + nX * b, sizeof(double) * nX);
      memcpy(U + (size_t)m * (N - 1) * b, U_in.data() + (size_t)m * (N - 1) * b, sizeof(double) * m * (N - 1));
      if (R->stats_resolve) memset(R->stats_resolve + (size_t)TOG_NSTATS * b, 0, sizeof(double) * TOG_NSTATS);
    }
    return finish(H1);
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
    const double ta = now_s();
    if ((rc = run(&dm.d, &oal, device, x0t.data(), Ut.data(), nullptr, false, TOG_MODE_AL, H, opts->max_steps, hcap)))
      return rc;
    R->time_al = now_s() - ta;
    const std::vector<char> err = raised(H.h, B, rc);
    if (rc) return rc;
    // projected Newton on the minimum-time problem (its H from MinTimeCost's hessian!, tog_pn.hpp)
    if (opts->projected_newton && (rc = phase2(H, err))) return rc;
    if ((rc = tog_get(H.h, TOG_FIELD_X, Xt.data())) || (rc = tog_get(H.h, TOG_FIELD_U, Ut.data()))) return rc;
    if ((rc = read_al(H.h, R))) return rc;
    for (long long b = 0; b < B; b++) {  // process_results!: X[1:n], U[1:m]; h separately
      if (err[b]) continue;  // minimum_time_problem's copy raised: prob untouched
      if (X)
        for (int k = 0; k < N; k++)
          for (int i = 0; i < n; i++) X[i + n * (k + (size_t)N * b)] = Xt[i + nt * (k + (size_t)N * b)];
      for (int k = 0; k < N - 1; k++) {
        for (int i = 0; i < m; i++) U[i + m * (k + (size_t)(N - 1) * b)] = Ut[i + mt * (k + (size_t)(N - 1) * b)];
        if (h_out) h_out[k + (size_t)(N - 1) * b] = Ut[m + mt * (k + (size_t)(N - 1) * b)];
      }
    }
    return finish(H);
  }
  // feasible start, fixed time: solve!(prob_altro, solver.solver_al), the AL solver itself (an unconstrained
  // problem too: the solver-level solve! has no iLQR fallback), then projected Newton
  tog_options o = oal;
  Handle H;
  const double ta = now_s();
  if ((rc = run(desc, &o, device, x0, U, nullptr, false, TOG_MODE_AL, H, opts->max_steps, hcap))) return rc;
  R->time_al = now_s() - ta;
  const std::vector<char> err = raised(H.h, B, rc);
  if (rc) return rc;
  if (opts->projected_newton) {
    // a raised trajectory never reaches projected Newton: its X, U (the AL phase's, prob_altro = prob) are
    // put back after the batched projection
    std::vector<double> Xs(nX * B), Us((size_t)m * (N - 1) * B);
    if ((rc = tog_get(H.h, TOG_FIELD_X, Xs.data())) || (rc = tog_get(H.h, TOG_FIELD_U, Us.data()))) return rc;
    std::vector<double> pn((size_t)TOG_PN_NSTATS * B);
    const double tp = now_s();
    if ((rc = tog_solve_pn(H.h, &opts->opts_pn, pn.data()))) return rc;
    R->time_pn = now_s() - tp;
    if (R->hist_pn && (rc = tog_get_pn_history(H.h, R->hist_pn, nullptr))) return rc;
    bool any = false;
    for (long long b = 0; b < B; b++) any = any || err[b];
    if (any) {
      std::vector<double> Xp(nX * B), Up((size_t)m * (N - 1) * B);
      if ((rc = tog_get(H.h, TOG_FIELD_X, Xp.data())) || (rc = tog_get(H.h, TOG_FIELD_U, Up.data()))) return rc;
      const size_t nu = (size_t)m * (N - 1), np = 2 * (size_t)opts->opts_pn.n_steps;
      for (long long b = 0; b < B; b++) {
        if (!err[b]) continue;
        memcpy(Xp.data() + nX * b, Xs.data() + nX * b, sizeof(double) * nX);
        memcpy(Up.data() + nu * b, Us.data() + nu * b, sizeof(double) * nu);
        memset(pn.data() + (size_t)TOG_PN_NSTATS * b, 0, sizeof(double) * TOG_PN_NSTATS);
        if (R->hist_pn)
          for (size_t i = 0; i < np; i++) R->hist_pn[np * b + i] = NAN;
      }
      if ((rc = tog_set(H.h, TOG_FIELD_X, Xp.data())) || (rc = tog_set(H.h, TOG_FIELD_U, Up.data()))) return rc;
    }
    if (R->stats_pn) memcpy(R->stats_pn, pn.data(), sizeof(double) * pn.size());
  }
  // (the statistics rows after projected Newton: its TOG_TRAJ_PN_ERROR lands in the flags)
  if ((rc = read_al(H.h, R))) return rc;
  std::vector<double> Xs(nX * B);
  if ((rc = tog_get(H.h, TOG_FIELD_X, Xs.data())) || (rc = tog_get(H.h, TOG_FIELD_U, U))) return rc;
  if (X) memcpy(X, Xs.data(), sizeof(double) * nX * B);
  return finish(H);
}

}  // extern "C"
