// tog_altro_desc.hpp — the ALTRO descriptor transforms of tog_altro.cpp (infeasible_problem and
// minimum_time_problem as tog_problem_desc -> tog_problem_desc). Plain host C++ over include/tog.h, kept in a
// header of its own so that tests/c/asan_oracle.cpp can build them under -fsanitize=address,undefined
// without the HIP runtime.
#pragma once
#include <math.h>
#include <string.h>

#include <vector>

#include "../../include/tog.h"

extern "C" int32_t tog__fail(int32_t code, const char* msg);  // tog_runtime.cpp: sets tog_last_error

namespace tog_altro {


// A transformed tog_problem_desc and every array it points into.
struct Desc {
  tog_problem_desc d{};
  std::vector<double> Q, R, H, q, r, Qf, qf;
  std::vector<double> kc;                         // a time-varying Objective's rows (tog_problem_desc.stage_costs)
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
    d.stage_costs = kc.empty() ? nullptr : kc.data();
    d.n_sets = (int32_t)sets.size();
    d.sets = sets.empty() ? nullptr : sets.data();
    d.knot_set = knot_set.data();
  }
};

// one stage cost [Q; R; H; q; r; c]: the shared one, or knot k's row of a time-varying Objective
struct StageCost {
  const double *Q, *R, *H, *q, *r;
  double c;
};

inline StageCost stage_of(const tog_problem_desc* s, int k) {
  if (!s->stage_costs) return {s->Q, s->R, s->H, s->q, s->r, s->c};
  const int n = s->n, m = s->m;
  const double* p = s->stage_costs + (size_t)k * (n * n + m * m + m * n + n + m + 1);
  return {p, p + n * n, p + n * n + m * m, p + n * n + m * m + m * n, p + n * n + m * m + m * n + n,
          p[n * n + m * m + m * n + n + m]};
}

// the transformed stage costs: f(cost) -> row [Q; R; H; q; r; c] of the new sizes (n, m), applied to the
// shared cost or to every knot of the table; the shared fields hold knot 0's
template <class F>
inline void map_stage_costs(const tog_problem_desc* s, int n, int m, Desc& o, F f) {
  const int knots = s->stage_costs ? s->N - 1 : 1;
  std::vector<double> row;
  for (int k = 0; k < knots; k++) {
    row = f(stage_of(s, k));
    if (s->stage_costs) o.kc.insert(o.kc.end(), row.begin(), row.end());
    if (k > 0) continue;
    const double* p = row.data();
    o.Q.assign(p, p + n * n), p += n * n;
    o.R.assign(p, p + m * m), p += m * m;
    o.H.assign(p, p + m * n), p += m * n;
    o.q.assign(p, p + n), p += n;
    o.r.assign(p, p + m), p += m;
    o.d.c = *p;
  }
}

inline int con_len(const tog_constraint& c, int n, int m) {  // doubles of a constraint's data
  switch (c.type) {
    case TOG_CON_BOUND: return 2 * n + 2 * m;
    case TOG_CON_GOAL: return c.count > 0 ? c.count : n;
    case TOG_CON_CIRCLES: return 3 * c.count;
    case TOG_CON_SPHERES: return 4 * c.count;
    case TOG_CON_USER: return 3;
    default: return 0;
  }
}

inline std::vector<double> copy_data(const tog_constraint& c, int n, int m) {
  const int L = con_len(c, n, m);
  return c.data && L > 0 ? std::vector<double>(c.data, c.data + L) : std::vector<double>();
}

inline bool is_constrained(const tog_problem_desc* d) {
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
inline int infeasible_desc(const tog_problem_desc* s, double R_inf, Desc& o) {
  const int n = s->n, m = s->m, N = s->N, mi = m + n;
  o.d = *s;
  o.d.m = mi;
  o.d.flags = (s->flags & ~TOG_PROB_TF_MIN) | TOG_PROB_INFEASIBLE;
  o.Qf.assign(s->Qf, s->Qf + n * n);
  o.qf.assign(s->qf, s->qf + n);
  map_stage_costs(s, n, mi, o, [&](const StageCost& c) {
    std::vector<double> row((size_t)n * n + mi * mi + mi * n + n + mi + 1, 0.0);
    double *Q = row.data(), *R = Q + n * n, *H = R + mi * mi, *q = H + mi * n, *r = q + n;
    for (int i = 0; i < n * n; i++) Q[i] = c.Q[i];
    for (int j = 0; j < m; j++)
      for (int i = 0; i < m; i++) R[i + mi * j] = c.R[i + m * j];
    for (int i = 0; i < n; i++) R[(m + i) + mi * (m + i)] = R_inf * 1.0 / s->dt;
    for (int j = 0; j < n; j++)
      for (int i = 0; i < m; i++) H[i + mi * j] = c.H[i + m * j];
    for (int i = 0; i < n; i++) q[i] = c.q[i];
    for (int i = 0; i < m; i++) r[i] = c.r[i];
    r[mi] = c.c;
    return row;
  });
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
              // [x_max; x_min; u_max; u_min] over the augmented controls: the slack entries are unbounded
              // (and never get rows, trim=false included: the bound keeps the model's m, build_rows)
              std::vector<double> b(2 * n + 2 * mi);
              for (int i = 0; i < 2 * n; i++) b[i] = con.data[i];
              for (int i = 0; i < mi; i++) {
                b[2 * n + i] = i < m ? con.data[2 * n + i] : INFINITY;
                b[2 * n + mi + i] = i < m ? con.data[2 * n + m + i] : -INFINITY;
              }
              cs.push_back({TOG_CON_BOUND, con.count, nullptr});
              ds.push_back(std::move(b));
            } else {
              // circles, spheres, user functions c(x, u[1:m]): the plugin evaluates them on the model's
              // controls, their Jacobian columns over the slack controls are zero (_∇c's view, :137-143)
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
inline int min_time_desc(const tog_problem_desc* s, double R_min_time, double dt_max, double dt_min, Desc& o) {
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
  map_stage_costs(s, nt, mt, o, [&](const StageCost& c) {
    std::vector<double> row;
    for (auto v : {pad(c.Q, n, n, nt, nt), pad(c.R, m, m, mt, mt), pad(c.H, m, n, mt, nt), pad(c.q, n, 1, nt, 1),
                   pad(c.r, m, 1, mt, 1)})
      row.insert(row.end(), v.begin(), v.end());
    row.push_back(c.c);
    return row;
  });
  o.Qf = pad(s->Qf, n, n, nt, nt);
  o.qf = pad(s->qf, n, 1, nt, 1);
  // @assert has_bounds(prob.constraints) (minimum_time.jl:6)
  bool has_bounds = false;
  for (int k = 0; k < N && !has_bounds; k++) {
    const int si = s->knot_set ? s->knot_set[k] : -1;
    if (si < 0 || si >= s->n_sets) continue;
    for (int c = 0; c < s->sets[si].n_con; c++) has_bounds = has_bounds || s->sets[si].con[c].type == TOG_CON_BOUND;
  }
  if (!has_bounds) return tog__fail(TOG_ERR_ARG, "minimum time: the problem has no BoundConstraint (minimum_time.jl:6)");
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
          // (user rows keep their function over the base model's x, u: MinTime<M>::con)
          if (con.type == TOG_CON_INFEASIBLE)
            return tog__fail(TOG_ERR_UNSUPPORTED, "minimum time of a problem that already has slack constraint rows");
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

// minimum_time_problem(infeasible_problem(prob)) (altro_methods.jl:98-124): x = [x; τ], u = [u; s; h]; the cost
// is the infeasible problem's (R_inf I/dt on the slacks, infeasible.jl:2-33) zero-padded for [τ; h], and every
// set is mintime_constraints' over the infeasible problem (minimum_time.jl:125-141): the non-bound constraints,
// infeasible_constraints at the stage knots, the combined bound, h_k = τ_k at 1 < k < N. combine(bnd, mt_bnd)
// sizes the bound by the infeasible problem's BoundConstraint, which keeps the model's (n, m): its √dt bounds
// land on u[m+1], the first slack control, and h is unbounded; a knot without a bound gets
// BoundConstraint(n, m + n) combined, whose √dt bounds are on h. Reproduced as written.
inline int infeasible_min_time_desc(const tog_problem_desc* s, double R_inf, double R_min_time, double dt_max,
                                    double dt_min, Desc& o) {
  const int n = s->n, m = s->m, N = s->N, mi = m + n, nt = n + 1, mt = mi + 1;
  o.d = *s;
  o.d.n = nt;
  o.d.m = mt;
  o.d.flags = (s->flags & ~TOG_PROB_TF_MIN) | TOG_PROB_INFEASIBLE | TOG_PROB_MIN_TIME;
  o.d.R_min_time = R_min_time;
  auto pad = [](const double* A, int r, int c, int R, int Cc) {
    std::vector<double> out((size_t)R * Cc, 0.0);
    for (int j = 0; j < c; j++)
      for (int i = 0; i < r; i++) out[i + (size_t)R * j] = A[i + (size_t)r * j];
    return out;
  };
  map_stage_costs(s, nt, mt, o, [&](const StageCost& c) {
    // infeasible_problem's cost (R = blockdiag(R, R_inf I/dt), H = [H; 0], r = [r; 0]), then the padding
    std::vector<double> R((size_t)mi * mi, 0.0), H((size_t)mi * n, 0.0), r(mi, 0.0);
    for (int j = 0; j < m; j++)
      for (int i = 0; i < m; i++) R[i + mi * j] = c.R[i + m * j];
    for (int i = 0; i < n; i++) R[(m + i) + mi * (m + i)] = R_inf * 1.0 / s->dt;
    for (int j = 0; j < n; j++)
      for (int i = 0; i < m; i++) H[i + mi * j] = c.H[i + m * j];
    for (int i = 0; i < m; i++) r[i] = c.r[i];
    std::vector<double> row;
    for (auto v : {pad(c.Q, n, n, nt, nt), pad(R.data(), mi, mi, mt, mt), pad(H.data(), mi, n, mt, nt),
                   pad(c.q, n, 1, nt, 1), pad(r.data(), mi, 1, mt, 1)})
      row.insert(row.end(), v.begin(), v.end());
    row.push_back(c.c);
    return row;
  });
  o.Qf = pad(s->Qf, n, n, nt, nt);
  o.qf = pad(s->qf, n, 1, nt, 1);
  bool has_bounds = false;  // @assert has_bounds(prob.constraints) (minimum_time.jl:6)
  for (int k = 0; k < N && !has_bounds; k++) {
    const int si = s->knot_set ? s->knot_set[k] : -1;
    if (si < 0 || si >= s->n_sets) continue;
    for (int c = 0; c < s->sets[si].n_con; c++) has_bounds = has_bounds || s->sets[si].con[c].type == TOG_CON_BOUND;
  }
  if (!has_bounds) return tog__fail(TOG_ERR_ARG, "minimum time: the problem has no BoundConstraint (minimum_time.jl:6)");
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
          if (con.type == TOG_CON_USER || con.type == TOG_CON_INFEASIBLE || con.type == TOG_CON_MIN_TIME_EQ)
            return tog__fail(TOG_ERR_UNSUPPORTED, "infeasible minimum time with user, slack or time-step rows");
          tog_constraint cc = con;
          if (cc.type == TOG_CON_GOAL && cc.count == 0) cc.count = n;  // the goal stays on x[1:n]
          cs.push_back(cc);
          ds.push_back(copy_data(con, n, m));
        }
      }
      if (pos != 1) {  // infeasible_constraints, after the others (update_constraint_set_jacobians order)
        cs.push_back({TOG_CON_INFEASIBLE, 0, nullptr});
        ds.push_back({});
      }
      // the combined bound over [x; τ], [u; s; h]
      std::vector<double> b(2 * nt + 2 * mt);
      for (int i = 0; i < nt; i++) {
        b[i] = (bnd && i < n) ? bnd->data[i] : INFINITY;
        b[nt + i] = (bnd && i < n) ? bnd->data[n + i] : -INFINITY;
      }
      for (int i = 0; i < mt; i++) {
        b[2 * nt + i] = (bnd && i < m) ? bnd->data[2 * n + i] : INFINITY;
        b[2 * nt + mt + i] = (bnd && i < m) ? bnd->data[2 * n + m + i] : -INFINITY;
      }
      const int ih = bnd ? m : mi;  // u[m+1] (the first slack) when the knot had a bound, else h
      b[2 * nt + ih] = sqrt(dt_max);
      b[2 * nt + mt + ih] = sqrt(dt_min);
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

}  // namespace tog_altro
