/* tog_oracle_cost.c — TEST INFRASTRUCTURE ONLY (included by tog_oracle.c): CPU restatement of
 * GenericCost (src/cost.jl:239-347) for the parity tests of the device cost plugins
 * (csrc/tog_cost_plugin.hpp, csrc/plugins/cost_*.hip).
 *
 * auto_expansion_function (src/cost.jl:289-322): ForwardDiff.gradient! and ForwardDiff.hessian! of
 * ℓ over z = [x; u] (ℓf over xN). The Hessian is the Jacobian of the gradient: a gradient dual whose
 * value and partials are duals in one Jacobian direction j (ForwardDiff v0.10.3 nesting,
 * Manifest.toml:164-168). hd_* below is that number with w gradient partials; the inner level uses the
 * Dual<1> rules of the Jacobian kernels (x*y partial = fma(yv, xp, xv*yp)). The example costs are the
 * reference test's mycost (test/cost_tests.jl:98-132, both constructors) and SoftObstacleCost
 * (csrc/plugins/cost_soft_obstacle.hip), written as the same expression trees as the plugins. */

#define HDW 32

typedef struct {
  int w;
  double v, t;
  double g[HDW], h[HDW];
} hd;
typedef struct {
  double v, t;
} d1;

static d1 d1_mul(d1 a, d1 b) { d1 r = {a.v * b.v, fma(b.v, a.t, a.v * b.t)}; return r; }
static d1 d1_add(d1 a, d1 b) { d1 r = {a.v + b.v, a.t + b.t}; return r; }
static d1 d1_inv(d1 a) {
  const double c = -(1.0 / (a.v * a.v));
  d1 r = {1.0 / a.v, c * a.t};
  return r;
}
static d1 d1_div(d1 a, d1 b) {
  const double iy = 1.0 / b.v, c2 = -(a.v / (b.v * b.v));
  d1 r = {a.v / b.v, fma(a.t, iy, b.t * c2)};
  return r;
}
static d1 d1_neg(d1 a) { d1 r = {-a.v, -a.t}; return r; }

static hd hd_const(int w, double v) {
  hd r;
  r.w = w;
  r.v = v;
  r.t = 0.0;
  for (int i = 0; i < w; i++) r.g[i] = r.h[i] = 0.0;
  return r;
}
static hd hd_add(hd a, hd b) {
  hd r = a;
  r.v = a.v + b.v;
  r.t = a.t + b.t;
  for (int i = 0; i < a.w; i++) {
    r.g[i] = a.g[i] + b.g[i];
    r.h[i] = a.h[i] + b.h[i];
  }
  return r;
}
static hd hd_sub(hd a, hd b) {
  hd r = a;
  r.v = a.v - b.v;
  r.t = a.t - b.t;
  for (int i = 0; i < a.w; i++) {
    r.g[i] = a.g[i] - b.g[i];
    r.h[i] = a.h[i] - b.h[i];
  }
  return r;
}
static hd hd_mul(hd a, hd b) {
  hd r = a;
  const d1 av = {a.v, a.t}, bv = {b.v, b.t};
  const d1 rv = d1_mul(av, bv);
  r.v = rv.v;
  r.t = rv.t;
  for (int i = 0; i < a.w; i++) {
    const d1 ap = {a.g[i], a.h[i]}, bp = {b.g[i], b.h[i]};
    const d1 p = d1_add(d1_mul(ap, bv), d1_mul(bp, av));
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
static hd hd_scale(double s, hd a) { /* s*x and x*s: (s xv, s xp) */
  hd r = a;
  r.v = s * a.v;
  r.t = s * a.t;
  for (int i = 0; i < a.w; i++) {
    r.g[i] = s * a.g[i];
    r.h[i] = s * a.h[i];
  }
  return r;
}
static hd hd_addc(hd a, double s) { hd r = a; r.v = a.v + s; return r; }
static hd hd_caddc(double s, hd a) { hd r = a; r.v = s + a.v; return r; }
static hd hd_subc(hd a, double s) { hd r = a; r.v = a.v - s; return r; }
static hd hd_div(hd a, hd b) {
  hd r = a;
  const d1 av = {a.v, a.t}, bv = {b.v, b.t};
  const d1 iy = d1_inv(bv);
  const d1 c2 = d1_neg(d1_div(av, d1_mul(bv, bv)));
  const d1 rv = d1_div(av, bv);
  r.v = rv.v;
  r.t = rv.t;
  for (int i = 0; i < a.w; i++) {
    const d1 ap = {a.g[i], a.h[i]}, bp = {b.g[i], b.h[i]};
    const d1 p = d1_add(d1_mul(ap, iy), d1_mul(bp, c2));
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
static hd hd_cdiv(double s, hd b) { return hd_div(hd_const(b.w, s), b); }
static hd hd_unary(hd a, d1 f, d1 df) {
  hd r = a;
  r.v = f.v;
  r.t = f.t;
  for (int i = 0; i < a.w; i++) {
    const d1 ap = {a.g[i], a.h[i]};
    const d1 p = d1_mul(df, ap);
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
static hd hd_sin(hd a) {
  const double s = tog_sin(a.v), c = tog_cos(a.v);
  const d1 f = {s, c * a.t}, df = {c, (-s) * a.t};
  return hd_unary(a, f, df);
}
static hd hd_cos(hd a) {
  const double s = tog_sin(a.v), c = tog_cos(a.v);
  const d1 f = {c, (-s) * a.t}, df = {-s, (-c) * a.t};
  return hd_unary(a, f, df);
}
static hd hd_sqrt(hd a) {
  const double sv = sqrt(a.v);
  const d1 f = {sv, (1.0 / (2.0 * sv)) * a.t};
  const d1 two = {2.0, 0.0};
  const d1 df = d1_inv(d1_mul(two, f));
  return hd_unary(a, f, df);
}

/* cost ids of the example plugins */
enum { OC_COST_MYCOST = 0, OC_COST_SOFT_OBSTACLE = 1 };

static void oc_cost_dims(int id, int* n, int* m) {
  if (id == OC_COST_MYCOST) { *n = 2; *m = 1; }
  else { *n = 4; *m = 2; }
}

/* mycost(x, u) = cos(x1) + u'Ru + Q x2^2 ; mycost(xN) = cos(xN1) + xN2^2 (test/cost_tests.jl:100-107) */
static hd mycost_stage(const hd* x, const hd* u) {
  return hd_add(hd_add(hd_cos(x[0]), hd_mul(u[0], hd_scale(0.1, u[0]))), hd_scale(0.1, hd_mul(x[1], x[1])));
}
static hd mycost_term(const hd* x) { return hd_add(hd_cos(x[0]), hd_mul(x[1], x[1])); }

/* SoftObstacleCost (csrc/plugins/cost_soft_obstacle.hip) */
static hd soft_stage(const hd* x, const hd* u) {
  const double w = 0.5, eps = 0.1, ox = 1.0, oy = 0.5;
  const hd dx = hd_subc(x[0], ox), dy = hd_subc(x[1], oy);
  const hd track = hd_scale(0.5, hd_add(hd_mul(x[0], x[0]), hd_mul(x[1], x[1])));
  const hd obs = hd_cdiv(w, hd_add(hd_caddc(eps, hd_mul(dx, dx)), hd_mul(dy, dy)));
  const hd speed = hd_sqrt(hd_add(hd_caddc(1.0, hd_mul(x[2], x[2])), hd_mul(x[3], x[3])));
  const hd effort = hd_mul(hd_scale(0.5, hd_add(hd_mul(u[0], u[0]), hd_mul(u[1], u[1]))), speed);
  return hd_add(hd_add(hd_add(track, obs), effort), hd_scale(0.1, hd_mul(hd_sin(x[2]), x[3])));
}
static hd soft_term(const hd* x) {
  return hd_add(hd_scale(10.0, hd_add(hd_mul(x[0], x[0]), hd_mul(x[1], x[1]))),
                hd_cdiv(1.0, hd_add(hd_caddc(1.0, hd_mul(x[2], x[2])), hd_mul(x[3], x[3]))));
}

/* cost_expansion!(E, cost::GenericCost, x, u) / (S, cost, xN) and stage_cost (src/cost.jl:324-345) for
 * `count` points: X (n, count), U (m, count) column-major; outputs J (count), Ex (n), Eu (m),
 * Exx (n, n), Euu (m, m), Eux (m, n) per point (terminal: J, Ex, Exx). analytic != 0 evaluates the
 * GenericCost(ℓ, ℓf, grad, hess, n, m) form of mycost (test/cost_tests.jl:112-132) instead. */
OC_EXPORT int oc_generic_cost_expand(int id, int analytic, int terminal, const double* X, const double* U,
                                     long long count, double* J, double* Ex, double* Eu, double* Exx,
                                     double* Euu, double* Eux) {
  int n, m;
  if (id != OC_COST_MYCOST && id != OC_COST_SOFT_OBSTACLE) return -1;
  if (analytic && id != OC_COST_MYCOST) return -1;
  oc_cost_dims(id, &n, &m);
  const int w = terminal ? n : n + m;
  for (long long p = 0; p < count; p++) {
    const double* x = X + p * n;
    const double* u = terminal ? NULL : U + p * m;
    if (analytic) {
      if (terminal) {
        J[p] = tog_cos(x[0]) + x[1] * x[1];
        double* Qf = Exx + p * n * n;
        Qf[0] = -tog_cos(x[0]); Qf[1] = 0.0; Qf[2] = 0.0; Qf[3] = 2.0;
        Ex[p * n] = -tog_sin(x[0]);
        Ex[p * n + 1] = 2.0 * x[1];
      } else {
        J[p] = (tog_cos(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1]);
        double* Q = Exx + p * n * n;
        Q[0] = -tog_cos(x[0]); Q[1] = 0.0; Q[2] = 0.0; Q[3] = 2.0 * 0.1;
        Euu[p * m * m] = 2.0 * 0.1;
        Eux[p * m * n] = 0.0;
        Eux[p * m * n + 1] = 0.0;
        Ex[p * n] = -tog_sin(x[0]);
        Ex[p * n + 1] = (2.0 * 0.1) * x[1];
        Eu[p * m] = (2.0 * 0.1) * u[0];
      }
      continue;
    }
    for (int j = 0; j < w; j++) {
      hd z[HDW];
      for (int i = 0; i < w; i++) {
        z[i] = hd_const(w, i < n ? x[i] : u[i - n]);
        z[i].g[i] = 1.0;
      }
      z[j].t = 1.0;
      hd l;
      if (id == OC_COST_MYCOST)
        l = terminal ? mycost_term(z) : mycost_stage(z, z + n);
      else
        l = terminal ? soft_term(z) : soft_stage(z, z + n);
      if (j == 0) {
        J[p] = l.v;
        for (int i = 0; i < n; i++) Ex[p * n + i] = l.g[i];
        if (!terminal)
          for (int i = 0; i < m; i++) Eu[p * m + i] = l.g[n + i];
      }
      if (j < n) {
        for (int i = 0; i < n; i++) Exx[p * n * n + i + n * j] = l.h[i];
        if (!terminal)
          for (int i = 0; i < m; i++) Eux[p * m * n + i + m * j] = l.h[n + i];
      } else {
        for (int i = 0; i < m; i++) Euu[p * m * m + i + m * (j - n)] = l.h[n + i];
      }
    }
  }
  return 0;
}
