/*
 * tog_oracle.c — TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline "port").
 *
 * A plain-C, fp64, single-trajectory restatement of TrajectoryOptimization.jl's
 * iLQR / augmented-Lagrangian hot path (reference mounted read-only at
 * /root/reference; every function cites the file:line it follows). It is NOT
 * part of the product: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, as the checker. The product (libtog.so, HIP) never
 * links or calls it.
 *
 * Parity pinning: the reference cannot run here (no Julia toolchain; SURVEY.md
 * §8c). This restatement is pinned by re-running the reference's own test
 * assertions (tests/test_oracle.py: test/sqrt_bp_tests.jl, test/cost_tests.jl,
 * test/constraint_tests.jl, test/model_tests.jl, test/test_utils.jl,
 * test/quadrotor_tests.jl convergence thresholds) and by LAPACK cross-checks
 * of its linear algebra (numpy.linalg). Rounding-level differences from Julia
 * (BLAS summation order, ForwardDiff op order, LAPACK blocking) are expected;
 * the parity bar is 1e-6 relative.
 *
 * Third-party arithmetic restated here: ForwardDiff v0.10.3 forward-mode duals
 * (Manifest.toml:164-168) and the Julia 1.1 LinearAlgebra/LAPACK routines used
 * by backward_pass.jl (geqrf Householder, potrf, getrf/getrs, lowrankdowndate!,
 * cond via singular values).
 */
#include <math.h>
#include <time.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/tog.h"
#include "../include/tog_math.h"
#include "../include/tog_kuka.h"

#define DMAX 24 /* max partials: n+m+1 of a model (slack columns are never dual) */
#define OM 32   /* max controls, including the n slack controls of an infeasible problem */
#define OP 128  /* max constraint rows per knot (quadrotor_maze infeasible: 69) */
#define OC_EXPORT __attribute__((visibility("default")))

/* =====================================================================
 * Dual numbers — ForwardDiff.Dual semantics (value + partials)
 * ===================================================================== */
typedef struct {
  double v;
  double p[DMAX];
} dual;

static _Thread_local int g_nd = 0; /* number of active partials (0 => primal evaluation); per thread: oc_solve_batch runs trajectories on OpenMP threads */

static inline dual dc(double v) {
  dual r;
  r.v = v;
  for (int i = 0; i < g_nd; i++) r.p[i] = 0.0;
  return r;
}
static inline dual dadd(dual a, dual b) {
  dual r;
  r.v = a.v + b.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = a.p[i] + b.p[i];
  return r;
}
static inline dual dsub(dual a, dual b) {
  dual r;
  r.v = a.v - b.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = a.p[i] - b.p[i];
  return r;
}
static inline dual dneg(dual a) {
  dual r;
  r.v = -a.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = -a.p[i];
  return r;
}
/* ForwardDiff: x*y -> Dual(xv*yv, yv*x.p + xv*y.p) (dual.jl _mul_partials) */
static inline dual dmul(dual a, dual b) {
  dual r;
  r.v = a.v * b.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = fma(b.v, a.p[i], a.v * b.p[i]);
  return r;
}
static inline dual dscale(dual a, double s) { /* Real * Dual */
  dual r;
  r.v = s * a.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = s * a.p[i];
  return r;
}
static inline dual ddivc(dual a, double s) { /* Dual / Real */
  dual r;
  r.v = a.v / s;
  for (int i = 0; i < g_nd; i++) r.p[i] = a.p[i] / s;
  return r;
}
static inline dual ddiv6(dual a) { /* Dual / 6 (tog_div6: the correctly rounded quotient) */
  dual r;
  r.v = tog_div6(a.v);
  for (int i = 0; i < g_nd; i++) r.p[i] = tog_div6(a.p[i]);
  return r;
}
/* ForwardDiff: x/y -> Dual(xv/yv, x.p*inv(yv) + y.p*(-(xv/(yv*yv)))) */
static inline dual ddiv(dual a, dual b) {
  dual r;
  double iy = 1.0 / b.v, c2 = -(a.v / (b.v * b.v));
  r.v = a.v / b.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = fma(a.p[i], iy, b.p[i] * c2);
  return r;
}
static inline dual dinv(dual a) { /* inv(x): 1/v, -p/v^2 */
  dual r;
  r.v = 1.0 / a.v;
  double c = -(1.0 / (a.v * a.v));
  for (int i = 0; i < g_nd; i++) r.p[i] = c * a.p[i];
  return r;
}
static inline dual dsin(dual a) {
  dual r;
  r.v = tog_sin(a.v);
  double c = tog_cos(a.v);
  for (int i = 0; i < g_nd; i++) r.p[i] = c * a.p[i];
  return r;
}
static inline dual dcos(dual a) {
  dual r;
  r.v = tog_cos(a.v);
  double c = -tog_sin(a.v);
  for (int i = 0; i < g_nd; i++) r.p[i] = c * a.p[i];
  return r;
}
static inline dual dsqrt(dual a) {
  dual r;
  r.v = sqrt(a.v);
  double c = 1.0 / (2.0 * r.v);
  for (int i = 0; i < g_nd; i++) r.p[i] = c * a.p[i];
  return r;
}
static inline dual dsq(dual a) { /* x^2 (literal_pow -> ^(Dual,2)): v^2, 2v*p */
  dual r;
  r.v = a.v * a.v;
  double c = 2.0 * a.v;
  for (int i = 0; i < g_nd; i++) r.p[i] = c * a.p[i];
  return r;
}

/* =====================================================================
 * Continuous dynamics f!(xdot, x, u) on duals
 * ===================================================================== */
static const int model_n[TOG_MODEL_COUNT] = {2, 4, 13, 3, 2, 14};
static const int model_m[TOG_MODEL_COUNT] = {1, 1, 4, 2, 1, 7};

/* dynamics/double_integrator.jl:1-4 */
static void f_double_integrator(dual* xd, const dual* x, const dual* u) {
  xd[0] = x[1];
  xd[1] = u[0];
}

/* dynamics/pendulum.jl:3-12 */
static void f_pendulum(dual* xd, const dual* x, const dual* u) {
  const double m = 1.0, b = 0.1, lc = 0.5, I = 0.25, g = 9.81;
  xd[0] = x[1];
  /* (u - m*g*lc*sin(x1) - b*x2)/I */
  dual t = dsub(dsub(u[0], dscale(dsin(x[0]), m * g * lc)), dscale(x[1], b));
  xd[1] = ddivc(t, I);
}

/* dynamics/car.jl:3-8 */
static void f_car(dual* xd, const dual* x, const dual* u) {
  xd[0] = dmul(u[0], dcos(x[2]));
  xd[1] = dmul(u[0], dsin(x[2]));
  xd[2] = u[1];
}

/* dynamics/cartpole.jl:9-36:  qdd = -H \ (C*qd + G - B*u), Julia generic LU (generic_lufact!,
   partial pivoting; |H11|=1.2 > |H21| so never swaps for finite q2) */
static void f_cartpole(dual* xd, const dual* x, const dual* u) {
  const double mc = 1.0, mp = 0.2, l = 0.5, g = 9.81;
  dual s, c;
  if (isfinite(x[1].v)) {
    s = dsin(x[1]);
    c = dcos(x[1]);
  } else { /* cartpole.jl:18-24 */
    s = dc(INFINITY);
    c = dc(INFINITY);
  }
  /* H = [mc+mp, mp*l*c; mp*l*c, mp*l^2] */
  dual H11 = dc(mc + mp);
  dual H12 = dscale(c, mp * l);
  dual H21 = H12;
  dual H22 = dc(mp * (l * l));
  /* C*qd + G - B*u : C = [0 -mp*qd2*l*s; 0 0], G = [0; mp*g*l*s], B=[1;0] */
  /* row 1: 0*qd1 + C12*qd2 + 0 - u ; C12 = -mp*qd[2]*l*s = ((-mp*qd2)*l)*s */
  dual C12 = dmul(dscale(dscale(x[3], -mp), l), s);
  dual r1 = dadd(dmul(dc(0.0), x[2]), dmul(C12, x[3]));
  r1 = dsub(dadd(r1, dc(0.0)), u[0]);
  /* row 2: 0*qd1 + 0*qd2 + mp*g*l*s - 0*u */
  dual r2 = dadd(dmul(dc(0.0), x[2]), dmul(dc(0.0), x[3]));
  r2 = dsub(dadd(r2, dscale(s, mp * g * l)), dscale(u[0], 0.0));
  /* generic LU (no pivot swap when |H11| >= |H21|) */
  dual a11 = H11, a12 = H12, a21 = H21, a22 = H22, b1 = r1, b2 = r2;
  if (fabs(a21.v) > fabs(a11.v)) { /* partial pivoting swap */
    dual t;
    t = a11; a11 = a21; a21 = t;
    t = a12; a12 = a22; a22 = t;
    t = b1; b1 = b2; b2 = t;
  }
  dual l21 = dmul(a21, dinv(a11));
  dual u22 = dsub(a22, dmul(l21, a12));
  dual y2 = dsub(b2, dmul(l21, b1));
  dual q2 = ddiv(y2, u22);
  dual q1 = ddiv(dsub(b1, dmul(a12, q2)), a11);
  xd[0] = x[2];
  xd[1] = x[3];
  xd[2] = dneg(q1);
  xd[3] = dneg(q2);
}

/* dynamics/quadrotor.jl:10-71 with dynamics/quaternions.jl:23-40.
   Hamilton product a⊗b = (aw*bw - av·bv, aw*bv + bw*av + av×bv); quaternions.jl:23-27 computes
   w = s1*s2 - v1'v2, v = s1*v2 + s2*v1 + v2×v1 with (q2,q1) = (a,b). */
static void qmul(dual* r, const dual* a, const dual* b) {
  /* q1 = b, q2 = a */
  dual s1 = b[0], s2 = a[0];
  const dual* v1 = b + 1;
  const dual* v2 = a + 1;
  dual dot = dadd(dadd(dmul(v1[0], v2[0]), dmul(v1[1], v2[1])), dmul(v1[2], v2[2]));
  r[0] = dsub(dmul(s1, s2), dot);
  /* cross(v2, v1) */
  dual cx = dsub(dmul(v2[1], v1[2]), dmul(v2[2], v1[1]));
  dual cy = dsub(dmul(v2[2], v1[0]), dmul(v2[0], v1[2]));
  dual cz = dsub(dmul(v2[0], v1[1]), dmul(v2[1], v1[0]));
  r[1] = dadd(dadd(dmul(s1, v2[0]), dmul(s2, v1[0])), cx);
  r[2] = dadd(dadd(dmul(s1, v2[1]), dmul(s2, v1[1])), cy);
  r[3] = dadd(dadd(dmul(s1, v2[2]), dmul(s2, v1[2])), cz);
}

static void f_quadrotor(dual* xd, const dual* x, const dual* u) {
  const double mass = 0.5, L = 0.175, kf = 1.0, km = 0.0245;
  const double Jd[3] = {0.0023, 0.0023, 0.004};
  const double Jinv[3] = {1.0 / 0.0023, 1.0 / 0.0023, 1.0 / 0.004};
  const double grav[3] = {0.0, 0.0, -9.81};
  /* q = normalize(Quaternion(x[4:7])) : StaticArrays normalize = inv(norm(a))*a */
  dual nrm2 = dadd(dadd(dadd(dmul(x[3], x[3]), dmul(x[4], x[4])), dmul(x[5], x[5])), dmul(x[6], x[6]));
  dual inrm = dinv(dsqrt(nrm2));
  dual q[4];
  for (int i = 0; i < 4; i++) q[i] = dmul(inrm, x[3 + i]);
  const dual* v = x + 7;
  const dual* om = x + 10;
  dual F1 = dscale(u[0], kf), F2 = dscale(u[1], kf), F3 = dscale(u[2], kf), F4 = dscale(u[3], kf);
  dual Fz = dadd(dadd(dadd(F1, F2), F3), F4);
  dual M1 = dscale(u[0], km), M2 = dscale(u[1], km), M3 = dscale(u[2], km), M4 = dscale(u[3], km);
  dual tau[3];
  tau[0] = dscale(dsub(F2, F4), L);
  tau[1] = dscale(dsub(F3, F1), L);
  tau[2] = dsub(dadd(dsub(M1, M2), M3), M4);
  /* xd[1:3] = v */
  xd[0] = v[0];
  xd[1] = v[1];
  xd[2] = v[2];
  /* xd[4:7] = 0.5*q*Quaternion(0, omega) */
  dual hq[4], w4[4], qd[4];
  for (int i = 0; i < 4; i++) hq[i] = dscale(q[i], 0.5);
  w4[0] = dc(0.0);
  w4[1] = om[0];
  w4[2] = om[1];
  w4[3] = om[2];
  qmul(qd, hq, w4);
  for (int i = 0; i < 4; i++) xd[3 + i] = qd[i];
  /* xd[8:10] = g + (1/m)*(q*F),  q*F = vec(q*Quaternion(0,F)*inv(q)) */
  dual F4q[4], t1[4], qinv[4], t2[4];
  F4q[0] = dc(0.0);
  F4q[1] = dc(0.0);
  F4q[2] = dc(0.0);
  F4q[3] = Fz;
  qmul(t1, q, F4q);
  qinv[0] = q[0];
  qinv[1] = dneg(q[1]);
  qinv[2] = dneg(q[2]);
  qinv[3] = dneg(q[3]);
  qmul(t2, t1, qinv);
  for (int i = 0; i < 3; i++) xd[7 + i] = dadd(dc(grav[i]), dscale(t2[1 + i], 1.0 / mass));
  /* xd[11:13] = Jinv*(tau - cross(omega, J*omega)) (diagonal J, Jinv) */
  dual Jw[3];
  for (int i = 0; i < 3; i++) Jw[i] = dscale(om[i], Jd[i]);
  dual cr[3];
  cr[0] = dsub(dmul(om[1], Jw[2]), dmul(om[2], Jw[1]));
  cr[1] = dsub(dmul(om[2], Jw[0]), dmul(om[0], Jw[2]));
  cr[2] = dsub(dmul(om[0], Jw[1]), dmul(om[1], Jw[0]));
  for (int i = 0; i < 3; i++) xd[10 + i] = dscale(dsub(tau[i], cr[i]), Jinv[i]);
}

/* =====================================================================
 * Kuka iiwa 7-DoF (BASELINE config 5): Model(urdf) src/model.jl:394-431 -> RigidBodyDynamics
 * v2.1.0 dynamics!(ẋ, result, state, x, τ = I₇·u): q̇ = v, v̇ = M(q)⁻¹(τ − c(q,v)).
 * RBD itself (Manifest.toml:467-472) is absent here; this restates its published algorithms:
 * c(q,v) by recursive Newton-Euler with v̇ = 0 and the base accelerating at −g (dynamics_bias!),
 * M(q) by the composite-rigid-body algorithm (mass_matrix!), then a Cholesky solve (RBD's
 * dynamics_solve! for BLAS floats). Spatial quantities are carried in body coordinates
 * (Featherstone); RBD works in world coordinates, so values agree with RBD to rounding only:
 * PARITY UNPINNED against RBD; pinned to physics by tests/test_kuka.py. The HIP
 * model (csrc/tog_device.hpp Kuka) performs the identical operation sequence.
 * Kinematic/inertial tables: include/tog_kuka.h (from dynamics/urdf/kuka_iiwa.urdf:76-290).
 * ===================================================================== */
static const double KK_R0[7][9] = TOG_KUKA_R0;
static const double KK_P[7][3] = TOG_KUKA_P;
static const double KK_MASS[7] = TOG_KUKA_MASS;
static const double KK_COM[7][3] = TOG_KUKA_COM;
static const double KK_IC[7][6] = TOG_KUKA_IC;

/* dual + real constant: partials untouched (ForwardDiff +(::Dual, ::Real)) */
static inline dual daddc(dual a, double s) {
  a.v = a.v + s;
  return a;
}
/* body first moment h = m·c and inertia about the body origin IO = Ic + m(|c|²1 − c cᵀ) */
static void kk_body(int j, double* h, double IO[3][3]) {
  const double m = KK_MASS[j];
  const double* c = KK_COM[j];
  const double* I = KK_IC[j];
  const double cc = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
  const double Ic[3][3] = {{I[0], I[1], I[2]}, {I[1], I[3], I[4]}, {I[2], I[4], I[5]}};
  for (int a = 0; a < 3; a++) {
    h[a] = m * c[a];
    for (int b = 0; b < 3; b++) IO[a][b] = Ic[a][b] + m * ((a == b ? cc : 0.0) - c[a] * c[b]);
  }
}
/* y = R0ᵀ x (parent -> joint frame) and y = R0 x (joint -> parent) */
static void kk_r0t(int j, dual* y, const dual* x) {
  const double* R = KK_R0[j];
  for (int a = 0; a < 3; a++) y[a] = dadd(dadd(dscale(x[0], R[a]), dscale(x[1], R[3 + a])), dscale(x[2], R[6 + a]));
}
static void kk_r0(int j, dual* y, const dual* x) {
  const double* R = KK_R0[j];
  for (int a = 0; a < 3; a++)
    y[a] = dadd(dadd(dscale(x[0], R[3 * a]), dscale(x[1], R[3 * a + 1])), dscale(x[2], R[3 * a + 2]));
}
/* E x = Rz(q)ᵀ R0ᵀ x (parent -> child body) */
static void kk_E(int j, dual c, dual s, dual* y, const dual* x) {
  dual t[3];
  kk_r0t(j, t, x);
  y[0] = dadd(dmul(c, t[0]), dmul(s, t[1]));
  y[1] = dsub(dmul(c, t[1]), dmul(s, t[0]));
  y[2] = t[2];
}
/* Eᵀ x = R0 Rz(q) x (child body -> parent) */
static void kk_Et(int j, dual c, dual s, dual* y, const dual* x) {
  dual t[3];
  t[0] = dsub(dmul(c, x[0]), dmul(s, x[1]));
  t[1] = dadd(dmul(s, x[0]), dmul(c, x[1]));
  t[2] = x[2];
  kk_r0(j, y, t);
}
static void kk_cross(dual* y, const dual* a, const dual* b) {
  y[0] = dsub(dmul(a[1], b[2]), dmul(a[2], b[1]));
  y[1] = dsub(dmul(a[2], b[0]), dmul(a[0], b[2]));
  y[2] = dsub(dmul(a[0], b[1]), dmul(a[1], b[0]));
}
static void kk_cross_dc(dual* y, const dual* a, const double* r) { /* a × r, r constant */
  y[0] = dsub(dscale(a[1], r[2]), dscale(a[2], r[1]));
  y[1] = dsub(dscale(a[2], r[0]), dscale(a[0], r[2]));
  y[2] = dsub(dscale(a[0], r[1]), dscale(a[1], r[0]));
}
static void kk_cross_cd(dual* y, const double* r, const dual* b) { /* r × b, r constant */
  y[0] = dsub(dscale(b[2], r[1]), dscale(b[1], r[2]));
  y[1] = dsub(dscale(b[0], r[2]), dscale(b[2], r[0]));
  y[2] = dsub(dscale(b[1], r[0]), dscale(b[0], r[1]));
}
static void kk_symv(dual* y, const double IO[3][3], const dual* x) {
  for (int a = 0; a < 3; a++) y[a] = dadd(dadd(dscale(x[0], IO[a][0]), dscale(x[1], IO[a][1])), dscale(x[2], IO[a][2]));
}
/* spatial inertia times motion: [IO w + h × v ; m v − h × w] */
static void kk_inertia_mul(int j, dual* ang, dual* lin, const dual* w, const dual* v) {
  double h[3], IO[3][3];
  kk_body(j, h, IO);
  dual t[3], hx[3];
  kk_symv(t, IO, w);
  kk_cross_cd(hx, h, v);
  for (int a = 0; a < 3; a++) ang[a] = dadd(t[a], hx[a]);
  kk_cross_cd(hx, h, w);
  for (int a = 0; a < 3; a++) lin[a] = dsub(dscale(v[a], KK_MASS[j]), hx[a]);
}

/* dynamics_bias (RNEA, v̇ = 0) into tau[7]; also the per-joint cos/sin for reuse */
static void kk_bias(dual* tau, dual* cq, dual* sq, const dual* q, const dual* qd) {
  dual w[3], v[3], al[3], ln[3]; /* parent body: angular/linear velocity, acceleration */
  dual nf[7][3], ff[7][3];
  for (int a = 0; a < 3; a++) {
    w[a] = dc(0.0);
    v[a] = dc(0.0);
    al[a] = dc(0.0);
    ln[a] = dc(0.0);
  }
  ln[2] = dc(TOG_KUKA_GRAVITY); /* base acceleration −g, g = (0, 0, −9.81) */
  for (int j = 0; j < 7; j++) {
    const double* r = KK_P[j];
    cq[j] = dcos(q[j]);
    sq[j] = dsin(q[j]);
    dual t[3], tv[3], wj[3], vj[3], aj[3], lj[3];
    kk_cross_dc(t, w, r);
    for (int a = 0; a < 3; a++) tv[a] = dadd(v[a], t[a]);
    kk_E(j, cq[j], sq[j], wj, w);
    kk_E(j, cq[j], sq[j], vj, tv);
    wj[2] = dadd(wj[2], qd[j]);
    kk_cross_dc(t, al, r);
    for (int a = 0; a < 3; a++) tv[a] = dadd(ln[a], t[a]);
    kk_E(j, cq[j], sq[j], aj, al);
    kk_E(j, cq[j], sq[j], lj, tv);
    /* + v_j ×ₘ (S q̇_j), S = angular z */
    aj[0] = dadd(aj[0], dmul(wj[1], qd[j]));
    aj[1] = dsub(aj[1], dmul(wj[0], qd[j]));
    lj[0] = dadd(lj[0], dmul(vj[1], qd[j]));
    lj[1] = dsub(lj[1], dmul(vj[0], qd[j]));
    /* f = I a + v ×* (I v) */
    dual hva[3], hvl[3], iaa[3], ial[3], c1[3], c2[3];
    kk_inertia_mul(j, hva, hvl, wj, vj);
    kk_inertia_mul(j, iaa, ial, aj, lj);
    kk_cross(c1, wj, hva);
    kk_cross(c2, vj, hvl);
    for (int a = 0; a < 3; a++) nf[j][a] = dadd(iaa[a], dadd(c1[a], c2[a]));
    kk_cross(c1, wj, hvl);
    for (int a = 0; a < 3; a++) ff[j][a] = dadd(ial[a], c1[a]);
    for (int a = 0; a < 3; a++) {
      w[a] = wj[a];
      v[a] = vj[a];
      al[a] = aj[a];
      ln[a] = lj[a];
    }
  }
  for (int j = 6; j >= 0; j--) {
    tau[j] = nf[j][2];
    if (j > 0) {
      dual fp[3], np[3], rx[3];
      kk_Et(j, cq[j], sq[j], fp, ff[j]);
      kk_Et(j, cq[j], sq[j], np, nf[j]);
      kk_cross_cd(rx, KK_P[j], fp);
      for (int a = 0; a < 3; a++) {
        np[a] = dadd(np[a], rx[a]);
        nf[j - 1][a] = dadd(nf[j - 1][a], np[a]);
        ff[j - 1][a] = dadd(ff[j - 1][a], fp[a]);
      }
    }
  }
}

/* mass_matrix! by CRBA: lower triangle M[i][j], i >= j */
static void kk_mass(dual M[7][7], const dual* cq, const dual* sq) {
  double mc = KK_MASS[6], h0[3], IO0[3][3];
  dual hc[3], Ic[3][3];
  kk_body(6, h0, IO0);
  for (int a = 0; a < 3; a++) {
    hc[a] = dc(h0[a]);
    for (int b = 0; b < 3; b++) Ic[a][b] = dc(IO0[a][b]);
  }
  for (int j = 6; j >= 0; j--) {
    dual Fa[3], Fl[3];
    for (int a = 0; a < 3; a++) Fa[a] = Ic[a][2];
    Fl[0] = dneg(hc[1]);
    Fl[1] = hc[0];
    Fl[2] = dc(0.0);
    M[j][j] = Fa[2];
    for (int k = j; k >= 1; k--) {
      dual fl[3], fa[3], rx[3];
      kk_Et(k, cq[k], sq[k], fl, Fl);
      kk_Et(k, cq[k], sq[k], fa, Fa);
      kk_cross_cd(rx, KK_P[k], fl);
      for (int a = 0; a < 3; a++) {
        Fa[a] = dadd(fa[a], rx[a]);
        Fl[a] = fl[a];
      }
      M[j][k - 1] = Fa[2];
    }
    if (j > 0) {
      const double* r = KK_P[j];
      dual hr[3], W[3][3], col[3], row[3], Ir[3][3];
      kk_Et(j, cq[j], sq[j], hr, hc);
      for (int b = 0; b < 3; b++) { /* W = Eᵀ Ic (columns) */
        for (int a = 0; a < 3; a++) col[a] = Ic[a][b];
        kk_Et(j, cq[j], sq[j], row, col);
        for (int a = 0; a < 3; a++) W[a][b] = row[a];
      }
      for (int a = 0; a < 3; a++) { /* Ir = W E (rows) */
        kk_Et(j, cq[j], sq[j], row, W[a]);
        for (int b = 0; b < 3; b++) Ir[a][b] = row[b];
      }
      const double rr = (r[0] * r[0] + r[1] * r[1]) + r[2] * r[2];
      dual dot = dadd(dadd(dscale(hr[0], r[0]), dscale(hr[1], r[1])), dscale(hr[2], r[2]));
      dual sh = daddc(dscale(dot, 2.0), mc * rr);
      double hb[3], IOb[3][3];
      kk_body(j - 1, hb, IOb);
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
          dual t = dsub(Ir[a][b], dadd(dscale(hr[a], r[b]), dscale(hr[b], r[a])));
          t = daddc(t, -((mc * r[a]) * r[b]));
          if (a == b) t = dadd(t, sh);
          Ic[a][b] = daddc(t, IOb[a][b]);
        }
      for (int a = 0; a < 3; a++) hc[a] = daddc(daddc(hr[a], mc * r[a]), hb[a]);
      mc = mc + KK_MASS[j - 1];
    }
  }
}

static void f_kuka(dual* xd, const dual* x, const dual* u) {
  const dual* q = x;
  const dual* qd = x + 7;
  dual tau[7], cq[7], sq[7], M[7][7], L[7][7], y[7];
  kk_bias(tau, cq, sq, q, qd);
  kk_mass(M, cq, sq);
  for (int j = 0; j < 7; j++) { /* Cholesky M = L Lᵀ */
    dual s = M[j][j];
    for (int k = 0; k < j; k++) s = dsub(s, dmul(L[j][k], L[j][k]));
    L[j][j] = dsqrt(s);
    for (int i = j + 1; i < 7; i++) {
      dual t = M[i][j];
      for (int k = 0; k < j; k++) t = dsub(t, dmul(L[i][k], L[j][k]));
      L[i][j] = ddiv(t, L[j][j]);
    }
  }
  for (int i = 0; i < 7; i++) {
    dual t = dsub(u[i], tau[i]);
    for (int k = 0; k < i; k++) t = dsub(t, dmul(L[i][k], y[k]));
    y[i] = ddiv(t, L[i][i]);
  }
  for (int i = 6; i >= 0; i--) {
    dual t = y[i];
    for (int k = i + 1; k < 7; k++) t = dsub(t, dmul(L[k][i], xd[7 + k]));
    xd[7 + i] = ddiv(t, L[i][i]);
  }
  for (int i = 0; i < 7; i++) xd[i] = qd[i];
}

/* dynamics_bias(state) at (q, v): the hold torque of dynamics/kuka.jl:117-132 (v = 0) */
OC_EXPORT void oc_kuka_bias(double* tau, const double* q, const double* v) {
  int save = g_nd;
  g_nd = 0;
  dual Q[7], V[7], T[7], c[7], s[7];
  for (int i = 0; i < 7; i++) {
    Q[i].v = q[i];
    V[i].v = v[i];
  }
  kk_bias(T, c, s, Q, V);
  for (int i = 0; i < 7; i++) tau[i] = T[i].v;
  g_nd = save;
}
/* mass_matrix(state) (full, symmetric) for tests */
OC_EXPORT void oc_kuka_mass(double* Mout, const double* q) {
  int save = g_nd;
  g_nd = 0;
  dual Q[7], c[7], s[7], M[7][7];
  for (int i = 0; i < 7; i++) {
    Q[i].v = q[i];
    c[i] = dcos(Q[i]);
    s[i] = dsin(Q[i]);
  }
  kk_mass(M, c, s);
  for (int i = 0; i < 7; i++)
    for (int j = 0; j <= i; j++) Mout[i + 7 * j] = Mout[j + 7 * i] = M[i][j].v;
  g_nd = save;
}

static void model_f(int model, dual* xd, const dual* x, const dual* u) {
  switch (model) {
    case TOG_MODEL_DOUBLE_INTEGRATOR: f_double_integrator(xd, x, u); break;
    case TOG_MODEL_CARTPOLE: f_cartpole(xd, x, u); break;
    case TOG_MODEL_QUADROTOR: f_quadrotor(xd, x, u); break;
    case TOG_MODEL_CAR: f_car(xd, x, u); break;
    case TOG_MODEL_PENDULUM: f_pendulum(xd, x, u); break;
    case TOG_MODEL_KUKA: f_kuka(xd, x, u); break;
  }
}

/* ---------------------------------------------------------------------------------------------
 * Implicit integrators (src/integration.jl:44-73 midpoint_implicit, :171-205 rk3_implicit).
 * The reference differentiates fd! with ForwardDiff straight through the Newton loop, so its
 * iterate y and residual g carry partials, and ∇g = I - ½dt·∇f(Xm) is itself a nested-dual matrix.
 * This restatement runs the same loop on duals with ∇g taken at the values only: the dropped term
 * is (∇g⁻¹)' g, which vanishes with g, so the Jacobian agrees with the reference's to the loop's
 * own tolerance (‖g‖ <= 1e-12), and the values are the reference's loop exactly.
 * Parity trap (reproduced): rk3_implicit writes `fc1 = fc2 = fc3 = zero(x)`, one array under three
 * names, so after f(fc1,x,u); f(fc3,y,u) the midpoint term dt/8*(fc1 - fc3) is F - F, and
 * g = y - x - dt/6*F - 4/6*dt*F - dt/6*F with F = f(Xm) for all three.
 * --------------------------------------------------------------------------------------------- */
static void model_f(int model, dual* xd, const dual* x, const dual* u);

/* ∂f/∂x at the values of (x, u): ForwardDiff.jacobian(f_aug, zero(x), [x;u])[:, 1:n], one partial
   per column (each partial of a dual evaluation is independent of the others) */
static void jac_x_val(int model, int n, int m, double* A, const dual* x, const dual* u) {
  int save = g_nd;
  g_nd = 1;
  for (int j = 0; j < n; j++) {
    dual X[16], U[OM], F[16];
    for (int i = 0; i < n; i++) {
      X[i].v = x[i].v;
      X[i].p[0] = (i == j) ? 1.0 : 0.0;
    }
    for (int i = 0; i < m; i++) {
      U[i].v = u[i].v;
      U[i].p[0] = 0.0;
    }
    model_f(model, F, X, U);
    for (int i = 0; i < n; i++) A[i + n * j] = F[i].p[0];
  }
  g_nd = save;
}

/* LinearAlgebra.generic_norm2 (Julia 1.1): unscaled sum of squares when n·max² is finite and
   nonzero, else scaled by max|g| (NaN propagates) */
static double jl_norm2(const double* g, int n) {
  double mx = 0.0;
  for (int i = 0; i < n; i++) mx = tog_jlmax(mx, fabs(g[i]));
  if (mx != mx || mx == 0.0 || isinf(mx)) return mx;
  if (isfinite((double)n * mx * mx) && mx * mx != 0.0) {
    double s = g[0] * g[0];
    for (int i = 1; i < n; i++) s = s + g[i] * g[i];
    return sqrt(s);
  }
  double t = fabs(g[0]) / mx, s = t * t;
  for (int i = 1; i < n; i++) {
    t = fabs(g[i]) / mx;
    s = s + t * t;
  }
  return mx * sqrt(s);
}

/* δ = (-G) \ b (the reference's `-∇g\g` parses as (-∇g)\g): generic_lufact! with partial pivoting
   (first max |a_ik|, reciprocal scaling, column-by-column rank-1 updates), row swaps applied to b in
   order, unit-lower forward and upper backward substitution (naivesub!, column oriented). b is
   dual; the factor is real. */
static void lu_neg_solve(int n, const double* G, dual* b) {
  double a[16 * 16];
  for (int e = 0; e < n * n; e++) a[e] = -G[e];
  int piv[16];
  for (int k = 0; k < n; k++) {
    int kp = k;
    double amax = 0.0;
    for (int i = k; i < n; i++) {
      double ai = fabs(a[i + n * k]);
      if (ai > amax) {
        kp = i;
        amax = ai;
      }
    }
    piv[k] = kp;
    if (a[kp + n * k] != 0.0) {
      if (kp != k)
        for (int j = 0; j < n; j++) {
          double t = a[k + n * j];
          a[k + n * j] = a[kp + n * j];
          a[kp + n * j] = t;
        }
      double inv = 1.0 / a[k + n * k];
      for (int i = k + 1; i < n; i++) a[i + n * k] = a[i + n * k] * inv;
    }
    for (int j = k + 1; j < n; j++)
      for (int i = k + 1; i < n; i++) a[i + n * j] = a[i + n * j] - a[i + n * k] * a[k + n * j];
  }
  for (int k = 0; k < n; k++)
    if (piv[k] != k) {
      dual t = b[k];
      b[k] = b[piv[k]];
      b[piv[k]] = t;
    }
  for (int j = 0; j < n; j++)
    for (int i = j + 1; i < n; i++) b[i] = dsub(b[i], dscale(b[j], a[i + n * j]));
  for (int j = n - 1; j >= 0; j--) {
    b[j] = ddivc(b[j], a[j + n * j]);
    for (int i = j - 1; i >= 0; i--) b[i] = dsub(b[i], dscale(b[j], a[i + n * j]));
  }
}

static void implicit_step_dual(int model, int integ, int n, int m, dual* y, const dual* x, const dual* u, dual dt) {
  for (int i = 0; i < n; i++) y[i] = x[i];
  double gn = INFINITY;
  int cnt = 0;
  while (gn > 1e-12) {
    if (++cnt > 1000) { /* error("Integration convergence fail"): the state becomes NaN here */
      for (int i = 0; i < n; i++) y[i] = dc(NAN);
      return;
    }
    dual g[16], xm[16], F[16];
    double G[16 * 16], A[16 * 16];
    if (integ == TOG_MIDPOINT_IMPLICIT) {
      for (int i = 0; i < n; i++) xm[i] = dscale(dadd(x[i], y[i]), 0.5); /* Xm = 0.5*(x + y) */
      model_f(model, F, xm, u);                                            /* f(fc, Xm, u) */
      for (int i = 0; i < n; i++) g[i] = dsub(dsub(y[i], x[i]), dmul(dt, F[i])); /* y - x - dt*fc */
      jac_x_val(model, n, m, A, xm, u);
      double h = 0.5 * dt.v; /* ∇g = I - 0.5*dt*A */
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) G[i + n * j] = (i == j ? 1.0 : 0.0) - h * A[i + n * j];
    } else {
      dual d[16];
      model_f(model, F, y, u); /* f(fc1,x,u) then f(fc3,y,u) into the same array: F = f(y) */
      for (int i = 0; i < n; i++) d[i] = dsub(F[i], F[i]);
      dual dt8 = ddivc(dt, 8.0);
      for (int i = 0; i < n; i++) xm[i] = dadd(dscale(dadd(x[i], y[i]), 0.5), dmul(dt8, d[i]));
      model_f(model, F, xm, u); /* f(fc2, Xm, u): fc1 = fc2 = fc3 = f(Xm) */
      dual dt6 = ddivc(dt, 6.0), dt46 = dscale(dt, 4.0 / 6.0);
      for (int i = 0; i < n; i++)
        g[i] = dsub(dsub(dsub(dsub(y[i], x[i]), dmul(dt6, F[i])), dmul(dt46, F[i])), dmul(dt6, F[i]));
      double A2[16 * 16], M2[16 * 16];
      jac_x_val(model, n, m, A, xm, u); /* A1 */
      jac_x_val(model, n, m, A2, y, u);
      double c8 = dt.v / 8.0, c46 = (4.0 / 6.0) * dt.v, c6 = dt.v / 6.0;
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) M2[i + n * j] = (i == j ? 0.5 : 0.0) - c8 * A2[i + n * j];
      /* ∇g = I - (4/6*dt*A1)*(0.5I - dt/8*A2) - dt/6*A2, the product summed over k in order */
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) {
          double p = (c46 * A[i]) * M2[n * j];
          for (int k = 1; k < n; k++) p = p + (c46 * A[i + n * k]) * M2[k + n * j];
          G[i + n * j] = ((i == j ? 1.0 : 0.0) - p) - c6 * A2[i + n * j];
        }
    }
    double gv[16];
    for (int i = 0; i < n; i++) gv[i] = g[i].v;
    gn = jl_norm2(gv, n);
    lu_neg_solve(n, G, g); /* δy = -∇g\g */
    for (int i = 0; i < n; i++) y[i] = dadd(y[i], g[i]); /* y .+= δy */
  }
}

/* rk4: src/integration.jl:115-125 ; rk3: src/integration.jl:149-158 (dt is a Dual input) */
static void discrete_f_dual(int model, int integ, int n, dual* xn, const dual* x, const dual* u, dual dt) {
  dual k1[16], k2[16], k3[16], k4[16], t[16];
  if (integ == TOG_MIDPOINT_IMPLICIT || integ == TOG_RK3_IMPLICIT) {
    implicit_step_dual(model, integ, n, model_m[model], xn, x, u, dt);
    return;
  }
  if (integ == TOG_MIDPOINT) { /* src/integration.jl:26-33 */
    model_f(model, k1, x, u);
    dual h = ddivc(dt, 2.0); /* xdot .*= dt/2. */
    for (int i = 0; i < n; i++) k1[i] = dmul(k1[i], h);
    for (int i = 0; i < n; i++) t[i] = dadd(x[i], k1[i]);
    model_f(model, k2, t, u); /* f!(xdot, x + xdot, u) */
    for (int i = 0; i < n; i++) xn[i] = dadd(x[i], dmul(k2[i], dt)); /* x + xdot*dt */
    return;
  }
  model_f(model, k1, x, u);
  for (int i = 0; i < n; i++) k1[i] = dmul(k1[i], dt);
  for (int i = 0; i < n; i++) t[i] = dadd(x[i], ddivc(k1[i], 2.0));
  model_f(model, k2, t, u);
  for (int i = 0; i < n; i++) k2[i] = dmul(k2[i], dt);
  if (integ == TOG_RK4) {
    for (int i = 0; i < n; i++) t[i] = dadd(x[i], ddivc(k2[i], 2.0));
    model_f(model, k3, t, u);
    for (int i = 0; i < n; i++) k3[i] = dmul(k3[i], dt);
    for (int i = 0; i < n; i++) t[i] = dadd(x[i], k3[i]);
    model_f(model, k4, t, u);
    for (int i = 0; i < n; i++) k4[i] = dmul(k4[i], dt);
    /* x + (k1 + 2*k2 + 2*k3 + k4)/6 */
    for (int i = 0; i < n; i++) {
      dual s = dadd(dadd(dadd(k1[i], dscale(k2[i], 2.0)), dscale(k3[i], 2.0)), k4[i]);
      xn[i] = dadd(x[i], ddiv6(s));
    }
  } else {
    /* k3 = f(x - k1 + 2*k2) */
    for (int i = 0; i < n; i++) t[i] = dadd(dsub(x[i], k1[i]), dscale(k2[i], 2.0));
    model_f(model, k3, t, u);
    for (int i = 0; i < n; i++) k3[i] = dmul(k3[i], dt);
    /* x + (k1 + 4*k2 + k3)/6 */
    for (int i = 0; i < n; i++) {
      dual s = dadd(dadd(k1[i], dscale(k2[i], 4.0)), k3[i]);
      xn[i] = dadd(x[i], ddiv6(s));
    }
  }
}

/* evaluate!(ẋ, model::Model{M,Discrete}, x, u, dt)  src/model.jl:171-174 */
OC_EXPORT void oc_discrete_f(int model, int integ, double* xn, const double* x, const double* u, double dt) {
  int n = model_n[model], m = model_m[model];
  int save = g_nd;
  g_nd = 0;
  dual X[16], U[OM], XN[16];
  for (int i = 0; i < n; i++) X[i].v = x[i];
  for (int i = 0; i < m; i++) U[i].v = u[i];
  dual DT;
  DT.v = dt;
  discrete_f_dual(model, integ, n, XN, X, U, DT);
  for (int i = 0; i < n; i++) xn[i] = XN[i].v;
  g_nd = save;
}

/* continuous dynamics (for tests) */
OC_EXPORT void oc_continuous_f(int model, double* xd, const double* x, const double* u) {
  int n = model_n[model], m = model_m[model];
  g_nd = 0;
  dual X[16], U[OM], XD[16];
  for (int i = 0; i < n; i++) X[i].v = x[i];
  for (int i = 0; i < m; i++) U[i].v = u[i];
  model_f(model, XD, X, U);
  for (int i = 0; i < n; i++) xd[i] = XD[i].v;
}

/* ∇fd!(S, x, u, dt): ForwardDiff.jacobian!(S, fd_aug!, ẋ, [x;u;dt])  src/model.jl:491-512.
   S is n x (n+m+1) column-major, partitioned xx | xu | xdt (src/model.jl:341). Forward-mode duals
   straight through the integrator. */
static void discrete_jacobian_fd(int model, int integ, double* S, const double* x, const double* u, double dt) {
  int n = model_n[model], m = model_m[model];
  int L = n + m + 1;
  g_nd = L;
  dual X[16], U[OM], XN[16], DT;
  for (int i = 0; i < n; i++) {
    X[i] = dc(x[i]);
    X[i].p[i] = 1.0;
  }
  for (int i = 0; i < m; i++) {
    U[i] = dc(u[i]);
    U[i].p[n + i] = 1.0;
  }
  DT = dc(dt);
  DT.p[n + m] = 1.0;
  discrete_f_dual(model, integ, n, XN, X, U, DT);
  for (int j = 0; j < L; j++)
    for (int i = 0; i < n; i++) S[i + n * j] = XN[i].p[j];
  g_nd = 0;
}

/* The Kuka iiwa's RK3 Jacobian, "stage-chain" form (contract deviations): the same
   derivative as forward-mode duals through rk3 (src/integration.jl:149-158), evaluated as
     J_s = ∂f/∂[s; u] at each stage input s_1 = x, s_2 = x + k1/2, s_3 = (x - k1) + 2 k2 (dual numbers
           seeded at the stage input, 21 partials; the primal stage inputs are discrete_step's),
     K1 = J_1 dt,  T2 = I + K1/2,  F2 = J_2 [T2; E_u],  K2 = F2 dt,  T3 = (I - K1) + 2 K2,
     F3 = J_3 [T3; E_u],  K3 = F3 dt,  [A B] = I + ((K1 + 4 K2) + K3)/6,
   with RK3's elementwise operations in discrete_step's order and the two chain products as fma chains
   over j = 0..13, started from J_s's u column (0 for the x columns): the accumulation order of the
   fp64 matrix cores (v_mfma_f64_16x16x4_f64, k in order, tools/microbench/mfma_f64_order.hip) that
   evaluate them on the device (k_kuka_chain). Rows 0..6 of f are q̇ = v, so F rows 0..6 are T rows
   7..13. RigidBodyDynamics' own operation order is not reproduced either way; the
   notebook pin (tests/test_kuka.py) holds for both forms. */
static void kuka_rk3_jacobian_chain(double* S, const double* x, const double* u, double dt) {
  enum { n = 14, m = 7, L = 21 };
  const int save = g_nd;
  double k1[n], t2[n], t3[n];
  { /* primal stage inputs (discrete_f_dual's rk3 values) */
    g_nd = 0;
    dual X[n], U[m], F[n];
    for (int i = 0; i < n; i++) X[i] = dc(x[i]);
    for (int i = 0; i < m; i++) U[i] = dc(u[i]);
    f_kuka(F, X, U);
    for (int i = 0; i < n; i++) {
      k1[i] = F[i].v * dt;
      t2[i] = x[i] + k1[i] / 2.0;
    }
    for (int i = 0; i < n; i++) X[i] = dc(t2[i]);
    f_kuka(F, X, U);
    for (int i = 0; i < n; i++) t3[i] = (x[i] - k1[i]) + 2.0 * (F[i].v * dt);
  }
  double J[3][7][L]; /* rows 7..13 of J_s */
  const double* pts[3] = {x, t2, t3};
  g_nd = L;
  for (int st = 0; st < 3; st++) {
    dual Xs[n], Us[m], Fs[n];
    for (int i = 0; i < n; i++) {
      Xs[i] = dc(pts[st][i]);
      Xs[i].p[i] = 1.0;
    }
    for (int i = 0; i < m; i++) {
      Us[i] = dc(u[i]);
      Us[i].p[n + i] = 1.0;
    }
    f_kuka(Fs, Xs, Us);
    for (int i = 0; i < 7; i++)
      for (int p = 0; p < L; p++) J[st][i][p] = Fs[7 + i].p[p];
  }
  g_nd = save;
  static _Thread_local double K1[n][L], T[n][L], K2[n][L], Ssum[n][L];
  for (int i = 0; i < n; i++)
    for (int p = 0; p < L; p++) {
      const double f1 = (i < 7) ? ((p == 7 + i) ? 1.0 : 0.0) : J[0][i - 7][p];
      K1[i][p] = f1 * dt;
      T[i][p] = ((i == p) ? 1.0 : 0.0) + K1[i][p] / 2.0;
    }
  for (int st = 1; st < 3; st++) {
    double F[n][L];
    for (int p = 0; p < L; p++)
      for (int i = 0; i < n; i++) {
        if (i < 7) {
          F[i][p] = T[7 + i][p];
        } else {
          double acc = (p >= n) ? J[st][i - 7][p] : 0.0;
          for (int j = 0; j < n; j++) acc = fma(J[st][i - 7][j], T[j][p], acc);
          F[i][p] = acc;
        }
      }
    for (int i = 0; i < n; i++)
      for (int p = 0; p < L; p++) {
        const double kk = F[i][p] * dt;
        if (st == 1) {
          K2[i][p] = kk;
          T[i][p] = (((i == p) ? 1.0 : 0.0) - K1[i][p]) + 2.0 * kk;
          Ssum[i][p] = K1[i][p] + 4.0 * kk;
        } else {
          Ssum[i][p] = Ssum[i][p] + kk;
          S[i + n * p] = ((i == p) ? 1.0 : 0.0) + tog_div6(Ssum[i][p]);
        }
      }
  }
}

OC_EXPORT void oc_discrete_jacobian(int model, int integ, double* S, const double* x, const double* u, double dt) {
  discrete_jacobian_fd(model, integ, S, x, u, dt); /* (the dt column) */
#ifndef TOG_ORACLE_LITERAL /* literal: ForwardDiff through rk3, as the reference */
  if (model == TOG_MODEL_KUKA && integ == TOG_RK3) kuka_rk3_jacobian_chain(S, x, u, dt);
#endif
}
/* forward-mode duals through the integrator for every model (tests: the stage-chain form against it) */
OC_EXPORT void oc_discrete_jacobian_fd(int model, int integ, double* S, const double* x, const double* u, double dt) {
  discrete_jacobian_fd(model, integ, S, x, u, dt);
}

OC_EXPORT int oc_model_n(int model) { return model_n[model]; }
OC_EXPORT int oc_model_m(int model) { return model_m[model]; }

/* =====================================================================
 * Small dense linear algebra (column-major), restating Julia 1.1 / LAPACK
 * ===================================================================== */
#define IDX(i, j, ld) ((i) + (size_t)(j) * (ld))

/* C(r x c) = A^T(r x k) * B(k x c) where A is k x r */
static void matTmul(double* C, const double* A, int k, int r, const double* B, int c) {
  for (int j = 0; j < c; j++)
    for (int i = 0; i < r; i++) {
      double s = 0.0;
      for (int l = 0; l < k; l++) s = fma(A[IDX(l, i, k)], B[IDX(l, j, k)], s);
      C[IDX(i, j, r)] = s;
    }
}
/* C(r x c) = A(r x k) * B(k x c) */
static void matmul(double* C, const double* A, int r, int k, const double* B, int c) {
  for (int j = 0; j < c; j++)
    for (int i = 0; i < r; i++) {
      double s = 0.0;
      for (int l = 0; l < k; l++) s = fma(A[IDX(i, l, r)], B[IDX(l, j, k)], s);
      C[IDX(i, j, r)] = s;
    }
}

/* R factor of qr(P) for P (rows x cols), rows >= cols, LAPACK dgeqr2/dlarfg Householder.
   Julia: qr(P).R (chol_plus, backward_pass.jl:172-183). Writes the cols x cols upper triangle to R.
   Arithmetic contract v2, shared bit for bit with the device QRs:
   * sums over the rows below the diagonal (‖x‖², the reflector dot products) run in 4 interleaved
     accumulators, term t = i-(j+1) into accumulator t & 3, combined as (a0 + a1) + (a2 + a3): the
     dependent chain is a quarter as long (LAPACK's dnrm2 also reorders; the values agree to rounding);
   * β = -sign(α)·sqrt(α² + ‖x‖²) with one fma and one sqrt (dlapy2's rescaling only matters near
     overflow);
   contract v3: the reflector is kept unnormalised, v = [α-β; x] (dlarfg divides x by α-β and keeps
   τ = (β-α)/β; H = I - τ v̂v̂' is the same matrix). With v'v = -2β(α-β), H y = y + v·(v'y)/(β(α-β)):
   one reciprocal 1/(β(α-β)) per column, no scaling pass over the column, and every applied column
   costs one fma per row for v'y and one for the update. */
static double sum4(const double* a) { return (a[0] + a[1]) + (a[2] + a[3]); }

#ifdef TOG_ORACLE_LITERAL
/* Literal mode (TOG_ORACLE_LITERAL, liboracle_literal.so): the reference's own arithmetic
   where the contract deviates from it. Householder QR as LAPACK's unblocked dgeqr2: dlarfg's
   normalised reflector (xnorm = dnrm2 as a plain sequential sum of squares, β = -sign(α) dlapy2(α,
   xnorm), τ = (β-α)/β, x scaled by 1/(α-β)), dlarf's application (w = Cᵀv summed in row order,
   C -= τ v wᵀ). Julia 1.1's qr(P) calls dgeqrt (compact WY): the same reflectors applied through
   blocked updates, i.e. this is the reference up to the blocking's rounding. */
static double dlapy2(double x, double y) {
  const double xa = fabs(x), ya = fabs(y), w = xa > ya ? xa : ya, z = xa < ya ? xa : ya;
  if (z == 0.0) return w;
  const double q = z / w;
  return w * sqrt(1.0 + q * q);
}
static void qr_R(double* R, double* P, int rows, int cols) {
  int kmax = rows < cols ? rows : cols;
  for (int j = 0; j < kmax; j++) {
    double alpha = P[IDX(j, j, rows)];
    double ss = 0.0;
    for (int i = j + 1; i < rows; i++) ss = ss + P[IDX(i, j, rows)] * P[IDX(i, j, rows)];
    const double xnorm = sqrt(ss);
    if (xnorm == 0.0) continue; /* τ = 0, H = I */
    const double beta = -copysign(dlapy2(alpha, xnorm), alpha);
    const double tau = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
    for (int i = j + 1; i < rows; i++) P[IDX(i, j, rows)] = P[IDX(i, j, rows)] * sc;
    P[IDX(j, j, rows)] = beta;
    for (int c = j + 1; c < cols; c++) { /* dlarf: v = [1; x], w = C'v, C = C - τ v w' */
      double w = P[IDX(j, c, rows)];
      for (int i = j + 1; i < rows; i++) w = w + P[IDX(i, j, rows)] * P[IDX(i, c, rows)];
      const double t = -tau * w;
      P[IDX(j, c, rows)] = P[IDX(j, c, rows)] + t;
      for (int i = j + 1; i < rows; i++) P[IDX(i, c, rows)] = P[IDX(i, c, rows)] + P[IDX(i, j, rows)] * t;
    }
  }
  for (int j = 0; j < cols; j++)
    for (int i = 0; i < cols; i++) R[IDX(i, j, cols)] = (i <= j && i < rows) ? P[IDX(i, j, rows)] : 0.0;
}
#else
static void qr_R(double* R, double* P, int rows, int cols) {
  int kmax = rows < cols ? rows : cols;
  for (int j = 0; j < kmax; j++) {
    double alpha = P[IDX(j, j, rows)];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = j + 1; i < rows; i++) acc[(i - j - 1) & 3] = fma(P[IDX(i, j, rows)], P[IDX(i, j, rows)], acc[(i - j - 1) & 3]);
    double ss = sum4(acc);
    if (ss == 0.0) continue; /* tau = 0, H = I */
    double beta = -copysign(sqrt(fma(alpha, alpha, ss)), alpha);
    double vd = alpha - beta;
    double rd = 1.0 / (beta * vd);
    P[IDX(j, j, rows)] = beta;
    /* apply H to P[j:rows, j+1:cols], v = [vd; P[j+1:rows, j]] */
    for (int c = j + 1; c < cols; c++) {
      double a4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int i = j + 1; i < rows; i++) a4[(i - j - 1) & 3] = fma(P[IDX(i, j, rows)], P[IDX(i, c, rows)], a4[(i - j - 1) & 3]);
      double p = fma(vd, P[IDX(j, c, rows)], sum4(a4)) * rd;
      P[IDX(j, c, rows)] = fma(vd, p, P[IDX(j, c, rows)]);
      for (int i = j + 1; i < rows; i++) P[IDX(i, c, rows)] = fma(P[IDX(i, j, rows)], p, P[IDX(i, c, rows)]);
    }
  }
  for (int j = 0; j < cols; j++)
    for (int i = 0; i < cols; i++) R[IDX(i, j, cols)] = (i <= j && i < rows) ? P[IDX(i, j, rows)] : 0.0;
}
#endif

/* Triangular solves of the square-root backward pass (contract v2): the diagonal reciprocals are
   formed first (independent divisions) and every substitution step multiplies by them, so the
   dependent chain per step is one multiply instead of one division (x_j = b_j·(1/U_jj)). */
#ifdef TOG_ORACLE_LITERAL
#define TOG_RCP_STEP(b, j) ((b) / A[IDX(j, j, n)]) /* literal: substitution by division (BLAS dtrsm) */
#else
#define TOG_RCP_STEP(b, j) ((b) * r[j])
#endif
static void solve_upper_rcp(const double* A, int n, double* B, int nrhs) { /* A upper: A \ B */
  double r[OM > 16 ? OM : 16];
  for (int j = 0; j < n; j++) r[j] = 1.0 / A[IDX(j, j, n)];
  for (int c = 0; c < nrhs; c++)
    for (int j = n - 1; j >= 0; j--) {
      double xj = TOG_RCP_STEP(B[IDX(j, c, n)], j);
      B[IDX(j, c, n)] = xj;
      for (int i = j - 1; i >= 0; i--) B[IDX(i, c, n)] = fma(-A[IDX(i, j, n)], xj, B[IDX(i, c, n)]);
    }
}
static void solve_uppert_rcp(const double* A, int n, double* B, int nrhs) { /* A upper: A' \ B */
  double r[OM > 16 ? OM : 16];
  for (int j = 0; j < n; j++) r[j] = 1.0 / A[IDX(j, j, n)];
  for (int c = 0; c < nrhs; c++)
    for (int j = 0; j < n; j++) {
      double xj = TOG_RCP_STEP(B[IDX(j, c, n)], j);
      B[IDX(j, c, n)] = xj;
      for (int i = j + 1; i < n; i++) B[IDX(i, c, n)] = fma(-A[IDX(j, i, n)], xj, B[IDX(i, c, n)]);
    }
}

/* chol_plus(A, B) = qr([A; B]).R, A n1 x c, B n2 x c (backward_pass.jl:172-179) */
static void chol_plus(double* R, const double* A, int n1, const double* B, int n2, int c) {
  int rows = n1 + n2;
  double* P = (double*)malloc(sizeof(double) * rows * c);
  for (int j = 0; j < c; j++) {
    for (int i = 0; i < n1; i++) P[IDX(i, j, rows)] = A[IDX(i, j, n1)];
    for (int i = 0; i < n2; i++) P[IDX(n1 + i, j, rows)] = B[IDX(i, j, n2)];
  }
  qr_R(R, P, rows, c);
  free(P);
}

/* upper Cholesky (dpotrf uplo=U) reading only the upper triangle; returns 0 on success
   (isposdef(Hermitian(A)), cholesky(A).U).  U written with zeros below the diagonal. */
static int chol_upper(double* Uo, const double* A, int n) {
  double* U = (double*)calloc((size_t)n * n, sizeof(double));
  int info = 0;
  for (int j = 0; j < n && !info; j++) {
    double s = A[IDX(j, j, n)];
    for (int k = 0; k < j; k++) s -= U[IDX(k, j, n)] * U[IDX(k, j, n)];
    if (!(s > 0.0)) {
      info = j + 1;
      break;
    }
    double ujj = sqrt(s);
    U[IDX(j, j, n)] = ujj;
    for (int c = j + 1; c < n; c++) {
      double t = A[IDX(j, c, n)];
      for (int k = 0; k < j; k++) t -= U[IDX(k, j, n)] * U[IDX(k, c, n)];
      U[IDX(j, c, n)] = t / ujj;
    }
  }
  if (!info && Uo) memcpy(Uo, U, sizeof(double) * n * n);
  free(U);
  return info;
}

/* X = A \ B with A n x n general (LU with partial pivoting, dgetrf/dgetrs; Julia `\`).
   Julia's `\` first checks istriu/istril and uses triangular substitution when applicable. */
static int is_triu(const double* A, int n) {
  for (int j = 0; j < n; j++)
    for (int i = j + 1; i < n; i++)
      if (A[IDX(i, j, n)] != 0.0) return 0;
  return 1;
}
static int is_tril(const double* A, int n) {
  for (int j = 0; j < n; j++)
    for (int i = 0; i < j; i++)
      if (A[IDX(i, j, n)] != 0.0) return 0;
  return 1;
}
static void solve_upper(const double* A, int n, double* B, int nrhs) {
  for (int c = 0; c < nrhs; c++)
    for (int j = n - 1; j >= 0; j--) {
      double xj = B[IDX(j, c, n)] / A[IDX(j, j, n)];
      B[IDX(j, c, n)] = xj;
      for (int i = j - 1; i >= 0; i--) B[IDX(i, c, n)] = fma(-A[IDX(i, j, n)], xj, B[IDX(i, c, n)]);
    }
}
static void solve_lower(const double* A, int n, double* B, int nrhs) {
  for (int c = 0; c < nrhs; c++)
    for (int j = 0; j < n; j++) {
      double xj = B[IDX(j, c, n)] / A[IDX(j, j, n)];
      B[IDX(j, c, n)] = xj;
      for (int i = j + 1; i < n; i++) B[IDX(i, c, n)] = fma(-A[IDX(i, j, n)], xj, B[IDX(i, c, n)]);
    }
}
static void lu_solve(const double* Ain, int n, double* B, int nrhs) {
  if (is_triu(Ain, n)) {
    solve_upper(Ain, n, B, nrhs);
    return;
  }
  if (is_tril(Ain, n)) {
    solve_lower(Ain, n, B, nrhs);
    return;
  }
  double* A = (double*)malloc(sizeof(double) * n * n);
  memcpy(A, Ain, sizeof(double) * n * n);
  int piv[32];
  for (int k = 0; k < n; k++) {
    int p = k;
    double amax = fabs(A[IDX(k, k, n)]);
    for (int i = k + 1; i < n; i++)
      if (fabs(A[IDX(i, k, n)]) > amax) {
        amax = fabs(A[IDX(i, k, n)]);
        p = i;
      }
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < n; j++) {
        double t = A[IDX(k, j, n)];
        A[IDX(k, j, n)] = A[IDX(p, j, n)];
        A[IDX(p, j, n)] = t;
      }
    double akk = A[IDX(k, k, n)];
    if (akk != 0.0) {
      double r = 1.0 / akk;
      for (int i = k + 1; i < n; i++) A[IDX(i, k, n)] *= r;
    }
    for (int j = k + 1; j < n; j++)
      for (int i = k + 1; i < n; i++) A[IDX(i, j, n)] = fma(-A[IDX(i, k, n)], A[IDX(k, j, n)], A[IDX(i, j, n)]);
  }
  for (int c = 0; c < nrhs; c++) {
    double* b = B + (size_t)c * n;
    for (int k = 0; k < n; k++)
      if (piv[k] != k) {
        double t = b[k];
        b[k] = b[piv[k]];
        b[piv[k]] = t;
      }
    for (int j = 0; j < n; j++)
      for (int i = j + 1; i < n; i++) b[i] = fma(-A[IDX(i, j, n)], b[j], b[i]);
    for (int j = n - 1; j >= 0; j--) {
      b[j] /= A[IDX(j, j, n)];
      for (int i = 0; i < j; i++) b[i] = fma(-A[IDX(i, j, n)], b[j], b[i]);
    }
  }
  free(A);
}

/* singular values of a small n x n matrix by one-sided Jacobi; returns cond = smax/smin (cond(A)) */
static double cond2(const double* Ain, int n) {
  double A[OM * OM], V[OM * OM];
  memcpy(A, Ain, sizeof(double) * n * n);
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0.0;
    for (int p = 0; p < n - 1; p++)
      for (int q = p + 1; q < n; q++) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int i = 0; i < n; i++) {
          alpha += A[IDX(i, p, n)] * A[IDX(i, p, n)];
          beta += A[IDX(i, q, n)] * A[IDX(i, q, n)];
          gamma += A[IDX(i, p, n)] * A[IDX(i, q, n)];
        }
        if (gamma == 0.0) continue;
        double c0 = fabs(gamma) / sqrt(alpha * beta);
        if (c0 > off) off = c0;
        if (c0 < 1e-15) continue;
        double zeta = (beta - alpha) / (2.0 * gamma);
        double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
        for (int i = 0; i < n; i++) {
          double ap = A[IDX(i, p, n)], aq = A[IDX(i, q, n)];
          A[IDX(i, p, n)] = c * ap - s * aq;
          A[IDX(i, q, n)] = s * ap + c * aq;
        }
      }
    if (off < 1e-15) break;
  }
  (void)V;
  double smax = 0.0, smin = INFINITY;
  for (int j = 0; j < n; j++) {
    double s = 0;
    for (int i = 0; i < n; i++) s += A[IDX(i, j, n)] * A[IDX(i, j, n)];
    s = sqrt(s);
    if (s > smax) smax = s;
    if (s < smin) smin = s;
  }
  if (isnan(smax) || isnan(smin)) return NAN;
  return smax / smin;
}

OC_EXPORT double oc_cond2(const double* A, int n) { return cond2(A, n); }
/* the deterministic sin/cos shared with the GPU (include/tog_math.h), for tests */
OC_EXPORT double oc_sin(double x) { return tog_sin(x); }
OC_EXPORT double oc_cos(double x) { return tog_cos(x); }
OC_EXPORT double oc_rsqrt(double x) { return tog_rsqrt(x); }
OC_EXPORT void oc_qr_R(double* R, double* P, int rows, int cols) { qr_R(R, P, rows, cols); }

/* chol_minus(A, B) (backward_pass.jl:186-192): Cholesky(copy(A), :U, 0) then
   lowrankdowndate!(C, B[i,:]) per row (Julia 1.1 LinearAlgebra cholesky.jl). Returns 0 or
   PosDefException index. */
static int chol_minus(double* Uo, const double* A, int n, const double* B, int nb) {
  double U[OM * OM], v[OM], rd[OM];
  memcpy(U, A, sizeof(double) * n * n);
#ifdef TOG_ORACLE_LITERAL
  /* literal: lowrankdowndate! (Julia 1.1 LinearAlgebra cholesky.jl) as written: s = v_i / A_ii,
     c = sqrt(1 - s^2), A_ii = c A_ii, tmp = (A_ij - s v_j) / c, v_j = c v_j - s tmp */
  (void)rd;
  for (int r = 0; r < nb; r++) {
    for (int j = 0; j < n; j++) v[j] = B[IDX(r, j, nb)];
    for (int i = 0; i < n; i++) {
      const double s = v[i] / U[IDX(i, i, n)];
      const double s2 = s * s;
      if (s2 > 1.0) return i + 1;
      const double c = sqrt(1.0 - s2);
      U[IDX(i, i, n)] = c * U[IDX(i, i, n)];
      for (int j = i + 1; j < n; j++) {
        const double tmp = (U[IDX(i, j, n)] - s * v[j]) / c;
        v[j] = c * v[j] - s * tmp;
        U[IDX(i, j, n)] = tmp;
      }
    }
  }
  memcpy(Uo, U, sizeof(double) * n * n);
  return 0;
#endif
  /* contract v4: the reciprocals of the diagonal are formed once and carried through the downdates
     (1/(c A_ii) = (1/A_ii)(1/c)); 1/c = tog_rsqrt(1 - s^2) and c = (1 - s^2)(1/c) replace the
     reference's sqrt and division by c (include/tog_math.h) */
  for (int i = 0; i < n; i++) rd[i] = 1.0 / U[IDX(i, i, n)];
  for (int r = 0; r < nb; r++) {
    for (int j = 0; j < n; j++) v[j] = B[IDX(r, j, nb)];
    for (int i = 0; i < n; i++) {
      double Aii = U[IDX(i, i, n)];
      double s = v[i] * rd[i];
      double s2 = s * s;
      if (s2 > 1.0) return i + 1;
      double y = 1.0 - s2;
      double rc = tog_rsqrt(y);
      double c = tog_rs_c(y, rc);
      U[IDX(i, i, n)] = c * Aii;
      rd[i] = rd[i] * rc;
      for (int j = i + 1; j < n; j++) {
        double tmp = (U[IDX(i, j, n)] - s * v[j]) * rc;
        v[j] = c * v[j] - s * tmp;
        U[IDX(i, j, n)] = tmp;
      }
    }
  }
  memcpy(Uo, U, sizeof(double) * n * n);
  return 0;
}
OC_EXPORT int oc_chol_minus(double* Uo, const double* A, int n, const double* B, int nb) {
  return chol_minus(Uo, A, n, B, nb);
}

/* =====================================================================
 * Problem (single trajectory view of tog_problem_desc)
 * ===================================================================== */
typedef struct {
  int type;     /* tog_constraint_type */
  int inequality;
  int p_stage, p_term;
  /* bound */
  double x_max[16], x_min[16], u_max[OM], u_min[OM];
  int ax_max[16], ax_min[16], au_max[OM], au_min[OM];
  /* goal */
  double xf[16];
  /* obstacles */
  int count;
  double obs[64 * 4];
  /* infeasible_constraints: the slack controls u[s0 : s0 + ns] */
  int s0, ns;
} oc_con;

typedef struct {
  int ncon;
  oc_con con[8];
  int p_stage, p_term;
} oc_cset;

typedef struct oc_solver {
  int model, integ, n, m, N;
  int slack, mb; /* infeasible problem: slack = n slack controls after the mb model controls */
  int mt;        /* minimum-time problem (add_min_time_controls): x = [x_b; τ], u = [u_b; h], dt_k = h_k² */
  double R_mt;   /* MinTimeCost R_min_time */
  double dt;
  double *Q, *R, *H, *q, *r, c, *Qf, *qf, cf;
  int nsets;
  oc_cset* sets;
  int* knot_set;
  int* p;   /* p[k] constraints at knot k */
  int pmax;
  tog_options opts;
  /* iLQR solver buffers (ilqr_solver.jl:93-144) */
  double *x0, *X, *U, *Xb, *Ub, *K, *d, *F; /* F: n x (n+m+1) per knot */
  double *Sxx, *Sx;                         /* S[k].xx, S[k].x */
  double *Qx, *Qu, *Qxx, *Quu, *Qux;        /* Q expansion per knot */
  double rho, drho;
  double dV[2];
  /* AL (augmented_lagrangian_solver.jl:111-118) */
  double *C, *lam, *mu;
  int* active;
  int* ineq; /* ineq[k*pmax+i] 1 if inequality */
  /* stats */
  int iterations, zero_count, bp_restarts, ls_trials, al_iter, total_steps, flags;
  double J, dJ, gradient, alpha, z, c_max, expected;
  /* per-iteration trace (for localisation) */
  int trace_len;
  double* trace; /* [J, alpha, rho, restarts, trials, z] per step */
  int al_mode;   /* the current inner solve's objective is the AL one (compute_gradient's prob.obj) */
  /* the solver.stats vectors: iLQR record_iteration! (ilqr_methods.jl:77-89) [cost, dJ, gradient] per inner
     record, AL record_iteration! (augmented_lagrangian_methods.jl:79-97) [iterations_inner, cost, c_max,
     penalty_max] per outer record (tog.h TOG_FIELD_HIST_*) */
  double* hin;
  int hin_n, hin_cap;
  double* hout;
  int hout_n, hout_cap;
  double* hpn; /* projected Newton record_iteration! (projected_newton.jl:23-29): [cost, c_max] per step */
  int hpn_n, hpn_cap;
  /* a time-varying Objective (src/objective.jl:15-29): per stage knot [Q; R; H; q; r; c] (tog.h
     stage_costs), or NULL (the stage cost Q, R, H, q, r, c at every stage knot) */
  double* kc;
  int kc_stride;
} oc_solver;

/* stage knot k's QuadraticCost (src/cost.jl:112-157): the shared one, or row k of the per-knot table */
static inline const double* kQ(const oc_solver* s, int k) { return s->kc ? s->kc + (size_t)k * s->kc_stride : s->Q; }
static inline const double* kR(const oc_solver* s, int k) {
  return s->kc ? s->kc + (size_t)k * s->kc_stride + s->n * s->n : s->R;
}
static inline const double* kH(const oc_solver* s, int k) {
  return s->kc ? s->kc + (size_t)k * s->kc_stride + s->n * s->n + s->m * s->m : s->H;
}
static inline const double* kq(const oc_solver* s, int k) {
  return s->kc ? s->kc + (size_t)k * s->kc_stride + s->n * s->n + s->m * s->m + s->m * s->n : s->q;
}
static inline const double* kr(const oc_solver* s, int k) {
  return s->kc ? s->kc + (size_t)k * s->kc_stride + s->n * s->n + s->m * s->m + s->m * s->n + s->n : s->r;
}
static inline double kc0(const oc_solver* s, int k) {
  return s->kc ? s->kc[(size_t)k * s->kc_stride + s->n * s->n + s->m * s->m + s->m * s->n + s->n + s->m] : s->c;
}

static void hist_push(double** buf, int* n, int* cap, int w, const double* rec) {
  if (*n == *cap) {
    *cap = *cap ? 2 * *cap : 256;
    *buf = realloc(*buf, sizeof(double) * w * (size_t)*cap);
  }
  memcpy(*buf + (size_t)w * *n, rec, sizeof(double) * w);
  (*n)++;
}

/* mb: the controls a bound row may constrain (m less the slack controls of an infeasible-start problem:
   its BoundConstraint keeps the model's m, update_constraint_set_jacobians constraint_sets.jl:135-150) */
/* mb: the controls of the model inside add_slack_controls / add_min_time_controls; slack: the slack count.
   A trim=false bound keeps one row per model control and one for the time step h (the slack controls get none;
   BoundConstraint(n̄, m̄, trim=false) keeps every u row of the problem it was built for); a trimmed
   bound has rows for its finite entries over all m (an infeasible problem's slack entries are infinite;
   the infeasible minimum-time problem's combined bound reaches u[1:m+1], minimum_time.jl:125-141) */
static void con_init(oc_con* oc, const tog_constraint* tc, int n, int m, int mb, int slack) {
  memset(oc, 0, sizeof(*oc));
  oc->type = tc->type;
  switch (tc->type) {
    case TOG_CON_BOUND: {
      /* src/constraints.jl:155-188: trim=true (count 0): active = isfinite.(bound); trim=false (count 1):
         every row active (an infinite bound then gives c = -Inf, and the AL terms NaN, as in the reference) */
      const double* D = tc->data;
      const int keep = (tc->count == 1);
      int cx = 0, cu = 0, cxn = 0, cun = 0;
      for (int i = 0; i < n; i++) {
        oc->x_max[i] = D[i];
        oc->x_min[i] = D[n + i];
        oc->ax_max[i] = keep || isfinite(D[i]);
        oc->ax_min[i] = keep || isfinite(D[n + i]);
        cx += oc->ax_max[i];
        cxn += oc->ax_min[i];
      }
      for (int i = 0; i < m; i++) {
        oc->u_max[i] = D[2 * n + i];
        oc->u_min[i] = D[2 * n + m + i];
        /* trim=false keeps the model's controls and the time step h (the last control when m - mb - slack = 1) */
        const int ku = i < mb || (i == m - 1 && m - mb - slack > 0);
        oc->au_max[i] = (keep ? ku : 1) && (keep || isfinite(D[2 * n + i]));
        oc->au_min[i] = (keep ? ku : 1) && (keep || isfinite(D[2 * n + m + i]));
        cu += oc->au_max[i];
        cun += oc->au_min[i];
      }
      oc->inequality = 1;
      oc->p_stage = cx + cu + cxn + cun;
      oc->p_term = cx + cxn; /* length(bnd, :terminal) constraints.jl:244-252 */
      break;
    }
    case TOG_CON_GOAL: { /* count: rows x[1:count] - xf (inds, constraints.jl:303); 0 = n */
      const int ng = tc->count > 0 ? tc->count : n;
      for (int i = 0; i < ng; i++) oc->xf[i] = tc->data[i];
      oc->inequality = 0;
      oc->p_stage = 0; /* terminal-only (term=:terminal) */
      oc->p_term = ng;
      break;
    }
    case TOG_CON_CIRCLES:
      oc->count = tc->count;
      memcpy(oc->obs, tc->data, sizeof(double) * 3 * tc->count);
      oc->inequality = 1;
      oc->p_stage = tc->count;
      oc->p_term = 0; /* stage-only: c(v,x,u) method only */
      break;
    case TOG_CON_SPHERES:
      oc->count = tc->count;
      memcpy(oc->obs, tc->data, sizeof(double) * 4 * tc->count);
      oc->inequality = 1;
      oc->p_stage = tc->count;
      oc->p_term = 0;
      break;
    case TOG_CON_INFEASIBLE: /* infeasible_constraints(n, m) src/constraints.jl:306-314 */
      oc->inequality = 0;
      oc->s0 = mb;
      oc->ns = slack;
      oc->p_stage = slack;
      oc->p_term = 0; /* :stage only */
      break;
    case TOG_CON_MIN_TIME_EQ: /* mintime_equality(n, m) minimum_time.jl:106-124, :stage */
      oc->inequality = 0;
      oc->p_stage = 1;
      oc->p_term = 0;
      break;
  }
}

/* evaluate constraint `oc` into v (stage: x,u; terminal: u == NULL), and its Jacobian rows
   into Jx (p x n, ld = ldj) and Ju (p x m) if non-NULL. src/constraints.jl:212-237,299-304,
   src/utils.jl:140-156 (ForwardDiff of the generic primitives = the analytic derivative). */
static int con_eval(const oc_con* oc, int n, int m, const double* x, const double* u, double* v,
                    double* Jx, double* Ju, int ldj) {
  int term = (u == NULL);
  int r = 0;
  switch (oc->type) {
    case TOG_CON_BOUND:
      if (!term) {
        for (int i = 0; i < n; i++)
          if (oc->ax_max[i]) {
            v[r] = x[i] - oc->x_max[i];
            if (Jx) Jx[r + ldj * i] = 1.0;
            r++;
          }
        for (int i = 0; i < m; i++)
          if (oc->au_max[i]) {
            v[r] = u[i] - oc->u_max[i];
            if (Ju) Ju[r + ldj * i] = 1.0;
            r++;
          }
        for (int i = 0; i < n; i++)
          if (oc->ax_min[i]) {
            v[r] = oc->x_min[i] - x[i];
            if (Jx) Jx[r + ldj * i] = -1.0;
            r++;
          }
        for (int i = 0; i < m; i++)
          if (oc->au_min[i]) {
            v[r] = oc->u_min[i] - u[i];
            if (Ju) Ju[r + ldj * i] = -1.0;
            r++;
          }
      } else {
        for (int i = 0; i < n; i++)
          if (oc->ax_max[i]) {
            v[r] = x[i] - oc->x_max[i];
            if (Jx) Jx[r + ldj * i] = 1.0;
            r++;
          }
        for (int i = 0; i < n; i++)
          if (oc->ax_min[i]) {
            v[r] = oc->x_min[i] - x[i];
            if (Jx) Jx[r + ldj * i] = -1.0;
            r++;
          }
      }
      break;
    case TOG_CON_GOAL:
      if (term) {
        for (int i = 0; i < oc->p_term; i++) {
          v[r] = x[i] - oc->xf[i];
          if (Jx) Jx[r + ldj * i] = 1.0;
          r++;
        }
      }
      break;
    case TOG_CON_CIRCLES:
      if (!term) {
        for (int o = 0; o < oc->count; o++) {
          double x0 = oc->obs[3 * o], y0 = oc->obs[3 * o + 1], rr = oc->obs[3 * o + 2];
          double dx = x[0] - x0, dy = x[1] - y0;
          v[r] = -((dx * dx + dy * dy) - rr * rr);
          if (Jx) {
            Jx[r + ldj * 0] = -(2.0 * dx);
            Jx[r + ldj * 1] = -(2.0 * dy);
          }
          r++;
        }
      }
      break;
    case TOG_CON_INFEASIBLE:
      /* inf_con(v, x, u) = copyto!(v, u[m+1:m+n]); ∇inf = [0 0 I] (src/constraints.jl:306-314) */
      if (!term) {
        for (int i = 0; i < oc->ns; i++) {
          v[r] = u[oc->s0 + i];
          if (Ju) Ju[r + ldj * (oc->s0 + i)] = 1.0;
          r++;
        }
      }
      break;
    case TOG_CON_MIN_TIME_EQ: /* con_eq(v, x, u): v[1] = u[end] - x[end]; ∇ = [0 .. -1 | 0 .. 1] */
      if (!term) {
        v[r] = u[m - 1] - x[n - 1];
        if (Jx) Jx[r + ldj * (n - 1)] = -1.0;
        if (Ju) Ju[r + ldj * (m - 1)] = 1.0;
        r++;
      }
      break;
    case TOG_CON_SPHERES:
      if (!term) {
        for (int o = 0; o < oc->count; o++) {
          double x0 = oc->obs[4 * o], y0 = oc->obs[4 * o + 1], z0 = oc->obs[4 * o + 2], rr = oc->obs[4 * o + 3];
          double dx = x[0] - x0, dy = x[1] - y0, dz = x[2] - z0;
          v[r] = -(((dx * dx + dy * dy) + dz * dz) - rr * rr);
          if (Jx) {
            Jx[r + ldj * 0] = -(2.0 * dx);
            Jx[r + ldj * 1] = -(2.0 * dy);
            Jx[r + ldj * 2] = -(2.0 * dz);
          }
          r++;
        }
      }
      break;
  }
  return r;
}

/* evaluate!(c, C::ConstraintSet, x[, u]) (constraint_sets.jl:106-118) + jacobian
   (constraint_sets.jl:121-131). Jx: p x n (ld p), Ju: p x m. Returns p. */
static int set_eval(const oc_solver* s, int k, const double* x, const double* u, double* c, double* Jx, double* Ju,
                    int* ineq) {
  int si = s->knot_set[k];
  if (si < 0) return 0;
  const oc_cset* set = &s->sets[si];
  int term = (k == s->N - 1);
  int p = term ? set->p_term : set->p_stage;
  if (Jx) memset(Jx, 0, sizeof(double) * p * s->n);
  if (Ju) memset(Ju, 0, sizeof(double) * p * s->m);
  int r = 0;
  for (int i = 0; i < set->ncon; i++) {
    const oc_con* oc = &set->con[i];
    int pr = term ? oc->p_term : oc->p_stage;
    if (pr == 0) continue;
    con_eval(oc, s->n, s->m, x, term ? NULL : u, c + r, Jx ? Jx + r : NULL, Ju ? Ju + r : NULL, p);
    if (ineq)
      for (int j = 0; j < pr; j++) ineq[r + j] = oc->inequality;
    r += pr;
  }
  return p;
}

static void desc_load(oc_solver* s, const tog_problem_desc* d) {
  s->model = d->model;
  s->integ = d->integrator;
  s->n = d->n;
  s->m = d->m;
  s->N = d->N;
  s->dt = d->dt;
  /* add_min_time_controls(add_slack_controls(model)) (altro_methods.jl:98-124): x = [x; τ], u = [u; s; h] */
  s->mt = (d->flags & TOG_PROB_MIN_TIME) ? 1 : 0;
  s->slack = (d->flags & TOG_PROB_INFEASIBLE) ? d->n - s->mt : 0;
  s->mb = d->m - s->slack - s->mt;
  s->R_mt = s->mt ? d->R_min_time : 0.0;
  int n = s->n, m = s->m, N = s->N;
  s->Q = malloc(sizeof(double) * n * n);
  memcpy(s->Q, d->Q, sizeof(double) * n * n);
  s->R = malloc(sizeof(double) * m * m);
  memcpy(s->R, d->R, sizeof(double) * m * m);
  s->H = malloc(sizeof(double) * m * n);
  memcpy(s->H, d->H, sizeof(double) * m * n);
  s->q = malloc(sizeof(double) * n);
  memcpy(s->q, d->q, sizeof(double) * n);
  s->r = malloc(sizeof(double) * m);
  memcpy(s->r, d->r, sizeof(double) * m);
  s->c = d->c;
  s->kc_stride = n * n + m * m + m * n + n + m + 1;
  s->kc = NULL;
  if (d->stage_costs) {
    s->kc = malloc(sizeof(double) * (size_t)s->kc_stride * (d->N - 1));
    memcpy(s->kc, d->stage_costs, sizeof(double) * (size_t)s->kc_stride * (d->N - 1));
  }
  s->Qf = malloc(sizeof(double) * n * n);
  memcpy(s->Qf, d->Qf, sizeof(double) * n * n);
  s->qf = malloc(sizeof(double) * n);
  memcpy(s->qf, d->qf, sizeof(double) * n);
  s->cf = d->cf;
  s->nsets = d->n_sets;
  s->sets = calloc(d->n_sets > 0 ? d->n_sets : 1, sizeof(oc_cset));
  for (int i = 0; i < d->n_sets; i++) {
    oc_cset* os = &s->sets[i];
    os->ncon = d->sets[i].n_con;
    for (int j = 0; j < os->ncon; j++) {
      con_init(&os->con[j], &d->sets[i].con[j], n, m, s->mb, s->slack);
      os->p_stage += os->con[j].p_stage;
      os->p_term += os->con[j].p_term;
    }
  }
  s->knot_set = malloc(sizeof(int) * N);
  s->p = malloc(sizeof(int) * N);
  s->pmax = 0;
  for (int k = 0; k < N; k++) {
    s->knot_set[k] = d->knot_set ? d->knot_set[k] : -1;
    int si = s->knot_set[k];
    s->p[k] = si < 0 ? 0 : (k == N - 1 ? s->sets[si].p_term : s->sets[si].p_stage);
    if (s->p[k] > s->pmax) s->pmax = s->p[k];
  }
}

#define Xk(s, k) ((s)->X + (size_t)(k) * (s)->n)
#define Uk(s, k) ((s)->U + (size_t)(k) * (s)->m)

OC_EXPORT oc_solver* oc_create(const tog_problem_desc* d, const tog_options* o) {
  oc_solver* s = calloc(1, sizeof(oc_solver));
  desc_load(s, d);
  s->opts = *o;
  int n = s->n, m = s->m, N = s->N, P = s->pmax > 0 ? s->pmax : 1;
  s->x0 = calloc(n, sizeof(double));
  s->X = calloc((size_t)n * N, sizeof(double));
  s->U = calloc((size_t)m * (N - 1), sizeof(double));
  s->Xb = calloc((size_t)n * N, sizeof(double));
  s->Ub = calloc((size_t)m * (N - 1), sizeof(double));
  s->K = calloc((size_t)m * n * (N - 1), sizeof(double));
  s->d = calloc((size_t)m * (N - 1), sizeof(double));
  s->F = calloc((size_t)n * (n + m + 1) * (N - 1), sizeof(double));
  s->Sxx = calloc((size_t)n * n * N, sizeof(double));
  s->Sx = calloc((size_t)n * N, sizeof(double));
  s->Qx = calloc((size_t)n * N, sizeof(double));
  s->Qu = calloc((size_t)m * N, sizeof(double));
  s->Qxx = calloc((size_t)n * n * N, sizeof(double));
  s->Quu = calloc((size_t)m * m * N, sizeof(double));
  s->Qux = calloc((size_t)m * n * N, sizeof(double));
  s->C = calloc((size_t)P * N, sizeof(double));
  s->lam = calloc((size_t)P * N, sizeof(double));
  s->mu = calloc((size_t)P * N, sizeof(double));
  s->active = calloc((size_t)P * N, sizeof(int));
  for (int i = 0; i < P * N; i++) s->mu[i] = o->penalty_initial; /* init_constraint_trajectories μ_init */
  s->ineq = calloc((size_t)P * N, sizeof(int));
  for (int k = 0; k < N; k++) {
    double cbuf[256];
    double xz[16] = {0}, uz[OM] = {0};
    set_eval(s, k, xz, k < N - 1 ? uz : NULL, cbuf, NULL, NULL, s->ineq + (size_t)k * P);
  }
  s->trace = calloc(6 * 4096, sizeof(double));
  return s;
}

OC_EXPORT void oc_destroy(oc_solver* s) {
  if (!s) return;
  free(s->Q); free(s->R); free(s->H); free(s->q); free(s->r); free(s->Qf); free(s->qf);
  free(s->sets); free(s->knot_set); free(s->p);
  free(s->x0); free(s->X); free(s->U); free(s->Xb); free(s->Ub); free(s->K); free(s->d); free(s->F);
  free(s->Sxx); free(s->Sx); free(s->Qx); free(s->Qu); free(s->Qxx); free(s->Quu); free(s->Qux);
  free(s->C); free(s->lam); free(s->mu); free(s->active); free(s->ineq); free(s->trace);
  free(s->hin); free(s->hout); free(s->hpn); free(s->kc);
  free(s);
}

OC_EXPORT int oc_pmax(oc_solver* s) { return s->pmax; }

/* initial_controls!, set_x0!, X0 = NaN (src/problem.jl:149-160,232) */
OC_EXPORT void oc_set_state(oc_solver* s, const double* x0, const double* U, const double* X) {
  memcpy(s->x0, x0, sizeof(double) * s->n);
  memcpy(s->U, U, sizeof(double) * s->m * (s->N - 1));
  if (X)
    memcpy(s->X, X, sizeof(double) * s->n * s->N);
  else
    for (int i = 0; i < s->n * s->N; i++) s->X[i] = NAN;
}

/* =====================================================================
 * Cost (src/cost.jl:171-181, src/objective.jl:40-48)
 * ===================================================================== */
static double stage_cost(const oc_solver* s, int k, const double* x, const double* u, double dt) {
  int n = s->n, m = s->m;
  const double *Q = kQ(s, k), *R = kR(s, k), *H = kH(s, k), *q = kq(s, k), *r = kr(s, k);
  /* 0.5*x'Q*x + 0.5*u'*R*u + q'x + r'u + c + u'*H*x, then *dt */
  double xQx = 0, uRu = 0, qx = 0, ru = 0, uHx = 0;
  for (int j = 0; j < n; j++) {
    double t = 0;
    for (int i = 0; i < n; i++) t = fma(0.5 * x[i], Q[IDX(i, j, n)], t);
    xQx = fma(t, x[j], xQx);
  }
  for (int j = 0; j < m; j++) {
    double t = 0;
    for (int i = 0; i < m; i++) t = fma(0.5 * u[i], R[IDX(i, j, m)], t);
    uRu = fma(t, u[j], uRu);
  }
  for (int i = 0; i < n; i++) qx = fma(q[i], x[i], qx);
  for (int i = 0; i < m; i++) ru = fma(r[i], u[i], ru);
  for (int j = 0; j < n; j++) {
    double t = 0;
    for (int i = 0; i < m; i++) t = fma(u[i], H[IDX(i, j, m)], t);
    uHx = fma(t, x[j], uHx);
  }
  return ((((xQx + uRu) + qx) + ru) + kc0(s, k) + uHx) * dt;
}
static double terminal_cost(const oc_solver* s, const double* x) {
  int n = s->n;
  double xQx = 0, qx = 0;
  for (int j = 0; j < n; j++) {
    double t = 0;
    for (int i = 0; i < n; i++) t = fma(0.5 * x[i], s->Qf[IDX(i, j, n)], t);
    xQx = fma(t, x[j], xQx);
  }
  for (int i = 0; i < n; i++) qx = fma(s->qf[i], x[i], qx);
  return (xQx + qx) + s->cf;
}

static double obj_cost(const oc_solver* s, const double* X, const double* U) {
  int n = s->n, m = s->m, N = s->N;
  double J = 0.0;
  for (int k = 0; k < N - 1; k++) {
    const double* u = U + (size_t)k * m;
    if (s->mt) { /* MinTimeCost (minimum_time.jl:148): stage_cost(cost, x, u, h) + R_min_time u[end]^2, h = get_dt */
      const double h = u[m - 1];
      J += stage_cost(s, k, X + (size_t)k * n, u, h * h) + s->R_mt * (h * h);
    } else {
      J += stage_cost(s, k, X + (size_t)k * n, u, s->dt);
    }
  }
  J += terminal_cost(s, X + (size_t)(N - 1) * n);
  return J;
}

/* update_constraints! + update_active_set! (constraint_sets.jl:221-260) */
static void update_constraints(oc_solver* s, const double* X, const double* U) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  for (int k = 0; k < N; k++) {
    if (s->p[k] == 0) continue;
    set_eval(s, k, X + (size_t)k * n, k < N - 1 ? U + (size_t)k * m : NULL, s->C + (size_t)k * P, NULL, NULL, NULL);
  }
}
static void update_active_set(oc_solver* s) {
  int N = s->N, P = s->pmax;
  for (int k = 0; k < N; k++)
    for (int i = 0; i < s->p[k]; i++) {
      size_t j = (size_t)k * P + i;
      s->active[j] = s->ineq[j] ? ((s->C[j] >= 0.0) || (s->lam[j] > 0.0)) : 1;
    }
}

/* AL cost (augmented_lagrangian_methods.jl:298-313): mutates C and the active set (A.10) */
static double al_cost(oc_solver* s, const double* X, const double* U) {
  int N = s->N, P = s->pmax;
  double J = obj_cost(s, X, U);
  update_constraints(s, X, U);
  update_active_set(s);
  double Jc = 0.0;
  for (int k = 0; k < N; k++) {
    /* aula_cost: λ'c + 1/2*c'Diagonal(a .* μ)*c */
    double lc = 0.0, cIc = 0.0;
    for (int i = 0; i < s->p[k]; i++) {
      size_t j = (size_t)k * P + i;
      lc = fma(s->lam[j], s->C[j], lc);
    }
    for (int i = 0; i < s->p[k]; i++) {
      size_t j = (size_t)k * P + i;
      double w = s->active[j] ? s->mu[j] : 0.0;
      cIc = fma(s->C[j] * w, s->C[j], cIc);
    }
    Jc += lc + 0.5 * cIc;
  }
  return J + Jc;
}

static double cost(oc_solver* s, int al, const double* X, const double* U) {
  return al ? al_cost(s, X, U) : obj_cost(s, X, U);
}

OC_EXPORT double oc_cost(oc_solver* s, int al) { return cost(s, al, s->X, s->U); }
OC_EXPORT double oc_cost_bar(oc_solver* s, int al) { return cost(s, al, s->Xb, s->Ub); }

/* =====================================================================
 * Rollouts (src/rollout.jl)
 * ===================================================================== */
/* evaluate!(x+, model, x, u, dt) of the solver's model. For an infeasible problem this is
   add_slack_controls (src/model.jl:761-779): f!(x+, x, u[1:m], dt) then x+ .+= u[m+1:m+n]. */
static void traj_f(const oc_solver* s, double* xn, const double* x, const double* u) {
  if (s->mt) { /* add_min_time_controls f!: h = u[end]; model.f(x+, x, u, h^2); x+[n̄] = h (minimum_time.jl:91-95) */
    const double h = u[s->m - 1];
    oc_discrete_f(s->model, s->integ, xn, x, u, h * h);
    for (int i = 0; i < s->slack; i++) xn[i] += u[s->mb + i]; /* an infeasible model inside: x+ .+= s */
    xn[s->n - 1] = h;
    return;
  }
  oc_discrete_f(s->model, s->integ, xn, x, u, s->dt);
  for (int i = 0; i < s->slack; i++) xn[i] += u[s->mb + i];
}

/* ∇f!(Z, x, u, dt) of the solver's model into F (n x (n+m+1)): the model's jacobian in
   columns [x; u[1:m]] and dt, and Diagonal(1.0I, n) in the slack columns (src/model.jl:771-774). */
static void traj_jacobian(const oc_solver* s, double* F, const double* x, const double* u) {
  int n = s->n, mb = s->mb, m = s->m;
  if (s->mt) {
    /* ∇f! of add_min_time_controls (minimum_time.jl:97-101): model.∇f(view(Z, idx.x, idx2), x, u, h^2) with
       idx2 = [x columns; u columns + n̄; last], Z[idx.x, end] .*= 2h, Z[n̄, end] = 1 */
    const int nb = n - 1, mbb = mb;
    const double h = u[m - 1];
    double Z[16 * (16 + OM + 1)];
    discrete_jacobian_fd(s->model, s->integ, Z, x, u, h * h); /* nb x (nb + mbb + 1) */
    memset(F, 0, sizeof(double) * n * (n + m + 1));
    for (int j = 0; j < nb; j++)
      for (int i = 0; i < nb; i++) F[i + n * j] = Z[i + nb * j];
    for (int j = 0; j < mbb; j++)
      for (int i = 0; i < nb; i++) F[i + n * (n + j)] = Z[i + nb * (nb + j)];
    /* an infeasible model inside: its ∇f! writes Diagonal(1.0I, n) in the slack columns (src/model.jl:771-774) */
    for (int j = 0; j < s->slack; j++) F[j + n * (n + mbb + j)] = 1.0;
    for (int i = 0; i < nb; i++) F[i + n * (n + m - 1)] = Z[i + nb * (nb + mbb)] * (2.0 * h);
    F[nb + n * (n + m - 1)] = 1.0;
    return;
  }
  if (!s->slack) {
    oc_discrete_jacobian(s->model, s->integ, F, x, u, s->dt);
    return;
  }
  double Z[16 * (16 + OM + 1)];
  oc_discrete_jacobian(s->model, s->integ, Z, x, u, s->dt); /* n x (n+mb+1) */
  memcpy(F, Z, sizeof(double) * n * (n + mb));
  for (int j = 0; j < n; j++)
    for (int i = 0; i < n; i++) F[i + n * (n + mb + j)] = (i == j) ? 1.0 : 0.0;
  memcpy(F + (size_t)n * (n + m), Z + (size_t)n * (n + mb), sizeof(double) * n);
}

/* slack_controls(prob) (src/solvers/altro/infeasible.jl:63-80), run on the original model
   with x[k+1] = f(x[k], U[k]); s_k = X[k+1] - x[k+1]; x[k+1] += s_k. Writes U[m+1:m+n]. */
OC_EXPORT void oc_slack_controls(oc_solver* s) {
  int n = s->n, m = s->m, N = s->N;
  if (!s->slack || s->mt) return; /* (the infeasible minimum-time problem takes its slacks from infeasible_problem) */
  double x[16], xn[16];
  memcpy(x, s->x0, sizeof(double) * n);
  for (int k = 0; k < N - 1; k++) {
    double* u = s->U + (size_t)k * m;
    oc_discrete_f(s->model, s->integ, xn, x, u, s->dt);
    const double* Xn = s->X + (size_t)(k + 1) * n;
    for (int i = 0; i < n; i++) {
      u[s->mb + i] = Xn[i] - xn[i];
      x[i] = xn[i] + u[s->mb + i];
    }
  }
}

/* rollout!(prob) src/rollout.jl:25-38: open loop only if any X non-finite */
OC_EXPORT void oc_rollout_open_loop(oc_solver* s) {
  int n = s->n, m = s->m, N = s->N;
  int finite = 1;
  for (int i = 0; i < n * N; i++)
    if (!isfinite(s->X[i])) finite = 0;
  if (finite) return;
  memcpy(s->X, s->x0, sizeof(double) * n);
  for (int k = 0; k < N - 1; k++)
    traj_f(s, s->X + (size_t)(k + 1) * n, s->X + (size_t)k * n, s->U + (size_t)k * m);
}

/* rollout!(prob, solver, alpha) src/rollout.jl:2-23 */
OC_EXPORT int oc_rollout(oc_solver* s, double alpha) {
  int n = s->n, m = s->m, N = s->N;
  memcpy(s->Xb, s->x0, sizeof(double) * n);
  for (int k = 1; k < N; k++) {
    const double* xb = s->Xb + (size_t)(k - 1) * n;
    const double* x = s->X + (size_t)(k - 1) * n;
    double dx[16];
    for (int i = 0; i < n; i++) dx[i] = xb[i] - x[i]; /* state_diff */
    double* ub = s->Ub + (size_t)(k - 1) * m;
    const double* Kk = s->K + (size_t)(k - 1) * m * n;
    const double* dk = s->d + (size_t)(k - 1) * m;
    /* Ū = U + K*δx + alpha*d */
    for (int i = 0; i < m; i++) {
      double t = 0.0;
      for (int j = 0; j < n; j++) t = fma(Kk[IDX(i, j, m)], dx[j], t);
      ub[i] = (s->U[(size_t)(k - 1) * m + i] + t) + alpha * dk[i];
    }
    traj_f(s, s->Xb + (size_t)k * n, xb, ub);
    double nx = 0, nu = 0;
    int bad = 0;
    for (int i = 0; i < n; i++) {
      double a = fabs(s->Xb[(size_t)k * n + i]);
      if (!(a <= nx)) nx = a;
      if (isnan(a)) bad = 1;
    }
    for (int i = 0; i < m; i++) {
      double a = fabs(ub[i]);
      if (!(a <= nu)) nu = a;
      if (isnan(a)) bad = 1;
    }
    if (bad || !(nx < s->opts.max_state_value && nu < s->opts.max_control_value)) return 0;
  }
  return 1;
}

/* =====================================================================
 * Jacobians (src/solvers.jl:126 -> src/model.jl:301-306)
 * ===================================================================== */
OC_EXPORT void oc_jacobians(oc_solver* s) {
  int n = s->n, m = s->m, N = s->N, L = n + m + 1;
  for (int k = 0; k < N - 1; k++)
    traj_jacobian(s, s->F + (size_t)k * n * L, Xk(s, k), Uk(s, k));
}

/* =====================================================================
 * Cost expansion (ilqr_methods.jl:55-62 -> objective.jl:51-94, cost.jl:183-198,
 * AL: augmented_lagrangian_methods.jl:186-276)
 * ===================================================================== */
static void expansion_stage(oc_solver* s, int k) {
  int n = s->n, m = s->m;
  const double* x = Xk(s, k);
  const double* u = Uk(s, k);
  /* minimum time: τ = u[end], dt = τ^2 (MinTimeCost cost_expansion!, minimum_time.jl:155-188) */
  double dt = s->mt ? u[m - 1] * u[m - 1] : s->dt;
  double* Qx = s->Qx + (size_t)k * n;
  double* Qu = s->Qu + (size_t)k * m;
  double gx[16], gu[OM]; /* unscaled Qx, Qu (MinTimeCost's tmp and Q.ux rows) */
  const double *cQ = kQ(s, k), *cR = kR(s, k), *cH = kH(s, k), *cq = kq(s, k), *cr = kr(s, k);
  /* Q.x .= cost.Q*x + cost.q + cost.H'*u ; Q.u .= cost.R*u + cost.r + cost.H*x ; then Q*dt */
  for (int i = 0; i < n; i++) {
    double a = 0, b = 0;
    for (int j = 0; j < n; j++) a = fma(cQ[IDX(i, j, n)], x[j], a);
    for (int j = 0; j < m; j++) b = fma(cH[IDX(j, i, m)], u[j], b);
    gx[i] = (a + cq[i]) + b;
    Qx[i] = gx[i] * dt;
  }
  for (int i = 0; i < m; i++) {
    double a = 0, b = 0;
    for (int j = 0; j < m; j++) a = fma(cR[IDX(i, j, m)], u[j], a);
    for (int j = 0; j < n; j++) b = fma(cH[IDX(i, j, m)], x[j], b);
    gu[i] = (a + cr[i]) + b;
    Qu[i] = gu[i] * dt;
  }
  for (int i = 0; i < n * n; i++) s->Qxx[(size_t)k * n * n + i] = cQ[i] * dt;
  for (int i = 0; i < m * m; i++) s->Quu[(size_t)k * m * m + i] = cR[i] * dt;
  for (int i = 0; i < m * n; i++) s->Qux[(size_t)k * m * n + i] = cH[i] * dt;
  if (s->mt) {
    /* ℓ1 = stage_cost(cost.cost, x, u); tmp = 2τ Qu; Q.u[end] = τ(2ℓ1 + R); Q.uu[u, end] = tmp;
       Q.uu[end, end] = 2ℓ1 + R; Q.ux[end, x] = 2τ Qx'; Q.x[end] = R x[end]; Q.xx[end, end] = R */
    const double R = s->R_mt, tau = u[m - 1];
    const double l1 = stage_cost(s, k, x, u, 1.0);
    const double w = 2.0 * l1 + R, t2 = 2.0 * tau;
    double* Quu = s->Quu + (size_t)k * m * m;
    double* Qux = s->Qux + (size_t)k * m * n;
    for (int i = 0; i < m - 1; i++) {
      const double tmp = t2 * gu[i];
      Quu[IDX(i, m - 1, m)] = tmp;
      Quu[IDX(m - 1, i, m)] = tmp;
    }
    Qu[m - 1] = tau * w;
    Quu[IDX(m - 1, m - 1, m)] = w;
    for (int j = 0; j < n - 1; j++) Qux[IDX(m - 1, j, m)] = t2 * gx[j];
    Qx[n - 1] = R * x[n - 1];
    s->Qxx[(size_t)k * n * n + IDX(n - 1, n - 1, n)] = R;
  }
}
static void expansion_terminal(oc_solver* s) {
  int n = s->n, k = s->N - 1;
  const double* x = Xk(s, k);
  for (int i = 0; i < n * n; i++) s->Qxx[(size_t)k * n * n + i] = s->Qf[i];
  for (int i = 0; i < n; i++) {
    double a = 0;
    for (int j = 0; j < n; j++) a = fma(s->Qf[IDX(i, j, n)], x[j], a);
    s->Qx[(size_t)k * n + i] = a + s->qf[i];
  }
  if (s->mt) { /* MinTimeCost terminal: S.xx[end,end] = R_min_time, S.x[end] = R_min_time xN[end] */
    s->Qxx[(size_t)k * n * n + IDX(n - 1, n - 1, n)] = s->R_mt;
    s->Qx[(size_t)k * n + n - 1] = s->R_mt * x[n - 1];
  }
}

/* returns 0, or -1 on PosDefException in the sqrt expansion */
OC_EXPORT int oc_cost_expansion(oc_solver* s, int sq, int al) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  for (int k = 0; k < N - 1; k++) {
    expansion_stage(s, k);
    if (sq) { /* objective.jl:70-86 */
      double U[OM * OM];
      if (chol_upper(U, s->Qxx + (size_t)k * n * n, n)) return -1;
      memcpy(s->Qxx + (size_t)k * n * n, U, sizeof(double) * n * n);
      if (chol_upper(U, s->Quu + (size_t)k * m * m, m)) return -1;
      memcpy(s->Quu + (size_t)k * m * m, U, sizeof(double) * m * m);
    }
  }
  expansion_terminal(s);
  if (sq) {
    double U[OM * OM];
    if (chol_upper(U, s->Qxx + (size_t)(N - 1) * n * n, n)) return -1;
    memcpy(s->Qxx + (size_t)(N - 1) * n * n, U, sizeof(double) * n * n);
  }
  if (!al) return 0;
  /* AL terms */
  double cx[OP * 16], cu[OP * OM], cval[OP];
  for (int k = 0; k < N; k++) {
    int p = s->p[k];
    if (p == 0) continue;
    int term = (k == N - 1);
    set_eval(s, k, Xk(s, k), term ? NULL : Uk(s, k), cval, cx, term ? NULL : cu, NULL);
    const double* c = s->C + (size_t)k * P; /* obj.C[k] (last evaluated, A.10) */
    const double* lam = s->lam + (size_t)k * P;
    const double* mu = s->mu + (size_t)k * P;
    double w[OP], g[OP], ws[OP];
    for (int i = 0; i < p; i++) {
      /* a = active_set(c, λ) */
      int ineq = s->ineq[(size_t)k * P + i];
      int a = ineq ? ((c[i] >= 0.0) || (lam[i] > 0.0)) : 1;
      w[i] = a ? mu[i] : 0.0;
      ws[i] = a ? sqrt(mu[i]) : 0.0;
      g[i] = w[i] * c[i] + lam[i];
    }
    double* Qx = s->Qx + (size_t)k * n;
    double* Qxx = s->Qxx + (size_t)k * n * n;
    if (!sq) {
      /* Q.xx .+= cx'Iμ*cx ; Q.uu .+= cu'Iμ*cu ; Q.ux .+= cu'Iμ*cx */
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) {
          double t = 0;
          for (int r = 0; r < p; r++) t = fma(cx[r + p * i] * w[r], cx[r + p * j], t);
          Qxx[IDX(i, j, n)] += t;
        }
      if (!term) {
        double* Quu = s->Quu + (size_t)k * m * m;
        double* Qux = s->Qux + (size_t)k * m * n;
        for (int j = 0; j < m; j++)
          for (int i = 0; i < m; i++) {
            double t = 0;
            for (int r = 0; r < p; r++) t = fma(cu[r + p * i] * w[r], cu[r + p * j], t);
            Quu[IDX(i, j, m)] += t;
          }
        for (int j = 0; j < n; j++)
          for (int i = 0; i < m; i++) {
            double t = 0;
            for (int r = 0; r < p; r++) t = fma(cu[r + p * i] * w[r], cx[r + p * j], t);
            Qux[IDX(i, j, m)] += t;
          }
      }
    } else {
      /* chol_plus!(Q.xx, Iμ_sqrt*cx) ; chol_plus!(Q.uu, Iμ_sqrt*cu)  (no ux term, A.5) */
      double M[OP * OM], R[OM * OM];
      for (int j = 0; j < n; j++)
        for (int r = 0; r < p; r++) M[r + p * j] = ws[r] * cx[r + p * j];
      chol_plus(R, Qxx, n, M, p, n);
      memcpy(Qxx, R, sizeof(double) * n * n);
      if (!term) {
        double* Quu = s->Quu + (size_t)k * m * m;
        for (int j = 0; j < m; j++)
          for (int r = 0; r < p; r++) M[r + p * j] = ws[r] * cu[r + p * j];
        chol_plus(R, Quu, m, M, p, m);
        memcpy(Quu, R, sizeof(double) * m * m);
      }
    }
    /* Q.x .+= cx'g ; Q.u .+= cu'g */
    for (int i = 0; i < n; i++) {
      double t = 0;
      for (int r = 0; r < p; r++) t = fma(cx[r + p * i], g[r], t);
      Qx[i] += t;
    }
    if (!term) {
      double* Qu = s->Qu + (size_t)k * m;
      for (int i = 0; i < m; i++) {
        double t = 0;
        for (int r = 0; r < p; r++) t = fma(cu[r + p * i], g[r], t);
        Qu[i] += t;
      }
    }
  }
  return 0;
}

/* =====================================================================
 * Regularisation (ilqr_methods.jl:164-176)
 * ===================================================================== */
static void reg_update(oc_solver* s, int increase) {
  const tog_options* o = &s->opts;
  if (increase) {
    s->drho = fmax(s->drho * o->bp_reg_increase_factor, o->bp_reg_increase_factor);
    s->rho = fmax(s->rho * s->drho, o->bp_reg_min);
    if (s->rho > o->bp_reg_max) s->flags |= TOG_TRAJ_MAX_REG;
  } else {
    s->drho = fmin(s->drho / o->bp_reg_increase_factor, 1.0 / o->bp_reg_increase_factor);
    s->rho = s->rho * s->drho * (double)(s->rho * s->drho > o->bp_reg_min);
  }
}

/* =====================================================================
 * Backward passes (src/solvers/ilqr/backward_pass.jl)
 * ===================================================================== */
static void backward_std(oc_solver* s) {
  int n = s->n, m = s->m, N = s->N, L = n + m + 1;
  double* Sxx = s->Sxx;
  double* Sx = s->Sx;
  memcpy(Sxx + (size_t)(N - 1) * n * n, s->Qxx + (size_t)(N - 1) * n * n, sizeof(double) * n * n);
  memcpy(Sx + (size_t)(N - 1) * n, s->Qx + (size_t)(N - 1) * n, sizeof(double) * n);
  s->dV[0] = s->dV[1] = 0.0;
  s->bp_restarts = 0;
  double AtS[256], T[OM * OM], Quu_reg[OM * OM], Qux_reg[OM * 16], Kk[OM * 16], dk[OM], tmp[OM * OM];
  int k = N - 2;
  while (k >= 0) {
    const double* Fk = s->F + (size_t)k * n * L;
    const double* A = Fk;         /* fdx n x n */
    const double* B = Fk + n * n; /* fdu n x m */
    const double* S1 = Sxx + (size_t)(k + 1) * n * n;
    const double* s1 = Sx + (size_t)(k + 1) * n;
    double* Qx = s->Qx + (size_t)k * n;
    double* Qu = s->Qu + (size_t)k * m;
    double* Qxx = s->Qxx + (size_t)k * n * n;
    double* Quu = s->Quu + (size_t)k * m * m;
    double* Qux = s->Qux + (size_t)k * m * n;
    /* Q[k].x .+= fdx'*S[k+1].x ; Q[k].u .+= fdu'*S[k+1].x */
    matTmul(tmp, A, n, n, s1, 1);
    for (int i = 0; i < n; i++) Qx[i] += tmp[i];
    matTmul(tmp, B, n, m, s1, 1);
    for (int i = 0; i < m; i++) Qu[i] += tmp[i];
    /* Q[k].xx .+= fdx'*S*fdx  ((fdx'S)fdx, A.16) */
    matTmul(AtS, A, n, n, S1, n);
    matmul(T, AtS, n, n, A, n);
    for (int i = 0; i < n * n; i++) Qxx[i] += T[i];
    /* Q[k].uu .+= fdu'*S*fdu */
    double BtS[OM * 16];
    matTmul(BtS, B, n, m, S1, n);
    matmul(T, BtS, m, n, B, m);
    for (int i = 0; i < m * m; i++) Quu[i] += T[i];
    /* Q[k].ux .+= fdu'*S*fdx */
    matmul(T, BtS, m, n, A, n);
    for (int i = 0; i < m * n; i++) Qux[i] += T[i];

    if (s->opts.bp_reg_type == 1) { /* :state */
      double BtB[OM * OM], BtA[OM * 16];
      matTmul(BtB, B, n, m, B, m);
      matTmul(BtA, B, n, m, A, n);
      for (int i = 0; i < m * m; i++) Quu_reg[i] = Quu[i] + s->rho * BtB[i];
      for (int i = 0; i < m * n; i++) Qux_reg[i] = Qux[i] + s->rho * BtA[i];
    } else { /* :control */
      for (int i = 0; i < m * m; i++) Quu_reg[i] = Quu[i];
      for (int i = 0; i < m; i++) Quu_reg[i + m * i] += s->rho;
      memcpy(Qux_reg, Qux, sizeof(double) * m * n);
    }
    /* if !isposdef(Hermitian(Quu_reg)) -> increase ρ and restart at N-1 (A.1: Q not reset) */
    if (chol_upper(NULL, Quu_reg, m)) {
      reg_update(s, 1);
      s->bp_restarts++;
      k = N - 2;
      s->dV[0] = s->dV[1] = 0.0;
      if (s->bp_restarts > TOG_BP_MAX_RESTARTS) { /* restart cap: stop the trajectory (tog.h) */
        s->flags |= TOG_TRAJ_MAX_REG | TOG_TRAJ_BP_ABORTED;
        return; /* no :decrease, ΔV = 0 */
      }
      continue;
    }
    /* K = -(Quu_reg\Qux_reg) ; d = -(Quu_reg\Q.u) */
    memcpy(Kk, Qux_reg, sizeof(double) * m * n);
    lu_solve(Quu_reg, m, Kk, n);
    for (int i = 0; i < m * n; i++) Kk[i] = -1.0 * Kk[i];
    memcpy(dk, Qu, sizeof(double) * m);
    lu_solve(Quu_reg, m, dk, 1);
    for (int i = 0; i < m; i++) dk[i] = -1.0 * dk[i];
    memcpy(s->K + (size_t)k * m * n, Kk, sizeof(double) * m * n);
    memcpy(s->d + (size_t)k * m, dk, sizeof(double) * m);
    /* S[k].x = Q.x + K'*Q.uu*d + K'*Q.u + Q.ux'*d */
    double KtQuu[OM * 16];
    matTmul(KtQuu, Kk, m, n, Quu, m); /* n x m */
    double* Sk = Sxx + (size_t)k * n * n;
    double* sk = Sx + (size_t)k * n;
    {
      double a[16], b[16], c[16];
      matmul(a, KtQuu, n, m, dk, 1);
      matTmul(b, Kk, m, n, Qu, 1);
      matTmul(c, Qux, m, n, dk, 1);
      for (int i = 0; i < n; i++) sk[i] = ((Qx[i] + a[i]) + b[i]) + c[i];
    }
    /* S[k].xx = Q.xx + K'*Q.uu*K + K'*Q.ux + Q.ux'*K ; symmetrise */
    {
      double a[256], b[256], c[256];
      matmul(a, KtQuu, n, m, Kk, n);
      matTmul(b, Kk, m, n, Qux, n);
      matTmul(c, Qux, m, n, Kk, n);
      for (int i = 0; i < n * n; i++) Sk[i] = ((Qxx[i] + a[i]) + b[i]) + c[i];
      double tS[256];
      for (int j = 0; j < n; j++)
        for (int i = 0; i < n; i++) tS[IDX(i, j, n)] = 0.5 * (Sk[IDX(i, j, n)] + Sk[IDX(j, i, n)]);
      memcpy(Sk, tS, sizeof(double) * n * n);
    }
    /* ΔV[1] += d'*Q.u ; ΔV[2] += 0.5*d'*Q.uu*d */
    {
      double a = 0.0, b = 0.0;
      for (int i = 0; i < m; i++) a = fma(dk[i], Qu[i], a);
      for (int j = 0; j < m; j++) {
        double t = 0.0;
        for (int i = 0; i < m; i++) t = fma(0.5 * dk[i], Quu[IDX(i, j, m)], t);
        b = fma(t, dk[j], b);
      }
      s->dV[0] += a;
      s->dV[1] += b;
    }
    k--;
  }
  reg_update(s, 0);
}

static void backward_sqrt(oc_solver* s) {
  int n = s->n, m = s->m, N = s->N, L = n + m + 1;
  double* Sxx = s->Sxx;
  double* Sx = s->Sx;
  memcpy(Sxx + (size_t)(N - 1) * n * n, s->Qxx + (size_t)(N - 1) * n * n, sizeof(double) * n * n);
  memcpy(Sx + (size_t)(N - 1) * n, s->Qx + (size_t)(N - 1) * n, sizeof(double) * n);
  s->dV[0] = s->dV[1] = 0.0;
  s->bp_restarts = 0;
  double tmp_x[256], tmp_u[OM * 16], R[OM * OM], Quu_reg[OM * OM], Qux_reg[OM * 16], Kk[OM * 16], dk[OM], t[OM * OM];
  int k = N - 2;
  while (k >= 0) {
    const double* Fk = s->F + (size_t)k * n * L;
    const double* A = Fk;
    const double* B = Fk + n * n;
    const double* S1 = Sxx + (size_t)(k + 1) * n * n; /* factor */
    const double* s1 = Sx + (size_t)(k + 1) * n;
    double* Qx = s->Qx + (size_t)k * n;
    double* Qu = s->Qu + (size_t)k * m;
    double* Qxx = s->Qxx + (size_t)k * n * n;
    double* Quu = s->Quu + (size_t)k * m * m;
    double* Qux = s->Qux + (size_t)k * m * n;
    matTmul(t, A, n, n, s1, 1);
    for (int i = 0; i < n; i++) Qx[i] += t[i];
    matTmul(t, B, n, m, s1, 1);
    for (int i = 0; i < m; i++) Qu[i] += t[i];
    matmul(tmp_x, S1, n, n, A, n); /* S*fdx */
    matmul(tmp_u, S1, n, n, B, m); /* S*fdu */
    chol_plus(R, Qxx, n, tmp_x, n, n);
    memcpy(Qxx, R, sizeof(double) * n * n);
    chol_plus(R, Quu, m, tmp_u, n, m);
    memcpy(Quu, R, sizeof(double) * m * m);
    matTmul(t, tmp_u, n, m, tmp_x, n); /* tmp_u'*tmp_x */
    for (int i = 0; i < m * n; i++) Qux[i] += t[i];

    if (s->opts.bp_reg_type == 1) { /* :state: chol_plus(Q.uu, sqrt(ρ)*fdu) */
      double Bs[OM * 16], BtA[OM * 16];
      for (int i = 0; i < n * m; i++) Bs[i] = sqrt(s->rho) * B[i];
      chol_plus(Quu_reg, Quu, m, Bs, n, m);
      matTmul(BtA, B, n, m, A, n);
      for (int i = 0; i < m * n; i++) Qux_reg[i] = Qux[i] + s->rho * BtA[i];
    } else {
      double D[OM * OM];
      memset(D, 0, sizeof(D));
      for (int i = 0; i < m; i++) D[i + m * i] = sqrt(s->rho);
      chol_plus(Quu_reg, Quu, m, D, m, m);
      memcpy(Qux_reg, Qux, sizeof(double) * m * n);
    }
    /* if cond(Quu_reg) > 1e8: increase ρ, restart */
    if (cond2(Quu_reg, m) > 1e8) {
      reg_update(s, 1);
      s->bp_restarts++;
      k = N - 2;
      s->dV[0] = s->dV[1] = 0.0;
      if (s->bp_restarts > TOG_BP_MAX_RESTARTS) { /* restart cap: stop the trajectory (tog.h) */
        s->flags |= TOG_TRAJ_MAX_REG | TOG_TRAJ_BP_ABORTED;
        return; /* no :decrease, ΔV = 0 */
      }
      continue;
    }
    /* K = -Quu_reg\(Quu_reg'\Qux_reg) ; d = -Quu_reg\(Quu_reg'\Q.u) */
    /* (Quu_reg' \ and Quu_reg \ are triangular solves: Julia's `\` dispatches them to
       substitution; contract v2 multiplies by the diagonal reciprocals) */
    memcpy(Kk, Qux_reg, sizeof(double) * m * n);
    solve_uppert_rcp(Quu_reg, m, Kk, n);
    solve_upper_rcp(Quu_reg, m, Kk, n);
    for (int i = 0; i < m * n; i++) Kk[i] = -Kk[i];
    memcpy(dk, Qu, sizeof(double) * m);
    solve_uppert_rcp(Quu_reg, m, dk, 1);
    solve_upper_rcp(Quu_reg, m, dk, 1);
    for (int i = 0; i < m; i++) dk[i] = -dk[i];
    memcpy(s->K + (size_t)k * m * n, Kk, sizeof(double) * m * n);
    memcpy(s->d + (size_t)k * m, dk, sizeof(double) * m);
    /* S[k].x = Q.x + (K'*Q.uu')*(Q.uu*d) + K'*Q.u + Q.ux'*d */
    double* sk = Sx + (size_t)k * n;
    {
      double KtUt[OM * 16], Ud[OM], a[16], b[16], c[16];
      for (int j = 0; j < m; j++) /* K'*Quu' : n x m, (K'Quu')[i,j] = Σ_l K[l,i] Quu[j,l] */
        for (int i = 0; i < n; i++) {
          double acc = 0;
          for (int l = 0; l < m; l++) acc = fma(Kk[IDX(l, i, m)], Quu[IDX(j, l, m)], acc);
          KtUt[IDX(i, j, n)] = acc;
        }
      matmul(Ud, Quu, m, m, dk, 1);
      matmul(a, KtUt, n, m, Ud, 1);
      matTmul(b, Kk, m, n, Qu, 1);
      matTmul(c, Qux, m, n, dk, 1);
      for (int i = 0; i < n; i++) sk[i] = ((Qx[i] + a[i]) + b[i]) + c[i];
    }
    /* tmp1 = (Q.xx')\Q.ux'  (n x m) */
    double tmp1[OM * 16];
    int singular = 0;
    for (int i = 0; i < n; i++)
      if (Qxx[IDX(i, i, n)] == 0.0) singular = 1;
    for (int j = 0; j < m; j++)
      for (int i = 0; i < n; i++) tmp1[IDX(i, j, n)] = Qux[IDX(j, i, m)];
    if (singular) s->flags |= TOG_TRAJ_SINGULAR;
    solve_uppert_rcp(Qxx, n, tmp1, m); /* Q.xx upper-triangular: forward substitution */
    /* tmp2 = chol_minus(Q.uu, tmp1) */
    double tmp2[OM * OM];
    if (chol_minus(tmp2, Quu, m, tmp1, n)) {
      /* lowrankdowndate! throws PosDefException (backward_pass.jl:186-192): the solve of this
         trajectory stops here, like the restart cap (no :decrease, ΔV = 0) */
      s->flags |= TOG_TRAJ_SQRT_PD_FAIL | TOG_TRAJ_BP_ABORTED;
      s->dV[0] = s->dV[1] = 0.0;
      return;
    }
    /* S[k].xx = chol_plus(Q.xx + tmp1*K, tmp2*K) */
    {
      double top[256], bot[OM * 16];
      matmul(top, tmp1, n, m, Kk, n);
      for (int i = 0; i < n * n; i++) top[i] = Qxx[i] + top[i];
      matmul(bot, tmp2, m, m, Kk, n);
      chol_plus(Sxx + (size_t)k * n * n, top, n, bot, m, n);
    }
    /* ΔV */
    {
      double a = 0.0, Ud[OM], b = 0.0;
      for (int i = 0; i < m; i++) a = fma(dk[i], Qu[i], a);
      matmul(Ud, Quu, m, m, dk, 1);
      for (int i = 0; i < m; i++) b = fma(Ud[i], Ud[i], b);
      s->dV[0] += a;
      s->dV[1] += 0.5 * b;
    }
    k--;
  }
  reg_update(s, 0);
}

OC_EXPORT int oc_backward(oc_solver* s, int sq, double* dV) {
  if (sq)
    backward_sqrt(s);
  else
    backward_std(s);
  if (dV) {
    dV[0] = s->dV[0];
    dV[1] = s->dV[1];
  }
  return s->bp_restarts;
}

/* =====================================================================
 * Forward pass (src/solvers/ilqr/forward_pass.jl:5-85)
 * ===================================================================== */
OC_EXPORT double oc_forward(oc_solver* s, int al, double J_prev) {
  const tog_options* o = &s->opts;
  int n = s->n, m = s->m, N = s->N;
  double J = INFINITY, alpha = 1.0, z = -1.0, expected = 0.0;
  int iter = 0;
  s->ls_trials = 0;
  while ((z <= o->line_search_lower_bound || z > o->line_search_upper_bound) && J >= J_prev) {
    if (iter > o->iterations_linesearch) {
      memcpy(s->Xb, s->X, sizeof(double) * n * N);
      memcpy(s->Ub, s->U, sizeof(double) * m * (N - 1));
      J = cost(s, al, s->Xb, s->Ub);
      z = 0.0;
      alpha = 0.0;
      expected = 0.0;
      reg_update(s, 1);
      s->rho += o->bp_reg_fp;
      break;
    }
    int ok = oc_rollout(s, alpha);
    s->ls_trials++;
    if (!ok) {
      iter++;
      alpha /= 2.0;
      continue;
    }
    J = cost(s, al, s->Xb, s->Ub);
    expected = -alpha * (s->dV[0] + alpha * s->dV[1]);
    if (expected > 0.0)
      z = (J_prev - J) / expected;
    else
      z = -1.0;
    iter++;
    alpha /= 2.0;
  }
  s->alpha = 2.0 * alpha;
  s->z = z;
  s->expected = expected;
  if (J > J_prev) s->flags |= TOG_TRAJ_COST_INCREASED;
  return J;
}

/* =====================================================================
 * Solves
 * ===================================================================== */
/* gradient_type :ℓ2 / :ℓinf (ilqr_methods.jl:96-99): norm(compute_gradient(prob, solver)) with
   compute_gradient (:104-116) = vcat(Q[1].x, Q[1].u, ..., Q[N-1].x, Q[N-1].u, Q[N].x) of the plain
   (not square-root) cost_expansion! of the current objective (the AL one inside AL solves) at the new
   X, U; the AL terms use obj.C, the constraint values of the accepted trajectory (the last cost
   evaluation, A.10). ℓinf is LinearAlgebra.generic_normInf (NaN propagates). ℓ2: Julia 1.1 hands
   vectors of 32 or more Float64 to BLAS.nrm2, whose summation order and precision are the BLAS
   build's; this restatement takes generic_norm2's unscaled double sum in index order (jl_norm2), so
   the two agree to rounding (the convergence test grad < tol is unpinned within that rounding). */
static double expansion_gradient_norm(oc_solver* s, int linf) {
  int n = s->n, m = s->m, N = s->N;
  oc_cost_expansion(s, 0, s->al_mode); /* overwrites solver.Q, as reset!(solver.Q) + cost_expansion! */
  size_t len = (size_t)(N - 1) * (n + m) + n;
  double* g = (double*)malloc(sizeof(double) * len);
  size_t e = 0;
  for (int k = 0; k < N - 1; k++) {
    for (int i = 0; i < n; i++) g[e++] = s->Qx[(size_t)k * n + i];
    for (int i = 0; i < m; i++) g[e++] = s->Qu[(size_t)k * m + i];
  }
  for (int i = 0; i < n; i++) g[e++] = s->Qx[(size_t)(N - 1) * n + i];
  double r;
  if (linf) {
    r = fabs(g[0]);
    for (size_t i = 1; i < len; i++) {
      double v = fabs(g[i]);
      r = (isnan(r) || r > v) ? r : v;
    }
  } else {
    r = jl_norm2(g, (int)len);
  }
  free(g);
  return r;
}

/* gradient_todorov (ilqr_methods.jl:122-129) / gradient_feedforward (:135-137) / ℓ2, ℓinf (above) */
static double calc_gradient(oc_solver* s) {
  int m = s->m, N = s->N;
  if (s->opts.gradient_type == 2 || s->opts.gradient_type == 3)
    return expansion_gradient_norm(s, s->opts.gradient_type == 3);
  if (s->opts.gradient_type == 1) {
    double g = 0.0;
    for (int k = 0; k < N - 1; k++) {
      double t = 0;
      for (int i = 0; i < m; i++) t = fma(s->d[(size_t)k * m + i], s->d[(size_t)k * m + i], t);
      t = sqrt(t);
      if (t > g) g = t;
    }
    return g;
  }
  double sum = 0.0;
  for (int k = 0; k < N - 1; k++) {
    double mx = -INFINITY;
    for (int i = 0; i < m; i++) {
      double v = fabs(s->d[(size_t)k * m + i]) / (fabs(s->U[(size_t)k * m + i]) + 1.0);
      if (v > mx || isnan(v)) mx = v;
    }
    sum += mx;
  }
  return sum / N; /* mean over N entries, entry N = 0 (A.3) */
}

static void record_iteration(oc_solver* s, double J, double dJ) {
  s->iterations++;
  s->J = J;
  s->dJ = dJ;
  s->gradient = calc_gradient(s);
  if (dJ == 0.0)
    s->zero_count++;
  else
    s->zero_count = 0;
  const double rec[3] = {J, dJ, s->gradient};
  hist_push(&s->hin, &s->hin_n, &s->hin_cap, 3, rec);
}

static void record_outer(oc_solver* s, double J, double mumax) { /* augmented_lagrangian_methods.jl:79-97 */
  const double rec[4] = {(double)s->iterations, J, s->c_max, mumax};
  hist_push(&s->hout, &s->hout_n, &s->hout_cap, 4, rec);
}

static int evaluate_convergence(oc_solver* s, double cost_tol, double grad_tol) {
  if (0.0 < s->dJ && s->dJ < cost_tol) return 1;
  if (s->gradient < grad_tol) return 1;
  if (s->iterations >= s->opts.iterations) return 1;
  if (s->zero_count > s->opts.dJ_counter_limit) return 1;
  return 0;
}

/* one iLQR step! (ilqr_methods.jl:47-53) + the bookkeeping of solve! (:21-42).
   returns 1 if the inner solve finished (converged or early exit). */
static int ilqr_iterate(oc_solver* s, int al, double cost_tol, double grad_tol) {
  oc_jacobians(s);
  if (oc_cost_expansion(s, s->opts.square_root, al)) s->flags |= TOG_TRAJ_SQRT_PD_FAIL;
  oc_backward(s, s->opts.square_root, NULL);
  if (s->flags & TOG_TRAJ_BP_ABORTED) return 1; /* restart cap hit: the trajectory stops here */
  double J = oc_forward(s, al, s->J);
  /* error("Cost increased during Forward Pass") (forward_pass.jl:80-82): the solve ends there, with no
     bookkeeping of the step */
  if (s->flags & TOG_TRAJ_COST_INCREASED) return 1;
  s->total_steps++;
  if (s->trace_len < 4096) {
    double* t = s->trace + 6 * s->trace_len++;
    t[0] = J; t[1] = s->alpha; t[2] = s->rho; t[3] = s->bp_restarts; t[4] = s->ls_trials; t[5] = s->z;
  }
  if (J > s->opts.max_cost_value) {
    s->flags |= TOG_TRAJ_COST_BLOWUP;
    return 1;
  }
  memcpy(s->X, s->Xb, sizeof(double) * s->n * s->N);
  memcpy(s->U, s->Ub, sizeof(double) * s->m * (s->N - 1));
  double dJ = fabs(J - s->J);
  record_iteration(s, J, dJ);
  if (evaluate_convergence(s, cost_tol, grad_tol)) {
    if (s->iterations >= s->opts.iterations) s->flags |= TOG_TRAJ_MAX_ITERS;
    return 1;
  }
  return 0;
}

static void ilqr_reset(oc_solver* s) { /* reset!(solver) ilqr_solver.jl:146-154 */
  s->iterations = 0;
  s->zero_count = 0;
  s->rho = 0.0;
  s->drho = 0.0;
}

/* solve!(prob, iLQRSolver) ilqr_methods.jl:3-45 ; al selects the AL objective (inner solve) */
static void ilqr_solve(oc_solver* s, int al, double cost_tol, double grad_tol) {
  s->al_mode = al;
  ilqr_reset(s);
  oc_rollout_open_loop(s);
  double J_prev = cost(s, al, s->X, s->U);
  record_iteration(s, J_prev, INFINITY);
  for (int i = 0; i < s->opts.iterations; i++) {
    if (ilqr_iterate(s, al, cost_tol, grad_tol)) break;
  }
}

OC_EXPORT int oc_solve_ilqr(oc_solver* s) {
  s->flags = 0;
  s->total_steps = 0;
  s->trace_len = 0;
  s->hin_n = s->hout_n = 0;
  ilqr_solve(s, 0, s->opts.cost_tolerance, s->opts.gradient_norm_tolerance);
  s->flags |= TOG_TRAJ_CONVERGED;
  return s->total_steps;
}

/* max_violation(solver) augmented_lagrangian_methods.jl:171-184 */
static double max_violation(oc_solver* s) {
  int N = s->N, P = s->pmax;
  double c_max = 0.0;
  for (int k = 0; k < N; k++) {
    if (s->p[k] == 0) continue;
    double e = 0.0, im = -INFINITY;
    int ni = 0;
    for (int i = 0; i < s->p[k]; i++) {
      size_t j = (size_t)k * P + i;
      if (s->ineq[j]) {
        ni++;
        im = tog_jlmax(im, s->C[j]); /* maximum(C.inequality): NaN propagates */
      } else
        e = tog_jlmax(e, fabs(s->C[j])); /* norm(C.equality, Inf) */
    }
    c_max = tog_jlmax(e, c_max);
    if (ni > 0) c_max = tog_jlmax(tog_jlmax(0.0, im), c_max);
  }
  return c_max;
}

/* solve!(prob, AugmentedLagrangianSolver) augmented_lagrangian_methods.jl:2-31 */
OC_EXPORT int oc_solve_al(oc_solver* s) {
  const tog_options* o = &s->opts;
  int N = s->N, P = s->pmax;
  s->flags = 0;
  s->total_steps = 0;
  s->trace_len = 0;
  /* reset!(solver): λ = 0, μ = penalty_initial (augmented_lagrangian_solver.jl:173-187) */
  for (int i = 0; i < P * N; i++) {
    s->lam[i] = 0.0;
    s->mu[i] = o->penalty_initial;
  }
  oc_rollout_open_loop(s);
  s->hin_n = s->hout_n = 0;
  s->iterations = 0; /* the reset inner solver's stats[:iterations] */
  const double J0 = al_cost(s, s->X, s->U); /* record_iteration!(prob_al, solver, cost(prob_al)) */
  s->c_max = max_violation(s);
  double mu0 = 0.0; /* max_penalty(solver) */
  for (int k = 0; k < N; k++)
    for (int j = 0; j < s->p[k]; j++) mu0 = fmax(mu0, s->mu[(size_t)k * P + j]);
  record_outer(s, J0, mu0);
  for (int i = 1; i <= o->al_iterations; i++) {
    s->al_iter = i;
    /* set_tolerances! (:39-50) */
    double ct = (i != o->al_iterations) ? o->al_cost_tolerance_intermediate : o->al_cost_tolerance;
    double gt = (i != o->al_iterations) ? o->al_gradient_norm_tolerance_intermediate : o->al_gradient_norm_tolerance;
    ilqr_solve(s, 1, ct, gt);
    if (s->flags & TOG_TRAJ_BP_ABORTED) break; /* stopped by the restart cap (tog.h) */
    if (s->flags & TOG_TRAJ_COST_INCREASED) break; /* the inner solve raised */
    const double Jal = al_cost(s, s->X, s->U); /* J = cost(prob) */
    /* dual_update! (:107-118) */
    for (int k = 0; k < N; k++)
      for (int j = 0; j < s->p[k]; j++) {
        size_t q = (size_t)k * P + j;
        double l = s->lam[q] + s->mu[q] * s->C[q];
        l = tog_jlmax(o->dual_min, tog_jlmin(o->dual_max, l));
        if (s->ineq[q]) l = tog_jlmax(0.0, l);
        s->lam[q] = l;
      }
    update_active_set(s);
    /* penalty_update! (:121-126) */
    double mumax = 0.0;
    for (int k = 0; k < N; k++)
      for (int j = 0; j < s->p[k]; j++) {
        size_t q = (size_t)k * P + j;
        s->mu[q] = fmax(0.0, fmin(o->penalty_max, o->penalty_scaling * s->mu[q]));
        if (s->mu[q] > mumax) mumax = s->mu[q];
      }
    s->c_max = max_violation(s);
    record_outer(s, Jal, mumax);
    int conv = 0;
    if (o->kickout_max_penalty && mumax == o->penalty_max) conv = 1;
    if (s->c_max < o->constraint_tolerance) conv = 1;
    if (conv) {
      s->flags |= TOG_TRAJ_AL_CONVERGED;
      break;
    }
    if (i == o->al_iterations) s->flags |= TOG_TRAJ_AL_MAX_ITERS;
  }
  return s->total_steps;
}

/* =====================================================================
 * Field access
 * ===================================================================== */
OC_EXPORT void oc_get(oc_solver* s, int field, double* out) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax, L = n + m + 1;
  switch (field) {
    case TOG_FIELD_X: memcpy(out, s->X, sizeof(double) * n * N); break;
    case TOG_FIELD_U: memcpy(out, s->U, sizeof(double) * m * (N - 1)); break;
    case TOG_FIELD_XBAR: memcpy(out, s->Xb, sizeof(double) * n * N); break;
    case TOG_FIELD_UBAR: memcpy(out, s->Ub, sizeof(double) * m * (N - 1)); break;
    case TOG_FIELD_K: memcpy(out, s->K, sizeof(double) * m * n * (N - 1)); break;
    case TOG_FIELD_D: memcpy(out, s->d, sizeof(double) * m * (N - 1)); break;
    case TOG_FIELD_A:
      for (int k = 0; k < N - 1; k++) memcpy(out + (size_t)k * n * n, s->F + (size_t)k * n * L, sizeof(double) * n * n);
      break;
    case TOG_FIELD_B:
      for (int k = 0; k < N - 1; k++)
        memcpy(out + (size_t)k * n * m, s->F + (size_t)k * n * L + n * n, sizeof(double) * n * m);
      break;
    case TOG_FIELD_S: memcpy(out, s->Sxx, sizeof(double) * n * n * N); break;
    case TOG_FIELD_SX: memcpy(out, s->Sx, sizeof(double) * n * N); break;
    case TOG_FIELD_DV: out[0] = s->dV[0]; out[1] = s->dV[1]; break;
    case TOG_FIELD_LAMBDA: memcpy(out, s->lam, sizeof(double) * P * N); break;
    case TOG_FIELD_MU: memcpy(out, s->mu, sizeof(double) * P * N); break;
    case TOG_FIELD_C: memcpy(out, s->C, sizeof(double) * P * N); break;
    case TOG_FIELD_X0: memcpy(out, s->x0, sizeof(double) * n); break;
    case TOG_FIELD_RHO: out[0] = s->rho; out[1] = s->drho; break;
    case TOG_FIELD_Q: { /* per knot [Q.x; Q.u; Q.xx; Q.uu; Q.ux] (terminal: u parts 0) */
      size_t nq = (size_t)n + m + n * n + m * m + m * n;
      memset(out, 0, sizeof(double) * nq * N);
      for (int k = 0; k < N; k++) {
        double* q = out + (size_t)k * nq;
        memcpy(q, s->Qx + (size_t)k * n, sizeof(double) * n);
        memcpy(q + n + m, s->Qxx + (size_t)k * n * n, sizeof(double) * n * n);
        if (k < N - 1) {
          memcpy(q + n, s->Qu + (size_t)k * m, sizeof(double) * m);
          memcpy(q + n + m + n * n, s->Quu + (size_t)k * m * m, sizeof(double) * m * m);
          memcpy(q + n + m + n * n + m * m, s->Qux + (size_t)k * m * n, sizeof(double) * m * n);
        }
      }
      break;
    }
    case TOG_FIELD_STATS:
      memset(out, 0, sizeof(double) * TOG_NSTATS);
      out[TOG_STAT_J] = s->J;
      out[TOG_STAT_DJ] = s->dJ;
      out[TOG_STAT_GRADIENT] = s->gradient;
      out[TOG_STAT_ITERATIONS] = s->iterations;
      out[TOG_STAT_ZERO_COUNT] = s->zero_count;
      out[TOG_STAT_ALPHA] = s->alpha;
      out[TOG_STAT_Z] = s->z;
      out[TOG_STAT_C_MAX] = s->c_max;
      out[TOG_STAT_AL_ITER] = s->al_iter;
      out[TOG_STAT_TOTAL_STEPS] = s->total_steps;
      out[TOG_STAT_LS_TRIALS] = s->ls_trials;
      out[TOG_STAT_BP_RESTARTS] = s->bp_restarts;
      out[TOG_STAT_FLAGS] = s->flags;
      break;
  }
}

OC_EXPORT void oc_set(oc_solver* s, int field, const double* in) {
  int n = s->n, m = s->m, N = s->N, P = s->pmax;
  switch (field) {
    case TOG_FIELD_X: memcpy(s->X, in, sizeof(double) * n * N); break;
    case TOG_FIELD_U: memcpy(s->U, in, sizeof(double) * m * (N - 1)); break;
    case TOG_FIELD_K: memcpy(s->K, in, sizeof(double) * m * n * (N - 1)); break;
    case TOG_FIELD_D: memcpy(s->d, in, sizeof(double) * m * (N - 1)); break;
    case TOG_FIELD_LAMBDA: memcpy(s->lam, in, sizeof(double) * P * N); break;
    case TOG_FIELD_MU: memcpy(s->mu, in, sizeof(double) * P * N); break;
    case TOG_FIELD_DV: s->dV[0] = in[0]; s->dV[1] = in[1]; break;
    case TOG_FIELD_RHO: s->rho = in[0]; s->drho = in[1]; break;
    case TOG_FIELD_X0: memcpy(s->x0, in, sizeof(double) * n); break;
  }
}

OC_EXPORT void oc_update_constraints(oc_solver* s) {
  update_constraints(s, s->X, s->U);
  update_active_set(s);
}

OC_EXPORT int oc_get_trace(oc_solver* s, double* out) {
  memcpy(out, s->trace, sizeof(double) * 6 * s->trace_len);
  return s->trace_len;
}

OC_EXPORT double oc_max_violation(oc_solver* s) { return max_violation(s); }

/* the solver.stats vectors of the last solve: which 0 = inner records (3 doubles each), 1 = outer records
   (4 doubles each), 2 = projected Newton records (2 doubles each); out may be NULL (count only). Returns
   the record count. */
OC_EXPORT int oc_get_history(oc_solver* s, int which, double* out) {
  const int n = which == 2 ? s->hpn_n : (which ? s->hout_n : s->hin_n);
  const int w = which == 2 ? 2 : (which ? 4 : 3);
  const double* src = which == 2 ? s->hpn : (which ? s->hout : s->hin);
  if (out && n) memcpy(out, src, sizeof(double) * w * (size_t)n);
  return n;
}

/* =====================================================================
 * Batched CPU baseline: B independent solves over `nthreads` OpenMP threads.
 * Returns Σ iLQR step!s. (bench.py cpu_baseline leg)
 * ===================================================================== */
/* busy (optional): Σ over trajectories of the seconds each one's solve took (the CPU baseline's
   sustained rate is steps / (busy / nthreads): the heavy tail of iteration counts makes the wall time of a
   bounded sample a measure of its slowest trajectory, not of the cores' throughput) */
OC_EXPORT int64_t oc_solve_batch_timed(const tog_problem_desc* d, const tog_options* o, int mode, const double* x0,
                                       const double* U0, int64_t B, int nthreads, double* busy) {
  int n = d->n, m = d->m, N = d->N;
  int64_t total = 0;
  double bt = 0.0;
#ifdef _OPENMP
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1) reduction(+ : total, bt)
#endif
  for (int64_t b = 0; b < B; b++) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oc_solver* s = oc_create(d, o);
    oc_set_state(s, x0 + (size_t)b * n, U0 + (size_t)b * m * (N - 1), NULL);
    total += mode == TOG_MODE_AL ? oc_solve_al(s) : oc_solve_ilqr(s);
    oc_destroy(s);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    bt += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  }
  if (busy) *busy = bt;
  (void)nthreads;
  return total;
}
OC_EXPORT int64_t oc_solve_batch(const tog_problem_desc* d, const tog_options* o, int mode, const double* x0,
                                 const double* U0, int64_t B, int nthreads) {
  return oc_solve_batch_timed(d, o, mode, x0, U0, B, nthreads, NULL);
}

/* ALTRO phase 2: projected Newton feasible projection (oracle/tog_oracle_pn.c) */
#include "tog_oracle_pn.c"
#include "tog_oracle_cost.c"
