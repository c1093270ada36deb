// Host build of the HIP Kuka model (csrc/tog_device.hpp) checked bit for bit against the oracle's
// f_kuka: continuous dynamics, the RK3 step, the dual-number Jacobian through the step
// (oc_discrete_jacobian_fd), and the stage-chain Jacobian (oc_discrete_jacobian) as the
// device lanes of csrc/tog_kuka_jac.hpp compute it: the q-partial lanes (full dual), the v-partial
// lanes (mixed double/dual bias and solve), the u columns (tangent-only solves) and the chain with fma
// chains in k order (the matrix cores' order). Zeros compare equal regardless of sign. Built and run by
// tests/test_kuka.py (hipcc --cuda-host-only; no GPU needed). argv[1] = path of liboracle.so.
#include "tog_device.hpp"
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
using namespace tog;
typedef void (*jacf)(int, int, double*, const double*, const double*, double);
typedef void (*ctf)(int, double*, const double*, const double*);
typedef void (*dff)(int, int, double*, const double*, const double*, double);

static bool same(double a, double b) { return a == b ? true : memcmp(&a, &b, 8) == 0; }

// the stage Jacobian rows 7..13 at (s, u), lane by lane as the device computes them
static void stage_jac(double J[7][21], const double* s, const double* u) {
  for (int p = 0; p < 7; p++) {  // q partials: the full dual step
    Dual<1> xs[14], us[7], fd[14];
    for (int i = 0; i < 14; i++) { xs[i].v = s[i]; xs[i].g[0] = (i == p); }
    for (int i = 0; i < 7; i++) { us[i].v = u[i]; us[i].g[0] = 0.0; }
    Kuka::f(fd, xs, us);
    for (int i = 0; i < 7; i++) J[i][p] = fd[7 + i].g[0];
  }
  for (int p = 0; p < 7; p++) {  // v partials at fixed q
    double q[7], uu[7], L[7][7], cq[7], sq[7];
    Dual<1> qd[7], tau[7], vd[7];
    for (int i = 0; i < 7; i++) { q[i] = s[i]; qd[i].v = s[7 + i]; qd[i].g[0] = (i == p); uu[i] = u[i]; }
    Kuka::bias(tau, cq, sq, q, qd);
    Kuka::mass(L, cq, sq);
    Kuka::chol(L);
    Kuka::solve(vd, L, uu, tau);
    for (int i = 0; i < 7; i++) J[i][7 + p] = vd[i].g[0];
  }
  {  // u partials: tangent-only solves with the primal factor
    double tau[7], cq[7], sq[7], L[7][7], il[7];
    Kuka::bias(tau, cq, sq, s, s + 7);
    Kuka::mass(L, cq, sq);
    Kuka::chol(L);
    for (int i = 0; i < 7; i++) il[i] = 1.0 / L[i][i];
    for (int p = 0; p < 7; p++) {
      double y[7], g[7];
      for (int i = 0; i < 7; i++) {
        double t = (i == p) ? 1.0 : 0.0;
        for (int k = 0; k < i; k++) t = t - L[i][k] * y[k];
        y[i] = t * il[i];
      }
      for (int i = 6; i >= 0; i--) {
        double t = y[i];
        for (int k = i + 1; k < 7; k++) t = t - L[k][i] * g[k];
        g[i] = t * il[i];
      }
      for (int i = 0; i < 7; i++) J[i][14 + p] = g[i];
    }
  }
}

static void chain_jac(double* S, const double* x, const double* u, double dt) {
  double xd[14], k1[14], t2[14], t3[14];
  Kuka::f<double>(xd, x, u);
  for (int i = 0; i < 14; i++) { k1[i] = xd[i] * dt; t2[i] = x[i] + k1[i] / 2.0; }
  Kuka::f<double>(xd, t2, u);
  for (int i = 0; i < 14; i++) t3[i] = (x[i] - k1[i]) + 2.0 * (xd[i] * dt);
  double J[3][7][21];
  stage_jac(J[0], x, u);
  stage_jac(J[1], t2, u);
  stage_jac(J[2], t3, u);
  static double K1[14][21], T[14][21], Ss[14][21], F[14][21];
  for (int i = 0; i < 14; i++)
    for (int p = 0; p < 21; p++) {
      const double f1 = (i < 7) ? ((p == 7 + i) ? 1.0 : 0.0) : J[0][i - 7][p];
      K1[i][p] = f1 * dt;
      T[i][p] = ((i == p) ? 1.0 : 0.0) + K1[i][p] / 2.0;
    }
  for (int st = 1; st < 3; st++) {
    for (int p = 0; p < 21; p++)
      for (int i = 0; i < 14; i++) {
        if (i < 7) { F[i][p] = T[7 + i][p]; continue; }
        double acc = (p >= 14) ? J[st][i - 7][p] : 0.0;
        for (int j = 0; j < 16; j++) acc = fma(j < 14 ? J[st][i - 7][j] : 0.0, j < 14 ? T[j][p] : 0.0, acc);
        F[i][p] = acc;
      }
    for (int i = 0; i < 14; i++)
      for (int p = 0; p < 21; p++) {
        const double kk = F[i][p] * dt;
        if (st == 1) {
          T[i][p] = (((i == p) ? 1.0 : 0.0) - K1[i][p]) + 2.0 * kk;
          Ss[i][p] = K1[i][p] + 4.0 * kk;
        } else {
          S[i + 14 * p] = ((i == p) ? 1.0 : 0.0) + (Ss[i][p] + kk) / 6.0;
        }
      }
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  void* h = dlopen(argv[1], RTLD_NOW);
  if (!h) return 2;
  ctf cf = (ctf)dlsym(h, "oc_continuous_f");
  jacf jf = (jacf)dlsym(h, "oc_discrete_jacobian");
  jacf jfd = (jacf)dlsym(h, "oc_discrete_jacobian_fd");
  dff df = (dff)dlsym(h, "oc_discrete_f");
  if (!cf || !jf || !jfd || !df) return 2;
  double x[14], u[7], xd[14], xo[14], S[14 * 22], Sc[14 * 21];
  srand(1);
  int bad = 0;
  double maxrel = 0.0;
  for (int t = 0; t < 100; t++) {
    for (int i = 0; i < 14; i++) x[i] = (rand() / (double)RAND_MAX - 0.5) * 4;
    for (int i = 0; i < 7; i++) u[i] = (rand() / (double)RAND_MAX - 0.5) * 20;
    Kuka::f<double>(xd, x, u);
    cf(TOG_MODEL_KUKA, xo, x, u);
    for (int i = 0; i < 14; i++) if (!same(xd[i], xo[i])) { bad++; if (bad < 5) printf("f mismatch t=%d i=%d %.17g %.17g\n", t, i, xd[i], xo[i]); }
    discrete_step<Kuka, TOG_RK3>(xd, x, u, 0.1);
    df(TOG_MODEL_KUKA, TOG_RK3, xo, x, u, 0.1);
    for (int i = 0; i < 14; i++) if (!same(xd[i], xo[i])) { bad++; if (bad < 5) printf("fd mismatch t=%d i=%d %.17g %.17g\n", t, i, xd[i], xo[i]); }
    jfd(TOG_MODEL_KUKA, TOG_RK3, S, x, u, 0.1);
    for (int c = 0; c < 21; c++) {
      Dual<1> X[14], U[7], XN[14];
      for (int i = 0; i < 14; i++) { X[i].v = x[i]; X[i].g[0] = (i == c); }
      for (int i = 0; i < 7; i++) { U[i].v = u[i]; U[i].g[0] = (14 + i == c); }
      discrete_step<Kuka, TOG_RK3>(XN, X, U, 0.1);
      for (int i = 0; i < 14; i++) if (!same(XN[i].g[0], S[i + 14 * c])) { bad++; if (bad < 5) printf("jac mismatch t=%d c=%d i=%d %.17g %.17g\n", t, c, i, XN[i].g[0], S[i+14*c]); }
    }
    // stage-chain form: device lanes (host build) == oracle, and within rounding of the dual form
    double Sf[14 * 22];
    memcpy(Sf, S, sizeof(Sf));
    jf(TOG_MODEL_KUKA, TOG_RK3, S, x, u, 0.1);
    chain_jac(Sc, x, u, 0.1);
    for (int e = 0; e < 14 * 21; e++) {
      if (!same(Sc[e], S[e])) { bad++; if (bad < 5) printf("chain mismatch t=%d e=%d %.17g %.17g\n", t, e, Sc[e], S[e]); }
    }
    double dmax = 0.0, smax = 0.0;
    for (int e = 0; e < 14 * 21; e++) {
      dmax = fmax(dmax, fabs(S[e] - Sf[e]));
      smax = fmax(smax, fabs(Sf[e]));
    }
    if (dmax / smax > maxrel) maxrel = dmax / smax;
  }
  printf("bad=%d chain_vs_dual_rel=%.3e (max |diff| / max |entry| per Jacobian)\n", bad, maxrel);
  return (bad != 0 || maxrel > 1e-11);
}
