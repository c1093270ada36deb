// Host build of the HIP Kuka model (csrc/tog_device.hpp) checked bit for bit against the oracle's
// f_kuka: continuous dynamics, the RK3 step and the dual-number Jacobian columns. Built and run by
// tests/test_kuka.py (hipcc --cuda-host-only; no GPU needed). argv[1] = path of liboracle.so.
#include "tog_device.hpp"
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <dlfcn.h>
using namespace tog;
typedef void (*jacf)(int, int, double*, const double*, const double*, double);
typedef void (*ctf)(int, double*, const double*, const double*);
typedef void (*dff)(int, int, double*, const double*, const double*, double);
int main(int argc, char** argv) {
  if (argc < 2) return 2;
  void* h = dlopen(argv[1], RTLD_NOW);
  if (!h) return 2;
  ctf cf = (ctf)dlsym(h, "oc_continuous_f");
  jacf jf = (jacf)dlsym(h, "oc_discrete_jacobian");
  dff df = (dff)dlsym(h, "oc_discrete_f");
  double x[14], u[7], xd[14], xo[14], S[14 * 22];
  srand(1);
  int bad = 0;
  for (int t = 0; t < 100; t++) {
    for (int i = 0; i < 14; i++) x[i] = (rand() / (double)RAND_MAX - 0.5) * 4;
    for (int i = 0; i < 7; i++) u[i] = (rand() / (double)RAND_MAX - 0.5) * 20;
    Kuka::f<double>(xd, x, u);
    cf(TOG_MODEL_KUKA, xo, x, u);
    for (int i = 0; i < 14; i++) if (memcmp(&xd[i], &xo[i], 8)) { bad++; if (bad < 5) printf("f mismatch t=%d i=%d %.17g %.17g\n", t, i, xd[i], xo[i]); }
    discrete_step<Kuka, TOG_RK3>(xd, x, u, 0.1);
    df(TOG_MODEL_KUKA, TOG_RK3, xo, x, u, 0.1);
    for (int i = 0; i < 14; i++) if (memcmp(&xd[i], &xo[i], 8)) { bad++; if (bad < 5) printf("fd mismatch t=%d i=%d %.17g %.17g\n", t, i, xd[i], xo[i]); }
    jf(TOG_MODEL_KUKA, TOG_RK3, S, x, u, 0.1);
    for (int c = 0; c < 21; c++) {
      Dual<1> X[14], U[7], XN[14];
      for (int i = 0; i < 14; i++) { X[i].v = x[i]; X[i].g[0] = (i == c); }
      for (int i = 0; i < 7; i++) { U[i].v = u[i]; U[i].g[0] = (14 + i == c); }
      discrete_step<Kuka, TOG_RK3>(XN, X, U, 0.1);
      for (int i = 0; i < 14; i++) if (memcmp(&XN[i].g[0], &S[i + 14 * c], 8)) { bad++; if (bad < 5) printf("jac mismatch t=%d c=%d i=%d %.17g %.17g\n", t, c, i, XN[i].g[0], S[i+14*c]); }
    }
  }
  printf("bad=%d\n", bad);
  return bad != 0;
}
