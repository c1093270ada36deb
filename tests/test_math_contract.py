"""The shared arithmetic primitives of include/tog_math.h, run through the oracle build
(host and device compile the same header): tog_rsqrt, the 1/sqrt of chol_minus contract v4, within
2 ulp of the correctly rounded 1/sqrt on 2^20 points, and its boundary values; chol_minus at
s^2 == 1 exactly, where the reference's c = sqrt(1 - s^2) is 0 (backward_pass.jl:186-192,
lowrankdowndate!) and the diagonal must come out 0, not NaN."""
import ctypes as C

import numpy as np


def _ulp_dist(a, b):
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    return np.abs(ia - ib)


def test_rsqrt_within_2ulp_on_2pow20_points(oracle):
    L = oracle.lib()
    L.oc_rsqrt.restype = C.c_double
    L.oc_rsqrt.argtypes = [C.c_double]
    rng = np.random.default_rng(20)
    # normal range, log-uniform over the exponent range plus dense sampling of [0, 1] (chol_minus's y)
    y = np.concatenate([np.exp2(rng.uniform(-1020, 1020, 1 << 19)), rng.uniform(0, 1, 1 << 19)])
    y = y[y > 0]
    got = np.array([L.oc_rsqrt(float(v)) for v in y])
    ref = 1.0 / np.sqrt(y.astype(np.longdouble))
    ref = ref.astype(np.float64)
    assert _ulp_dist(got, ref).max() <= 2


def test_rsqrt_boundary_values(oracle):
    L = oracle.lib()
    L.oc_rsqrt.restype = C.c_double
    L.oc_rsqrt.argtypes = [C.c_double]
    assert L.oc_rsqrt(0.0) == np.inf
    assert L.oc_rsqrt(np.inf) == 0.0
    assert np.isnan(L.oc_rsqrt(-1.0))
    assert np.isnan(L.oc_rsqrt(np.nan))


def test_chol_minus_zero_cosine_gives_zero_diagonal(oracle):
    L = oracle.lib()
    dp = C.POINTER(C.c_double)
    L.oc_chol_minus.restype = C.c_int
    L.oc_chol_minus.argtypes = [dp, dp, C.c_int, dp, C.c_int]
    # A = [[2]], downdate by the row [2]: s = 2 * (1/2) = 1 exactly, so c = 0 and the factor is 0
    # (with more columns the reference's (A_ij - s x_j)/c then divides by zero and the next row's
    # downdate throws PosDefException; that is the TOG_TRAJ_SQRT_PD_FAIL path)
    A = np.array([[2.0]], order="F")
    Bv = np.array([[2.0]], order="F")
    U = np.full((1, 1), np.nan, order="F")
    rc = L.oc_chol_minus(U.ctypes.data_as(dp), A.ctypes.data_as(dp), 1, Bv.ctypes.data_as(dp), 1)
    assert rc == 0
    assert U[0, 0] == 0.0


def test_sincos_bit_identical_to_sin_and_cos(tmp_path):
    """tog_sincos (one reduction, both kernels, branch-free selection: the Kuka joints and every dual
    sin/cos) against tog_sin / tog_cos bit for bit, host build, over 2^18 points spread over the
    reduction's range plus the branch boundaries, signed zeros and non-finite values."""
    import pathlib
    import subprocess
    root = pathlib.Path(__file__).resolve().parents[1]
    src = tmp_path / "sc.c"
    src.write_text(r'''
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "tog_math.h"
int main(void) {
  long bad = 0, n = 0;
  const double sp[] = {0.0, -0.0, 7.85398163397448278999e-01, -7.85398163397448278999e-01,
                       7.853981633974482e-01, 7.853981633974484e-01, 1.5707963267948966, 3.141592653589793,
                       -3.141592653589793, 4.71238898038469, 1e-300, -1e-300, 5e5, -5e5,
                       1.0 / 0.0, -1.0 / 0.0, 0.0 / 0.0};
  uint64_t st = 88172645463325252ull;
  for (long i = 0; i < (1L << 18) + (long)(sizeof(sp) / sizeof(sp[0])); i++) {
    double x;
    if (i < (long)(sizeof(sp) / sizeof(sp[0]))) x = sp[i];
    else {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      const double u = (double)(st >> 11) / 9007199254740992.0;
      x = (i & 1) ? (u - 0.5) * 40.0 : (u - 0.5) * 4.0;
    }
    double s, c;
    tog_sincos(x, &s, &c);
    const double s0 = tog_sin(x), c0 = tog_cos(x);
    n++;
    if (memcmp(&s, &s0, 8) || memcmp(&c, &c0, 8)) {
      if (!(s != s && s0 != s0 && c != c && c0 != c0)) bad++;
    }
  }
  printf("%ld %ld\n", n, bad);
  return 0;
}
''')
    exe = tmp_path / "sc"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", str(root / "include"), str(src), "-o", str(exe), "-lm"],
                   check=True)
    n, bad = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert n > 1 << 18 and bad == 0


def test_div6_equals_division(tmp_path):
    """tog_div6 (Markstein's corrected product, the RK3/RK4 steps' final /6 on both sides) against x / 6.0
    bit for bit: 5e7 random bit patterns (the finite ones), a sweep of 1 + k ulp and 1.5 + k ulp over
    every 7th binade, and the ranges that take the division (zeros, subnormals, infinities, NaN)."""
    import pathlib
    import subprocess
    root = pathlib.Path(__file__).resolve().parents[1]
    src = tmp_path / "d6.c"
    src.write_text(r'''
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include "tog_math.h"
static long bad = 0, n = 0;
static void chk(double x) {
  const double a = tog_div6(x), b = x / 6.0;
  n++;
  if (memcmp(&a, &b, 8) && !(a != a && b != b)) bad++;
}
int main(void) {
  uint64_t st = 0x9E3779B97F4A7C15ull;
  for (long i = 0; i < 50000000L; i++) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    double x;
    memcpy(&x, &st, 8);
    chk(x);
  }
  for (int e = -1074; e <= 1023; e += 7)
    for (long k = -2000; k <= 2000; k++) {
      chk(ldexp(1.0 + k * 0x1p-52, e));
      chk(ldexp(1.5 + k * 0x1p-52, e));
    }
  const double sp[] = {0.0, -0.0, 1.0 / 0.0, -1.0 / 0.0, 0.0 / 0.0, 0x1p-1074, -0x1p-1074, 0x1p-1000, 0x1.fffffffffffffp-1001,
                       1.7976931348623157e308, -1.7976931348623157e308, 6.0, -6.0, 3.0};
  for (unsigned i = 0; i < sizeof(sp) / sizeof(sp[0]); i++) chk(sp[i]);
  printf("%ld %ld\n", n, bad);
  return 0;
}
''')
    exe = tmp_path / "d6"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", str(root / "include"), str(src), "-o", str(exe), "-lm"],
                   check=True)
    n, bad = map(int, subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split())
    assert n > 50000000 and bad == 0
