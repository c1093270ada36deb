/*
 * tog_math.h — deterministic transcendental primitives shared by host and device code.
 *
 * The hot path's arithmetic contract: every kernel and the CPU oracle evaluate the
 * same IEEE-754 fp64 operation sequence — no compiler contraction (-ffp-contract=off), explicit
 * fma() exactly where both sides write it, correctly rounded division and sqrt — so GPU results are
 * bit-identical to the CPU restatement. libm's sin/cos (glibc) and the GPU's OCML sin/cos may differ
 * in the last ulp, so the models that need them (cartpole, car, pendulum) use this one
 * implementation on both sides: fdlibm's __kernel_sin/__kernel_cos polynomials on [-pi/4, pi/4]
 * after a two-constant Cody-Waite reduction by pi/2: within 2 ulp of libm for |x| < 2^19, except
 * right next to the zeros (x ~ k*pi) where the absolute error stays below 2^-80.
 */
#ifndef TOG_MATH_H
#define TOG_MATH_H

#include <math.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TOG_HD __host__ __device__ inline
#else
#define TOG_HD static inline
#endif

TOG_HD double tog__ksin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double z = x * x;
  const double v = z * x;
  const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}

TOG_HD double tog__kcos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  const double z = x * x;
  const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + z * r);
}

/* reduce x to r in [-pi/4, pi/4], returns the quadrant */
TOG_HD int tog__rem_pio2(double x, double* r) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
  const double pio2_1t = 6.07710050650619224932e-11; /* pi/2 - pio2_1 */
  const double fn = rint(x * invpio2);
  *r = (x - fn * pio2_1) - fn * pio2_1t;
  return (int)((long long)fn & 3);
}

TOG_HD double tog_sin(double x) {
  if (!isfinite(x)) return x - x; /* NaN */
  if (fabs(x) < 7.85398163397448278999e-01) return tog__ksin(x);
  double r;
  const int q = tog__rem_pio2(x, &r);
  switch (q) {
    case 0: return tog__ksin(r);
    case 1: return tog__kcos(r);
    case 2: return -tog__ksin(r);
    default: return -tog__kcos(r);
  }
}

TOG_HD double tog_cos(double x) {
  if (!isfinite(x)) return x - x;
  if (fabs(x) < 7.85398163397448278999e-01) return tog__kcos(x);
  double r;
  const int q = tog__rem_pio2(x, &r);
  switch (q) {
    case 0: return tog__kcos(r);
    case 1: return -tog__ksin(r);
    case 2: return -tog__kcos(r);
    default: return tog__ksin(r);
  }
}

/* x / 6, correctly rounded, without the division sequence (the RK3 and RK4 steps end with one per state
 * entry, src/integration.jl:122,157): Markstein's correction -- q0 = RN(x r) with r = RN(1/6) is faithful,
 * the remainder x - 6 q0 is exact under fma, and RN(q0 + (x - 6 q0) r) is RN(x / 6). Equal to x / 6.0 bit
 * for bit on every x with 2^-1000 <= |x| <= DBL_MAX (tests/test_math_contract.py checks 4e8 values); zeros,
 * the subnormal range, infinities and NaN take the division. */
TOG_HD double tog_div6(double x) {
  const double r = 0.16666666666666666;
  const double q0 = x * r;
  const double e = fma(-q0, 6.0, x);
  const double q = fma(e, r, q0);
  const double ax = fabs(x);
  if (__builtin_expect(!(ax >= 0x1p-1000 && ax <= 1.7976931348623157e308), 0)) return x / 6.0;
  return q;
}

/* (tog_sin(x), tog_cos(x)) from one reduction and one evaluation of each kernel polynomial, branch-free:
 * bit-identical to the two calls (the same operations; the quadrant only selects and negates, which is
 * exact). The reduction runs on 0 for non-finite x (a NaN or infinite fn must not reach the integer
 * conversion) and its result is then discarded. Used where both are needed (the Kuka joints, and
 * every dual sin/cos, whose partials need the other function). */
TOG_HD void tog_sincos(double x, double* s, double* c) {
  const int fin = isfinite(x);
  double r;
  int q = tog__rem_pio2(fin ? x : 0.0, &r);
  if (fabs(x) < 7.85398163397448278999e-01) {
    r = x;
    q = 0;
  }
  const double ks = tog__ksin(r), kc = tog__kcos(r);
  const double s0 = (q & 1) ? kc : ks, c0 = (q & 1) ? ks : kc;
  const double sv = (q & 2) ? -s0 : s0, cv = ((q + 1) & 2) ? -c0 : c0;
  *s = fin ? sv : x - x;
  *c = fin ? cv : x - x;
}

/* Julia's max/min on floats (Base.max, Base.min): NaN in either argument propagates, unlike C's
 * fmax/fmin, which drop it. The AL bookkeeping uses them where the reference calls max/min/maximum/
 * norm(., Inf) (augmented_lagrangian_methods.jl:107-118, 171-184), so a NaN constraint value is
 * reported as a NaN violation on both sides instead of reading as feasible. */
/* 1/sqrt(y) of the rank-1 Cholesky downdates in the square-root backward pass (chol_minus,
 * contract v4): a bit-pattern seed (relative error below 3.5e-2) and four Newton
 * steps r += r (1/2 - (y/2) r^2) in fma form, so host and device produce the same bits; within 2 ulp
 * of the correctly rounded value for every normal y > 0 (tests/test_reference_kats.py checks 2^20
 * points). y == 0 gives +Inf, y == +Inf gives 0, y < 0 or NaN gives NaN. One long dependent chain replaces the sqrt
 * and the division of the reference's c = sqrt(1 - s^2), (.)/c. */
TOG_HD double tog_rsqrt(double y) {
  long long i;
  double r;
  __builtin_memcpy(&i, &y, sizeof(i));
  i = 0x5FE6EB50C7B537A9LL - (i >> 1);
  __builtin_memcpy(&r, &i, sizeof(r));
  const double h = 0.5 * y;
  for (int k = 0; k < 4; k++) {
    const double hr = h * r;
    const double e = fma(-hr, r, 0.5);
    r = fma(r, e, r);
  }
  return (y > 0.0 && y < INFINITY) ? r : ((y == 0.0) ? INFINITY : ((y == INFINITY) ? 0.0 : NAN));
}

/* c = sqrt(y) of chol_minus as y * tog_rsqrt(y), with the reference's c = sqrt(0) = 0 at y == 0
 * (s^2 == 1 exactly; y * rsqrt(y) would be 0 * Inf = NaN there). The reciprocal stays Inf. */
TOG_HD double tog_rs_c(double y, double rc) { return (y == 0.0) ? 0.0 : y * rc; }

TOG_HD double tog_jlmax(double a, double b) { return (a != a) ? a : ((b != b) ? b : fmax(a, b)); }
TOG_HD double tog_jlmin(double a, double b) { return (a != a) ? a : ((b != b) ? b : fmin(a, b)); }

#endif /* TOG_MATH_H */
