// tog_cost_plugin.hpp — GenericCost(ℓ, ℓf, n, m) (src/cost.jl:239-322) as a libtog cost plugin.
//
//   #include "tog_cost_plugin.hpp"
//   struct MyCost {
//     static constexpr int n = 2, m = 1;
//     template <class T> __host__ __device__ static T stage(const T* x, const T* u) { ... }   // ℓ(x, u)
//     template <class T> __host__ __device__ static T terminal(const T* x) { ... }            // ℓf(xN)
//   };
//   TOG_COST_PLUGIN(MyCost)
//
// The expansion is ForwardDiff's (auto_expansion_function, src/cost.jl:289-322): gradient and Hessian
// of ℓ over z = [x; u] (of ℓf over xN). ForwardDiff.hessian is the Jacobian of the gradient, i.e. a
// gradient dual whose value and partials are themselves duals in one Jacobian direction j
// (Dual{Tg}(Dual{Tj}, Partials{Dual{Tj}})); HDual<W> is that number with W gradient partials:
//   v, t      : value and its j-derivative                      (the Dual{Tj} value)
//   g[i], h[i]: ∂/∂z_i and ∂²/∂z_i∂z_j                            (the Dual{Tj} partials)
// Each lane of k_generic_cost evaluates ℓ once in HDual<n+m> for one (point, j) and writes Hessian
// column j; lane j = 0 also writes ℓ and the gradient. The product and quotient rules are ForwardDiff's
// (dual.jl: x*y -> (xv*yv, xp*yv + yp*xv); x/y -> (xv/yv, xp*inv(yv) + yp*(-(xv/(yv*yv))))) applied at
// both levels, with the inner level in the Dual<1> arithmetic of tog_device.hpp (r.g = fma(b.v, a.g,
// a.v*b.g)); oracle/tog_oracle_cost.c restates the same operations, so device and oracle agree bit for bit.
//
// GenericCost(ℓ, ℓf, grad, hess, n, m) (src/cost.jl:260-268, analytic derivatives): a cost struct with
// `static constexpr bool has_expansion = true` and
//   static void expansion(double* Q, double* R, double* H, double* q, double* r, const double* x, const double* u)
//   static void expansion_term(double* Qf, double* qf, const double* x)
// (column-major Q (n,n), R (m,m), H (m,n)) is evaluated as written, one lane per point.
#pragma once

#include <hip/hip_runtime.h>

#include "tog_device.hpp"

namespace tog {

template <int W>
struct HDual {
  double v, t;
  double g[W], h[W];
};

template <int W>
__host__ __device__ __forceinline__ double val_(const HDual<W>& a) { return a.v; }

template <int W>
__host__ __device__ __forceinline__ HDual<W> hconst(double v) {
  HDual<W> r;
  r.v = v;
  r.t = 0.0;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = r.h[i] = 0.0;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> cst_(double x, const HDual<W>&) { return hconst<W>(x); }

// Dual<1> helpers of the inner level: (a, at) op (b, bt)
struct D1 {
  double v, t;
};
__host__ __device__ __forceinline__ D1 d1_mul(D1 a, D1 b) { return {a.v * b.v, fma(b.v, a.t, a.v * b.t)}; }
__host__ __device__ __forceinline__ D1 d1_add(D1 a, D1 b) { return {a.v + b.v, a.t + b.t}; }
__host__ __device__ __forceinline__ D1 d1_inv(D1 a) {  // inv(x) -> (1/xv, -(1/(xv*xv)) xp)
  const double c = -(1.0 / (a.v * a.v));
  return {1.0 / a.v, c * a.t};
}
__host__ __device__ __forceinline__ D1 d1_div(D1 a, D1 b) {
  const double iy = 1.0 / b.v, c2 = -(a.v / (b.v * b.v));
  return {a.v / b.v, fma(a.t, iy, b.t * c2)};
}
__host__ __device__ __forceinline__ D1 d1_neg(D1 a) { return {-a.v, -a.t}; }

template <int W>
__host__ __device__ __forceinline__ HDual<W> operator+(const HDual<W>& a, const HDual<W>& b) {
  HDual<W> r;
  r.v = a.v + b.v;
  r.t = a.t + b.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = a.g[i] + b.g[i];
    r.h[i] = a.h[i] + b.h[i];
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator-(const HDual<W>& a, const HDual<W>& b) {
  HDual<W> r;
  r.v = a.v - b.v;
  r.t = a.t - b.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = a.g[i] - b.g[i];
    r.h[i] = a.h[i] - b.h[i];
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator-(const HDual<W>& a) {
  HDual<W> r;
  r.v = -a.v;
  r.t = -a.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = -a.g[i];
    r.h[i] = -a.h[i];
  }
  return r;
}
// x*y -> value xv*yv, partial i: xp_i*yv + yp_i*xv (both in Dual<1> arithmetic)
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator*(const HDual<W>& a, const HDual<W>& b) {
  HDual<W> r;
  const D1 av{a.v, a.t}, bv{b.v, b.t};
  const D1 rv = d1_mul(av, bv);
  r.v = rv.v;
  r.t = rv.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const D1 p = d1_add(d1_mul(D1{a.g[i], a.h[i]}, bv), d1_mul(D1{b.g[i], b.h[i]}, av));
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
// a constant is a dual with zero partials at both levels; products with it keep ForwardDiff's
// scalar rule (x*s -> (xv*s, xp*s))
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator*(const HDual<W>& a, double s) {
  HDual<W> r;
  r.v = a.v * s;
  r.t = a.t * s;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = a.g[i] * s;
    r.h[i] = a.h[i] * s;
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator*(double s, const HDual<W>& a) {
  HDual<W> r;
  r.v = s * a.v;
  r.t = s * a.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = s * a.g[i];
    r.h[i] = s * a.h[i];
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator/(const HDual<W>& a, double s) {
  HDual<W> r;
  r.v = a.v / s;
  r.t = a.t / s;
#pragma unroll
  for (int i = 0; i < W; i++) {
    r.g[i] = a.g[i] / s;
    r.h[i] = a.h[i] / s;
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator+(const HDual<W>& a, double s) {
  HDual<W> r = a;
  r.v = a.v + s;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator+(double s, const HDual<W>& a) {
  HDual<W> r = a;
  r.v = s + a.v;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator-(const HDual<W>& a, double s) {
  HDual<W> r = a;
  r.v = a.v - s;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator-(double s, const HDual<W>& a) {
  return hconst<W>(s) - a;
}
// x/y -> value xv/yv, partial i: xp_i*inv(yv) + yp_i*(-(xv/(yv*yv)))
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator/(const HDual<W>& a, const HDual<W>& b) {
  HDual<W> r;
  const D1 av{a.v, a.t}, bv{b.v, b.t};
  const D1 iy = d1_inv(bv);
  const D1 c2 = d1_neg(d1_div(av, d1_mul(bv, bv)));
  const D1 rv = d1_div(av, bv);
  r.v = rv.v;
  r.t = rv.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const D1 p = d1_add(d1_mul(D1{a.g[i], a.h[i]}, iy), d1_mul(D1{b.g[i], b.h[i]}, c2));
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> operator/(double s, const HDual<W>& b) {
  return hconst<W>(s) / b;
}
// unary rules f(x) -> (f(xv), f'(xv) xp) with f(xv), f'(xv) evaluated in Dual<1>
template <int W>
__host__ __device__ __forceinline__ HDual<W> hunary(const HDual<W>& a, D1 fv, D1 dfv) {
  HDual<W> r;
  r.v = fv.v;
  r.t = fv.t;
#pragma unroll
  for (int i = 0; i < W; i++) {
    const D1 p = d1_mul(dfv, D1{a.g[i], a.h[i]});
    r.g[i] = p.v;
    r.h[i] = p.t;
  }
  return r;
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> sin_(const HDual<W>& a) {
  double s, c;
  tog_sincos(a.v, &s, &c);
  return hunary(a, D1{s, c * a.t}, D1{c, (-s) * a.t});
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> cos_(const HDual<W>& a) {
  double s, c;
  tog_sincos(a.v, &s, &c);
  return hunary(a, D1{c, (-s) * a.t}, D1{-s, (-c) * a.t});
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> sqrt_(const HDual<W>& a) {
  const double sv = sqrt(a.v);
  const D1 f{sv, (1.0 / (2.0 * sv)) * a.t};        // sqrt(Dual<1>)
  const D1 df = d1_inv(d1_mul(D1{2.0, 0.0}, f));   // 1 / (2 sqrt(x)) in Dual<1>
  return hunary(a, f, df);
}
template <int W>
__host__ __device__ __forceinline__ HDual<W> inv_(const HDual<W>& a) {
  return hconst<W>(1.0) / a;
}

template <class C, class = void>
struct has_expansion : std::false_type {};
template <class C>
struct has_expansion<C, std::void_t<decltype(C::has_expansion)>> : std::integral_constant<bool, C::has_expansion> {};

// One lane per (point, Hessian column j). Outputs (column-major, count points): J (count), Ex (n),
// Eu (m), Exx (n, n), Euu (m, m), Eux (m, n); the terminal expansion writes only J, Ex, Exx.
template <class COST, bool TERM>
__global__ void __launch_bounds__(256) k_generic_cost(const double* __restrict__ X, const double* __restrict__ U,
                                                      long long count, double* J, double* Ex, double* Eu,
                                                      double* Exx, double* Euu, double* Eux) {
  constexpr int n = COST::n, m = COST::m;
  constexpr int W = TERM ? n : n + m;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= count * W) return;
  const long long p = gid / W;
  const int j = (int)(gid - p * W);
  HDual<W> z[W];
#pragma unroll
  for (int i = 0; i < W; i++) {
    z[i] = hconst<W>(i < n ? X[p * n + i] : U[p * m + (i - n)]);
    z[i].g[i] = 1.0;
  }
  z[j].t = 1.0;
  HDual<W> l;
  if constexpr (TERM)
    l = COST::terminal(z);
  else
    l = COST::stage(z, z + n);
  if (j == 0) {
    J[p] = l.v;
#pragma unroll
    for (int i = 0; i < n; i++) Ex[p * n + i] = l.g[i];
    if constexpr (!TERM) {
#pragma unroll
      for (int i = 0; i < m; i++) Eu[p * m + i] = l.g[n + i];
    }
  }
  if (j < n) {
#pragma unroll
    for (int i = 0; i < n; i++) Exx[p * n * n + i + n * j] = l.h[i];  // hess[xinds, xinds]
    if constexpr (!TERM) {
#pragma unroll
      for (int i = 0; i < m; i++) Eux[p * m * n + i + m * j] = l.h[n + i];  // hess[uinds, xinds]
    }
  } else if constexpr (!TERM) {
#pragma unroll
    for (int i = 0; i < m; i++) Euu[p * m * m + i + m * (j - n)] = l.h[n + i];  // hess[uinds, uinds]
  }
}

// GenericCost(ℓ, ℓf, grad, hess, n, m): the user's analytic expansion, one lane per point
template <class COST, bool TERM>
__global__ void __launch_bounds__(256) k_generic_cost_analytic(const double* __restrict__ X,
                                                               const double* __restrict__ U, long long count,
                                                               double* J, double* Ex, double* Eu, double* Exx,
                                                               double* Euu, double* Eux) {
  constexpr int n = COST::n, m = COST::m;
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= count) return;
  double x[n], u[m];
#pragma unroll
  for (int i = 0; i < n; i++) x[i] = X[p * n + i];
  if constexpr (TERM) {
    J[p] = COST::terminal(x);
    COST::expansion_term(Exx + p * n * n, Ex + p * n, x);
  } else {
#pragma unroll
    for (int i = 0; i < m; i++) u[i] = U[p * m + i];
    J[p] = COST::stage(x, u);
    COST::expansion(Exx + p * n * n, Euu + p * m * m, Eux + p * m * n, Ex + p * n, Eu + p * m, x, u);
  }
}

template <class COST>
int generic_cost_launch(int terminal, const double* X, const double* U, long long count, double* J, double* Ex,
                        double* Eu, double* Exx, double* Euu, double* Eux, hipStream_t s) {
  constexpr int n = COST::n, m = COST::m;
  if (count <= 0) return 0;
  const long long lanes = has_expansion<COST>::value ? count : count * (terminal ? n : n + m);
  const unsigned grid = (unsigned)((lanes + 255) / 256);
  if constexpr (has_expansion<COST>::value) {
    if (terminal)
      k_generic_cost_analytic<COST, true><<<grid, 256, 0, s>>>(X, U, count, J, Ex, Eu, Exx, Euu, Eux);
    else
      k_generic_cost_analytic<COST, false><<<grid, 256, 0, s>>>(X, U, count, J, Ex, Eu, Exx, Euu, Eux);
  } else {
    if (terminal)
      k_generic_cost<COST, true><<<grid, 256, 0, s>>>(X, U, count, J, Ex, Eu, Exx, Euu, Eux);
    else
      k_generic_cost<COST, false><<<grid, 256, 0, s>>>(X, U, count, J, Ex, Eu, Exx, Euu, Eux);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// (TOG_HEADER_HASH: the build's hash of every libtog header's text, tog_plugin.hpp)
constexpr long long cost_plugin_fingerprint() {
  return (0x7c057LL * 1000003LL + (long long)sizeof(HDual<3>)) ^ (long long)TOG_HEADER_HASH;
}

}  // namespace tog

#define TOG_COST_PLUGIN(COST)                                                                             \
  static_assert(COST::n >= 1 && COST::m >= 1 && COST::n + COST::m <= 32, "cost plugin: n + m <= 32");   \
  extern "C" long long tog_cost_plugin_fingerprint() { return tog::cost_plugin_fingerprint(); }           \
  extern "C" int tog_cost_plugin_dims(int* n, int* m) {                                                   \
    *n = COST::n;                                                                                         \
    *m = COST::m;                                                                                         \
    return 0;                                                                                             \
  }                                                                                                       \
  extern "C" int tog_cost_plugin_expand(int terminal, const double* X, const double* U, long long count,  \
                                        double* J, double* Ex, double* Eu, double* Exx, double* Euu,      \
                                        double* Eux, void* stream) {                                      \
    return tog::generic_cost_launch<COST>(terminal, X, U, count, J, Ex, Eu, Exx, Euu, Eux,               \
                                          (hipStream_t)stream);                                           \
  }
