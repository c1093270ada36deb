// tog_device.hpp — device-side data model and numerics shared by every HIP kernel.
//
// Reference: TrajectoryOptimization.jl (file:line citations are relative to /root/reference).
// Everything here is fp64. Models are written once, templated on the scalar type, so the same
// code evaluates the primal discrete dynamics (rollouts) and the ForwardDiff-equivalent dual
// number Jacobians (src/model.jl:491-522).
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/tog.h"
#include "../../include/tog_math.h"
#include "../../include/tog_kuka.h"

// Hash of the text of every libtog header (the Makefile's HDRS, in order; abi.header_hash() computes
// the same value for plugins generated at run time). libtog and every plugin are compiled with it and
// the plugin fingerprints include it, so tog_model_load / tog_generic_cost_load refuse a plugin built
// against other headers.
#ifndef TOG_HEADER_HASH
#define TOG_HEADER_HASH 0LL
#endif

namespace tog {

constexpr int NMAX = 16;  // max states (Kuka n=14)
constexpr int MMAX = 32;  // max controls (an infeasible problem adds n slack controls)

// ---------------------------------------------------------------------------------------------
// Constraint rows. A ConstraintSet (src/constraint_sets.jl) is flattened on the host into rows in
// the order of the reference's constraint vector C[k] (labels in insertion order; BoundConstraint
// parts [x_max; u_max; x_min; u_min] with infinite bounds trimmed, src/constraints.jl:155-188).
enum RowType : int {
  ROW_XMAX = 0,  // c = x[i] - a            (inequality)
  ROW_UMAX = 1,  // c = u[i] - a
  ROW_XMIN = 2,  // c = a - x[i]
  ROW_UMIN = 3,  // c = a - u[i]
  ROW_GOAL = 4,  // c = x[i] - a            (equality, goal_constraint src/constraints.jl:299-304)
  ROW_CIRCLE = 5,  // c = -((x1-a)^2 + (x2-b)^2 - r^2)            src/utils.jl:140-144
  ROW_SPHERE = 6,  // c = -((x1-a)^2 + (x2-b)^2 + (x3-c)^2 - r^2)  src/utils.jl:150-156
  ROW_USLACK = 7,  // c = u[i]  (equality; infeasible_constraints, src/constraints.jl:306-314)
  // Constraint{S}(c!, n, m, p) with a user function (src/constraints.jl:85-89, Jacobian by ForwardDiff):
  // row idx of the plugin model's con(fid = a, c, x, u) (p = b outputs)
  ROW_USER_INEQ = 8,
  ROW_USER_EQ = 9,
  ROW_MT_EQ = 10  // c = u[a] - x[idx] (equality; mintime_equality, src/solvers/altro/minimum_time.jl:106-124)
};
constexpr int PUSER = 16;  // max outputs of one user constraint function

struct ConRow {
  int type;
  int idx;
  double a, b, c, r;
};

// Problem description resident in device memory (read through uniform scalar loads).
struct DevProblem {
  int n, m, N, pmax;
  int model, integ, nrows, pad0;
  long long B;
  double dt;
  double Q[NMAX * NMAX], R[MMAX * MMAX], H[MMAX * NMAX], q[NMAX], r[MMAX], c;
  double Qf[NMAX * NMAX], qf[NMAX], cf;
  // upper Cholesky factors for the square-root expansion (src/objective.jl:70-94):
  // cholesky(Q*dt).U, cholesky(R*dt).U, cholesky(Qf).U — identical at every knot, factored once.
  double cQ[NMAX * NMAX], cR[MMAX * MMAX], cQf[NMAX * NMAX];
  int sqrt_ok;  // 0 if one of the Hessians is not PD (reference: error(...))
  // structure flags: Q, R, Qf diagonal and H == 0. The dense fma loops then only ever add exact
  // zeros off the diagonal, so the diagonal fast paths are bit-identical to them.
  int diag_cost;  // 0 dense; 1 diagonal Q/R/Qf, H = 0; 2 = 1 with +0.0 off-diagonals (literal zeros)
  int pad1;
  double R_min_time;  // MinTimeCost weight (minimum-time problems; Q, R, H, q, r, Qf, qf are the base
                      // cost's, zero-padded to the augmented sizes)
  // a time-varying Objective (tog_problem_desc.stage_costs): per stage knot [Q; R; H; q; r; c; cQ; cR]
  // (compact n, m; cQ, cR the square-root expansion's factors), or null (the fields above at every knot)
  const double* kc;
  int kc_stride, kc_pad;
  // the Q.xx entries any stage row can change in the std AL expansion (k_expand_team's pattern loop): the
  // union over rows of (state gradient indices)^2, by column: qpat[c] a bit per row i of column c, qoff[c]
  // its running count. qpat_on = 0: the general loop.
  int qpat_on, qpat_n;
  unsigned int qpat[NMAX];
  int qoff[NMAX];
  int qpat_max, qpat_pad;  // the most pattern entries in one column
  const int* knot_off;  // [N] first row of knot k
  const int* knot_cnt;  // [N] rows at knot k (p_k)
  const ConRow* rows;
  const int* knot_nx;   // [N] rows with a state gradient at knot k (expansion records, ne_of)
  tog_options o;
};

// Read-only device tables seen through the constant address space. The row tables are read at the
// same (knot, row) by every lane of a wave, so through these pointers a read is a scalar load
// (lgkmcnt only). Through the generic pointers of DevProblem it is a flat load, whose wait also
// drains every outstanding global load and store of the wave: in the rollouts that exposed a full
// memory round trip per row and knot (k_ls_spec at B = 1: 6 µs per knot).
template <class T>
using cptr = const T __attribute__((address_space(4)))*;
template <class T>
__device__ __forceinline__ cptr<T> as_const(const T* p) {
  return (cptr<T>)p;
}
// The same data through the global address space: a lane-indexed read is a global load (vmcnt only, not the
// flat load of a generic pointer), and, unlike the constant address space, the loads are not marked
// invariant, so they are not hoisted out of a knot loop into long-lived registers.
template <class T>
using gptr = const T __attribute__((address_space(1)))*;
template <class T>
__device__ __forceinline__ gptr<T> as_global(const T* p) {
  return (gptr<T>)p;
}
__device__ __forceinline__ cptr<ConRow> knot_rows(const DevProblem* P, int k) {
  return as_const(P->rows) + as_const(P->knot_off)[k];
}
__device__ __forceinline__ int knot_count(const DevProblem* P, int k) { return as_const(P->knot_cnt)[k]; }
// a row read through either pointer kind (member-wise for the constant address space: the implicit
// copy constructor takes a generic reference)
__device__ __forceinline__ ConRow load_row(cptr<ConRow> p) {
  ConRow r;
  r.type = p->type;
  r.idx = p->idx;
  r.a = p->a;
  r.b = p->b;
  r.c = p->c;
  r.r = p->r;
  return r;
}
__device__ __forceinline__ ConRow load_row(const ConRow* p) { return *p; }

// Per-trajectory solver state (the scalar fields of iLQRSolver/AugmentedLagrangianSolver and
// their stats dicts, ilqr_solver.jl:93-154, augmented_lagrangian_solver.jl:101-140).
struct TrajState {
  double rho, drho;          // ρ, dρ
  double J;                  // J_prev of the inner loop (cost of the current X, U)
  double dJ, grad, alpha, z, expected;
  double dV0, dV1;           // ΔV of the last backward pass
  double c_max, mu_max;
  double cost_tol, grad_tol; // current inner tolerances (set_tolerances!, :39-50)
  int iters, zero_cnt, al_iter, total_steps, ls_trials, bp_restarts, flags, active;
  // line search carried over to the next batch step (k_ls_decide, pending mode): the trials [0, ls_pend)
  // are evaluated and stored; the trajectory skips that step's Jacobians and backward pass
  int ls_pend, pad_;
  // records written to the iteration histories (DevBuffers::hist_in / hist_out; counted past the
  // capacity, so a truncated history is visible)
  int hn_in, hn_out;
};

// the regularisation scalars the backward pass mutates (kept in registers)
struct RegState {
  double rho, drho;
  int flags;
};

struct DevBuffers {
  double* x0;   // (n, B)
  double* X;    // (n, N, B)
  double* U;    // (m, N-1, B)
  double* Xb;   // X̄
  double* Ub;   // Ū
  double* AB;   // (n, n+m, N-1, B)  [A | B] per knot, column-major
  double* K;    // (m, n, N-1, B)
  double* d;    // (m, N-1, B)
  double* lam;  // (pmax, N, B)
  double* mu;   // (pmax, N, B)
  double* C;    // (pmax, N, B)
  double* Sdbg; // (n, n, N, B) or null
  double* sdbg; // (n, N, B) or null
  double* Qscr; // (nq, N, B) accumulated Q blocks for the restart replay path
  double* E;    // (ne, N, B) expansion records of k_expand_team (tog_bwd_team.hpp ne_of), or null
  double* lsJ;  // (NC, B) speculative line-search trial costs
  int* lsok;    // (NC, B) speculative line-search trial rollout status
  int nc;       // candidates evaluated per trajectory per launch (<= 64)
  int* ls_list;   // (2, B) ping-pong lists of trajectories still undecided after a speculative round
  int* ls_done;   // = ls_list + B: the trajectories whose inner solve finished this step (k_ls_book -> k_al_outer)
  int* ls_count;  // [LS_COUNT_SLOTS] list lengths, zeroed at the start of every forward pass
  int* ls_fb;     // (B) trajectories whose line search ran out of trials (k_ls_fallback), or null
  int bwd_stride;     // k_bwd_team: per-team LDS stride (doubles) of the launch
  int bwd_shmem;      // k_bwd_team: dynamic LDS bytes per block of the launch
  int bwd_stride2[2]; // [std, sqrt] strides
  int bwd_shmem2[2];  // [std, sqrt] LDS bytes
  int spec_tail_shmem; // LDS bytes of k_ls_spec_tail's chunk image (0: the tail uses k_ls_spec)
  int spec_tail2_shmem; // LDS bytes of k_ls_spec_tail2 (two staging images + the ring; 0: not admissible)
  int cost_diag;       // DevProblem::diag_cost (host copy: kernel variants that inline the diagonal cost)
  int tv;              // a time-varying Objective (DevProblem::kc): the team backward kernels' per-knot-cost variants
  int rows_lds;        // LDS bytes of a block's copy of the row tables (bulk k_ls_spec; 0: global tables)
  int ls_first;       // width of the first speculative round (>= nc: one round)
  int nknots;         // N (host-side launch geometry)
  int ls_pend_ok;     // solve steps may carry an undecided line search over to the next step
  double* cand;       // (NCP, n+m, N, B) every trial's rollout (candidate-copy line search), or null
  int ncp;            // candidate slots per element (nc rounded up to 8)
  int tail;           // few trajectories active (last host readback): latency-sized backward kernels
  int simds;          // SIMDs of the device (CUs x 4): a team backward of at most this many waves runs WPE = 1
  int* ls_win;        // (B) accepted trial of the current forward pass (k_ls_decide)
  double* ls_Jw;      // (B) its cost
  double* gk;         // (N, B) per-knot todorov gradient terms of the accepted Ū
  double* jws;        // Kuka RK3 Jacobian workspace (stage-chain form: KJ_WSK doubles per knot slot; the
                      // dual-staged A/B form: 2n duals per lane), or null
  int jac_chain;      // Kuka RK3 Jacobian in stage-chain form (tog_kuka_jac.hpp; 0: TOG_KUKA_JAC=dual A/B)
  int dense_stage_knots;  // some stage knot has a state-gradient row (k_expand_u / k_expand_team split)
  // compacted tail launches (tog_solve_step, k_list_active): the step's active trajectories and their
  // count; null outside a tail step (launch slot = trajectory index)
  int* act_list;
  int* act_count;
  TrajState* st;
  // per-trajectory iteration histories (tog_history_enable; null = off): the iLQR solver's
  // stats[:cost], [:dJ], [:gradient] (record_iteration!, ilqr_methods.jl:77-89) as hist_in (3, hcap, B),
  // and the AL solver's stats[:iterations_inner], [:cost], [:c_max], [:penalty_max]
  // (augmented_lagrangian_methods.jl:79-97) as hist_out (4, ocap, B)
  double* hist_in;
  double* hist_out;
  int hcap, ocap;
};

// iLQR record_iteration! (ilqr_methods.jl:77-89): one (J, dJ, gradient) record
__device__ __forceinline__ void hist_inner(const DevBuffers& Bf, long long b, TrajState& s, double J, double dJ,
                                           double g) {
  if (!Bf.hist_in) return;
  if (s.hn_in < Bf.hcap) {
    double* h = Bf.hist_in + ((size_t)b * Bf.hcap + s.hn_in) * 3;
    h[0] = J;
    h[1] = dJ;
    h[2] = g;
  }
  s.hn_in++;
}
// AL record_iteration! (augmented_lagrangian_methods.jl:79-97): (iterations_inner, cost, c_max, penalty_max)
__device__ __forceinline__ void hist_outer(const DevBuffers& Bf, long long b, TrajState& s, int inner, double J,
                                           double c_max, double mu_max) {
  if (!Bf.hist_out) return;
  if (s.hn_out < Bf.ocap) {
    double* h = Bf.hist_out + ((size_t)b * Bf.ocap + s.hn_out) * 4;
    h[0] = (double)inner;
    h[1] = J;
    h[2] = c_max;
    h[3] = mu_max;
  }
  s.hn_out++;
}

// ---------------------------------------------------------------------------------------------
// Scalar helpers (double and Dual share names)
__host__ __device__ __forceinline__ double sin_(double x) { return tog_sin(x); }
__host__ __device__ __forceinline__ double cos_(double x) { return tog_cos(x); }
__host__ __device__ __forceinline__ void sincos_(double x, double& s, double& c) { tog_sincos(x, &s, &c); }
__host__ __device__ __forceinline__ double div6_(double x) { return tog_div6(x); }
__host__ __device__ __forceinline__ double sqrt_(double x) { return sqrt(x); }
__host__ __device__ __forceinline__ double inv_(double x) { return 1.0 / x; }
__host__ __device__ __forceinline__ double val_(double x) { return x; }
__host__ __device__ __forceinline__ double cst_(double x, double) { return x; }

// ForwardDiff.Dual with W partials (Manifest.toml:164-168, ForwardDiff v0.10.3 dual.jl):
//   x*y -> (xv*yv, yv*x.p + xv*y.p);  x/y -> (xv/yv, x.p*inv(yv) + y.p*(-(xv/(yv*yv))))
template <int W>
struct Dual {
  double v;
  double g[W];
};

template <int W>
__host__ __device__ __forceinline__ double val_(const Dual<W>& a) { return a.v; }

template <int W>
__host__ __device__ __forceinline__ Dual<W> dconst(double v) {
  Dual<W> r;
  r.v = v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = 0.0;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> cst_(double x, const Dual<W>&) { return dconst<W>(x); }

template <int W>
__host__ __device__ __forceinline__ Dual<W> operator+(const Dual<W>& a, const Dual<W>& b) {
  Dual<W> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = a.g[i] + b.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator-(const Dual<W>& a, const Dual<W>& b) {
  Dual<W> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = a.g[i] - b.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator-(const Dual<W>& a) {
  Dual<W> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = -a.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator*(const Dual<W>& a, const Dual<W>& b) {
  Dual<W> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = fma(b.v, a.g[i], a.v * b.g[i]);
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator*(double s, const Dual<W>& a) {
  Dual<W> r;
  r.v = s * a.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = s * a.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator*(const Dual<W>& a, double s) {
  Dual<W> r;
  r.v = a.v * s;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = a.g[i] * s;
  return r;
}
// (the dual form keeps the division: tog_div6's per-component range branch measured slower in the
// Jacobian kernels -- quadrotor 0.87 -> 1.39 ms -- and both give the same bits)
template <int W>
__host__ __device__ __forceinline__ Dual<W> div6_(const Dual<W>& a) {
  return a / 6.0;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator/(const Dual<W>& a, double s) {
  Dual<W> r;
  r.v = a.v / s;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = a.g[i] / s;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator+(const Dual<W>& a, double s) {
  Dual<W> r = a;
  r.v = a.v + s;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator+(double s, const Dual<W>& a) {
  Dual<W> r = a;
  r.v = s + a.v;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator-(const Dual<W>& a, double s) {
  Dual<W> r = a;
  r.v = a.v - s;
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator-(double s, const Dual<W>& a) {  // a zero-tangent dual minus a
  Dual<W> r;
  r.v = s - a.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = -a.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> operator/(const Dual<W>& a, const Dual<W>& b) {
  Dual<W> r;
  const double iy = 1.0 / b.v, c2 = -(a.v / (b.v * b.v));
  r.v = a.v / b.v;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = fma(a.g[i], iy, b.g[i] * c2);
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> inv_(const Dual<W>& a) {
  Dual<W> r;
  r.v = 1.0 / a.v;
  const double c = -(1.0 / (a.v * a.v));
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = c * a.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> sin_(const Dual<W>& a) {
  Dual<W> r;
  double c;
  tog_sincos(a.v, &r.v, &c);
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = c * a.g[i];
  return r;
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> cos_(const Dual<W>& a) {
  Dual<W> r;
  double sv;
  tog_sincos(a.v, &sv, &r.v);
  const double c = -sv;
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = c * a.g[i];
  return r;
}
// (sin_(a), cos_(a)) from one tog_sincos (bit-identical to the two calls)
template <int W>
__host__ __device__ __forceinline__ void sincos_(const Dual<W>& a, Dual<W>& s, Dual<W>& c) {
  double sv, cv;
  tog_sincos(a.v, &sv, &cv);
  const double ns = -sv;
  s.v = sv;
  c.v = cv;
#pragma unroll
  for (int i = 0; i < W; i++) {
    s.g[i] = cv * a.g[i];
    c.g[i] = ns * a.g[i];
  }
}
template <int W>
__host__ __device__ __forceinline__ Dual<W> sqrt_(const Dual<W>& a) {
  Dual<W> r;
  r.v = sqrt(a.v);
  const double c = 1.0 / (2.0 * r.v);
#pragma unroll
  for (int i = 0; i < W; i++) r.g[i] = c * a.g[i];
  return r;
}

// ---------------------------------------------------------------------------------------------
// Continuous dynamics  ẋ = f(x, u)  

struct DoubleIntegrator {  // dynamics/double_integrator.jl:1-4
  static constexpr int n = 2, m = 1, id = TOG_MODEL_DOUBLE_INTEGRATOR;
  template <class T>
  __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    xd[0] = x[1];
    xd[1] = u[0];
  }
};

struct Pendulum {  // dynamics/pendulum.jl:3-12
  static constexpr int n = 2, m = 1, id = TOG_MODEL_PENDULUM;
  template <class T>
  __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const double mm = 1.0, b = 0.1, lc = 0.5, I = 0.25, g = 9.81;
    xd[0] = x[1];
    xd[1] = ((u[0] - (mm * g * lc) * sin_(x[0])) - b * x[1]) / I;
  }
};

struct Car {  // dynamics/car.jl:3-8
  static constexpr int n = 3, m = 2, id = TOG_MODEL_CAR;
  template <class T>
  __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    T s, c;
    sincos_(x[2], s, c);
    xd[0] = u[0] * c;
    xd[1] = u[0] * s;
    xd[2] = u[1];
  }
};

struct Cartpole {  // dynamics/cartpole.jl:9-36 ; qdd = -H \ (C*qd + G - B*u), generic 2x2 LU
  static constexpr int n = 4, m = 1, id = TOG_MODEL_CARTPOLE;
  template <class T>
  __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const double mc = 1.0, mp = 0.2, l = 0.5, g = 9.81;
    T s, c;
    if (isfinite(val_(x[1]))) {
      sincos_(x[1], s, c);
    } else {  // cartpole.jl:18-24
      s = cst_(INFINITY, x[1]);
      c = cst_(INFINITY, x[1]);
    }
    T a11 = cst_(mc + mp, x[0]);
    T a12 = (mp * l) * c;
    T a21 = a12;
    T a22 = cst_(mp * (l * l), x[0]);
    const T zero = cst_(0.0, x[0]);
    T C12 = ((-mp) * x[3]) * l * s;
    T b1 = ((zero * x[2] + C12 * x[3]) + zero) - u[0];
    T b2 = ((zero * x[2] + zero * x[3]) + (mp * g * l) * s) - 0.0 * u[0];
    if (fabs(val_(a21)) > fabs(val_(a11))) {  // partial pivoting
      T t = a11; a11 = a21; a21 = t;
      t = a12; a12 = a22; a22 = t;
      t = b1; b1 = b2; b2 = t;
    }
    T l21 = a21 * inv_(a11);
    T u22 = a22 - l21 * a12;
    T y2 = b2 - l21 * b1;
    T q2 = y2 / u22;
    T q1 = (b1 - a12 * q2) / a11;
    xd[0] = x[2];
    xd[1] = x[3];
    xd[2] = -q1;
    xd[3] = -q2;
  }
};

// Hamilton product a⊗b as dynamics/quaternions.jl:23-27 computes it (q2 = a, q1 = b).
template <class T>
__device__ __forceinline__ void qmul(T* r, const T* a, const T* b) {
  const T& s1 = b[0];
  const T& s2 = a[0];
  const T dot = (b[1] * a[1] + b[2] * a[2]) + b[3] * a[3];
  r[0] = s1 * s2 - dot;
  const T cx = a[2] * b[3] - a[3] * b[2];
  const T cy = a[3] * b[1] - a[1] * b[3];
  const T cz = a[1] * b[2] - a[2] * b[1];
  r[1] = (s1 * a[1] + s2 * b[1]) + cx;
  r[2] = (s1 * a[2] + s2 * b[2]) + cy;
  r[3] = (s1 * a[3] + s2 * b[3]) + cz;
}

struct Quadrotor {  // dynamics/quadrotor.jl:10-71, params :1-7
  static constexpr int n = 13, m = 4, id = TOG_MODEL_QUADROTOR;
  template <class T>
  __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const double mass = 0.5, L = 0.175, kf = 1.0, km = 0.0245;
    const double J0 = 0.0023, J1 = 0.0023, J2 = 0.004;
    const double Ji0 = 1.0 / 0.0023, Ji1 = 1.0 / 0.0023, Ji2 = 1.0 / 0.004;
    // q = normalize(x[4:7]) = inv(norm(q))*q
    const T nrm2 = ((x[3] * x[3] + x[4] * x[4]) + x[5] * x[5]) + x[6] * x[6];
    const T inrm = inv_(sqrt_(nrm2));
    T q[4];
#pragma unroll
    for (int i = 0; i < 4; i++) q[i] = inrm * x[3 + i];
    const T F1 = kf * u[0], F2 = kf * u[1], F3 = kf * u[2], F4 = kf * u[3];
    const T Fz = ((F1 + F2) + F3) + F4;
    const T M1 = km * u[0], M2 = km * u[1], M3 = km * u[2], M4 = km * u[3];
    const T tau0 = L * (F2 - F4);
    const T tau1 = L * (F3 - F1);
    const T tau2 = ((M1 - M2) + M3) - M4;
    xd[0] = x[7];
    xd[1] = x[8];
    xd[2] = x[9];
    // ẋ[4:7] = 0.5*q*Quaternion(0, ω)
    {
      T hq[4], w4[4], r[4];
#pragma unroll
      for (int i = 0; i < 4; i++) hq[i] = 0.5 * q[i];
      w4[0] = cst_(0.0, x[0]);
      w4[1] = x[10];
      w4[2] = x[11];
      w4[3] = x[12];
      qmul(r, hq, w4);
#pragma unroll
      for (int i = 0; i < 4; i++) xd[3 + i] = r[i];
    }
    // ẋ[8:10] = g + (1/m)*vec(q*Quaternion(0,F)*inv(q))
    {
      T F4q[4], t1[4], qi[4], t2[4];
      F4q[0] = cst_(0.0, x[0]);
      F4q[1] = F4q[0];
      F4q[2] = F4q[0];
      F4q[3] = Fz;
      qmul(t1, q, F4q);
      qi[0] = q[0];
      qi[1] = -q[1];
      qi[2] = -q[2];
      qi[3] = -q[3];
      qmul(t2, t1, qi);
      const double im = 1.0 / mass;
      xd[7] = 0.0 + im * t2[1];
      xd[8] = 0.0 + im * t2[2];
      xd[9] = -9.81 + im * t2[3];
    }
    // ẋ[11:13] = Jinv*(τ - ω × (Jω))
    {
      const T Jw0 = J0 * x[10], Jw1 = J1 * x[11], Jw2 = J2 * x[12];
      const T c0 = x[11] * Jw2 - x[12] * Jw1;
      const T c1 = x[12] * Jw0 - x[10] * Jw2;
      const T c2 = x[10] * Jw1 - x[11] * Jw0;
      xd[10] = Ji0 * (tau0 - c0);
      xd[11] = Ji1 * (tau1 - c1);
      xd[12] = Ji2 * (tau2 - c2);
    }
  }
};


// Kuka iiwa 7-DoF arm (BASELINE config 5): Model(urdf) src/model.jl:394-431 over RigidBodyDynamics
// v2.1.0 dynamics!: q̇ = v, v̇ = M(q)⁻¹(τ − c(q,v)), τ = I₇·u. RNEA bias (v̇ = 0, base at −g), CRBA
// mass matrix, Cholesky solve, spatial quantities in body coordinates. Tables from the reference's
// URDF (include/tog_kuka.h). Same operation sequence as the oracle's f_kuka (oracle/tog_oracle.c),
// operand for operand, so rollouts and dual Jacobians are bit-identical to it.
// Joint tables with the derived per-body inertia terms, built at compile time from include/tog_kuka.h.
struct KukaTab {
  double R0[7][9], P[7][3], M[7], H[7][3], IO[7][9];
  constexpr KukaTab() : R0{}, P{}, M{}, H{}, IO{} {
    constexpr double r0[7][9] = TOG_KUKA_R0, pp[7][3] = TOG_KUKA_P, mass[7] = TOG_KUKA_MASS,
                     com[7][3] = TOG_KUKA_COM, ic[7][6] = TOG_KUKA_IC;
    for (int j = 0; j < 7; j++) {
      for (int e = 0; e < 9; e++) R0[j][e] = r0[j][e];
      const double* c = com[j];
      const double cc = (c[0] * c[0] + c[1] * c[1]) + c[2] * c[2];
      const double icm[3][3] = {{ic[j][0], ic[j][1], ic[j][2]}, {ic[j][1], ic[j][3], ic[j][4]},
                                {ic[j][2], ic[j][4], ic[j][5]}};
      M[j] = mass[j];
      for (int a = 0; a < 3; a++) {
        P[j][a] = pp[j][a];
        H[j][a] = mass[j] * c[a];  // first moment m·c
        // inertia about the body origin: Ic + m(|c|²1 − c cᵀ)
        for (int b = 0; b < 3; b++) IO[j][3 * a + b] = icm[a][b] + mass[j] * ((a == b ? cc : 0.0) - c[a] * c[b]);
      }
    }
  }
};

struct Kuka {
  static constexpr int n = 14, m = 7, id = TOG_MODEL_KUKA;
  static constexpr KukaTab KT{};
  // Joint index laundered through an SGPR at each use: the tables are then read from constant memory
  // (scalar loads) where they are used, instead of ~200 fp64 literals being materialised once and
  // kept live in VGPRs across the three RK stages (which spilled 4 KB/lane in the Jacobian). The plain
  // double evaluation (rollouts, stage points: f<double>, LIT) takes the literals instead: the ±1 and 0
  // entries fold into operand modifiers and inline constants, and no table value is loaded (in the
  // rollout the hoisted scalar loads were spilled to VGPR lanes: 2.09 -> 1.71 ms for the 4096 x 8
  // rollouts alone, tools/microbench/kuka_f_bench.hip).
  __host__ __device__ __forceinline__ static int lj(int j) {
#ifdef __HIP_DEVICE_COMPILE__
    asm volatile("" : "+s"(j));
#endif
    return j;
  }
  __host__ __device__ __forceinline__ static double h_(int j, int a) { return KT.H[j][a]; }
  __host__ __device__ __forceinline__ static double io_(int j, int a, int b) { return KT.IO[j][3 * a + b]; }
  template <class T>
  __host__ __device__ __forceinline__ static void r0t(int j, T* y, const T* x) {  // R0ᵀ x
#pragma unroll
    for (int a = 0; a < 3; a++) y[a] = (x[0] * KT.R0[j][a] + x[1] * KT.R0[j][3 + a]) + x[2] * KT.R0[j][6 + a];
  }
  template <class T>
  __host__ __device__ __forceinline__ static void r0(int j, T* y, const T* x) {  // R0 x
#pragma unroll
    for (int a = 0; a < 3; a++)
      y[a] = (x[0] * KT.R0[j][3 * a] + x[1] * KT.R0[j][3 * a + 1]) + x[2] * KT.R0[j][3 * a + 2];
  }
  // (c, s) may be plain doubles while x carries partials: TC * T is then the product a zero-tangent
  // dual would give, fma(t.v, 0, c.v t.g) = c.v t.g (the stage-Jacobian lanes of tog_kuka_jac.hpp)
  template <class TC, class T>
  __host__ __device__ __forceinline__ static void E(int j, const TC& c, const TC& s, T* y, const T* x) {
    T t[3];
    r0t(j, t, x);
    y[0] = c * t[0] + s * t[1];
    y[1] = c * t[1] - s * t[0];
    y[2] = t[2];
  }
  template <class TC, class T>
  __host__ __device__ __forceinline__ static void Et(int j, const TC& c, const TC& s, T* y, const T* x) {
    T t[3];
    t[0] = c * x[0] - s * x[1];
    t[1] = s * x[0] + c * x[1];
    t[2] = x[2];
    r0(j, y, t);
  }
  template <class T>
  __host__ __device__ __forceinline__ static void cross(T* y, const T* a, const T* b) {
    y[0] = a[1] * b[2] - a[2] * b[1];
    y[1] = a[2] * b[0] - a[0] * b[2];
    y[2] = a[0] * b[1] - a[1] * b[0];
  }
  template <class T>
  __host__ __device__ __forceinline__ static void cross_dc(T* y, const T* a, const double* r) {
    y[0] = a[1] * r[2] - a[2] * r[1];
    y[1] = a[2] * r[0] - a[0] * r[2];
    y[2] = a[0] * r[1] - a[1] * r[0];
  }
  template <class T>
  __host__ __device__ __forceinline__ static void cross_cd(T* y, const double* r, const T* b) {
    y[0] = b[2] * r[1] - b[1] * r[2];
    y[1] = b[0] * r[2] - b[2] * r[0];
    y[2] = b[1] * r[0] - b[0] * r[1];
  }
  template <class T>
  __host__ __device__ __forceinline__ static void inertia_mul(int j, T* ang, T* lin, const T* w, const T* v) {
    const double h[3] = {h_(j, 0), h_(j, 1), h_(j, 2)};
    T hx[3];
#pragma unroll
    for (int a = 0; a < 3; a++) ang[a] = (w[0] * io_(j, a, 0) + w[1] * io_(j, a, 1)) + w[2] * io_(j, a, 2);
    cross_cd(hx, h, v);
#pragma unroll
    for (int a = 0; a < 3; a++) ang[a] = ang[a] + hx[a];
    cross_cd(hx, h, w);
#pragma unroll
    for (int a = 0; a < 3; a++) lin[a] = v[a] * KT.M[j] - hx[a];
  }

  // dynamics_bias: RNEA with v̇ = 0 -> tau; also cos/sin of q for the mass matrix. TQ (q, cos, sin) may
  // be double while T (q̇ and everything downstream) is a dual: the partials w.r.t. q̇ at fixed q.
  template <class T, class TQ, bool LIT = false>
  __host__ __device__ __forceinline__ static void bias(T* tau, TQ* cq, TQ* sq, const TQ* q, const T* qd) {
    const T z = cst_(0.0, qd[0]);
    T w[3] = {z, z, z}, v[3] = {z, z, z}, al[3] = {z, z, z}, ln[3] = {z, z, cst_(TOG_KUKA_GRAVITY, qd[0])};
    T nf[7][3], ff[7][3];
#pragma unroll
    for (int j = 0; j < 7; j++) {
      const int jl = LIT ? j : Kuka::lj(j);
      sincos_(q[j], sq[j], cq[j]);
      T t[3], tv[3], wj[3], vj[3], aj[3], lj[3];
      cross_dc(t, w, KT.P[jl]);
#pragma unroll
      for (int a = 0; a < 3; a++) tv[a] = v[a] + t[a];
      E(jl, cq[j], sq[j], wj, w);
      E(jl, cq[j], sq[j], vj, tv);
      wj[2] = wj[2] + qd[j];
      cross_dc(t, al, KT.P[jl]);
#pragma unroll
      for (int a = 0; a < 3; a++) tv[a] = ln[a] + t[a];
      E(jl, cq[j], sq[j], aj, al);
      E(jl, cq[j], sq[j], lj, tv);
      aj[0] = aj[0] + wj[1] * qd[j];
      aj[1] = aj[1] - wj[0] * qd[j];
      lj[0] = lj[0] + vj[1] * qd[j];
      lj[1] = lj[1] - vj[0] * qd[j];
      T hva[3], hvl[3], iaa[3], ial[3], c1[3], c2[3];
      inertia_mul(jl, hva, hvl, wj, vj);
      inertia_mul(jl, iaa, ial, aj, lj);
      cross(c1, wj, hva);
      cross(c2, vj, hvl);
#pragma unroll
      for (int a = 0; a < 3; a++) nf[j][a] = iaa[a] + (c1[a] + c2[a]);
      cross(c1, wj, hvl);
#pragma unroll
      for (int a = 0; a < 3; a++) {
        ff[j][a] = ial[a] + c1[a];
        w[a] = wj[a];
        v[a] = vj[a];
        al[a] = aj[a];
        ln[a] = lj[a];
      }
    }
#pragma unroll
    for (int j = 6; j >= 0; j--) {
      tau[j] = nf[j][2];
      if (j > 0) {
        T fp[3], np[3], rx[3];
        const int jl = LIT ? j : Kuka::lj(j);
        Et(jl, cq[j], sq[j], fp, ff[j]);
        Et(jl, cq[j], sq[j], np, nf[j]);
        cross_cd(rx, KT.P[jl], fp);
#pragma unroll
        for (int a = 0; a < 3; a++) {
          np[a] = np[a] + rx[a];
          nf[j - 1][a] = nf[j - 1][a] + np[a];
          ff[j - 1][a] = ff[j - 1][a] + fp[a];
        }
      }
    }
  }

  // mass_matrix by CRBA; lower triangle M[i][j], i >= j
  template <class T, bool LIT = false>
  __host__ __device__ __forceinline__ static void mass(T (*M)[7], const T* cq, const T* sq) {
    double mc = KT.M[6];
    T hc[3], Ic[3][3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      hc[a] = cst_(h_(6, a), cq[0]);
#pragma unroll
      for (int b = 0; b < 3; b++) Ic[a][b] = cst_(io_(6, a, b), cq[0]);
    }
#pragma unroll
    for (int j = 6; j >= 0; j--) {
      T Fa[3], Fl[3];
#pragma unroll
      for (int a = 0; a < 3; a++) Fa[a] = Ic[a][2];
      Fl[0] = -hc[1];
      Fl[1] = hc[0];
      Fl[2] = cst_(0.0, cq[0]);
      M[j][j] = Fa[2];
#pragma unroll
      for (int k = j; k >= 1; k--) {
        T fl[3], fa[3], rx[3];
        const int kl = LIT ? k : Kuka::lj(k);
        Et(kl, cq[k], sq[k], fl, Fl);
        Et(kl, cq[k], sq[k], fa, Fa);
        cross_cd(rx, KT.P[kl], fl);
#pragma unroll
        for (int a = 0; a < 3; a++) {
          Fa[a] = fa[a] + rx[a];
          Fl[a] = fl[a];
        }
        M[j][k - 1] = Fa[2];
      }
      if (j > 0) {
        const int jl = LIT ? j : Kuka::lj(j), jp = LIT ? j - 1 : Kuka::lj(j - 1);
        const double* r = KT.P[jl];
        T hr[3], W[3][3], col[3], row[3], Ir[3][3];
        Et(jl, cq[j], sq[j], hr, hc);
#pragma unroll
        for (int b = 0; b < 3; b++) {
#pragma unroll
          for (int a = 0; a < 3; a++) col[a] = Ic[a][b];
          Et(jl, cq[j], sq[j], row, col);
#pragma unroll
          for (int a = 0; a < 3; a++) W[a][b] = row[a];
        }
#pragma unroll
        for (int a = 0; a < 3; a++) {
          Et(jl, cq[j], sq[j], row, W[a]);
#pragma unroll
          for (int b = 0; b < 3; b++) Ir[a][b] = row[b];
        }
        const double rr = (r[0] * r[0] + r[1] * r[1]) + r[2] * r[2];
        const T dot = (hr[0] * r[0] + hr[1] * r[1]) + hr[2] * r[2];
        const T sh = dot * 2.0 + mc * rr;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
          for (int b = 0; b < 3; b++) {
            T t = Ir[a][b] - (hr[a] * r[b] + hr[b] * r[a]);
            t = t + (-((mc * r[a]) * r[b]));
            if (a == b) t = t + sh;
            Ic[a][b] = t + io_(jp, a, b);
          }
#pragma unroll
        for (int a = 0; a < 3; a++) hc[a] = (hr[a] + mc * r[a]) + h_(jp, a);
        mc = mc + KT.M[jp];
      }
    }
  }

  // Cholesky M = L Lᵀ in place (entry (i,j) of M is read once, before L[i][j] replaces it)
  template <class T>
  __host__ __device__ __forceinline__ static void chol(T (*L)[7]) {
#pragma unroll
    for (int j = 0; j < 7; j++) {
      T s = L[j][j];
#pragma unroll
      for (int k = 0; k < j; k++) s = s - L[j][k] * L[j][k];
      L[j][j] = sqrt_(s);
#pragma unroll
      for (int i = j + 1; i < 7; i++) {
        T t = L[i][j];
#pragma unroll
        for (int k = 0; k < j; k++) t = t - L[i][k] * L[j][k];
        L[i][j] = t / L[j][j];
      }
    }
  }
  // t / L_ii with the dual quotient's partials, x.p * inv(y) (the divisor's partials are zero when L is
  // a plain double: fma(x.p, 1/y, 0 * c2) = x.p * (1/y), not x.p / y)
  __host__ __device__ __forceinline__ static double kdiv(double t, double l) { return t / l; }
  template <int W>
  __host__ __device__ __forceinline__ static Dual<W> kdiv(const Dual<W>& t, const Dual<W>& l) { return t / l; }
  template <int W>
  __host__ __device__ __forceinline__ static Dual<W> kdiv(const Dual<W>& t, double l) {
    Dual<W> r;
    r.v = t.v / l;
    const double iy = 1.0 / l;
#pragma unroll
    for (int i = 0; i < W; i++) r.g[i] = t.g[i] * iy;
    return r;
  }
  // v̇ = L⁻ᵀ L⁻¹ (u − τ): forward then backward substitution
  template <class TL, class T, class TU>
  __host__ __device__ __forceinline__ static void solve(T* vd, const TL (*L)[7], const TU* u, const T* tau) {
    T y[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
      T t = u[i] - tau[i];
#pragma unroll
      for (int k = 0; k < i; k++) t = t - L[i][k] * y[k];
      y[i] = kdiv(t, L[i][i]);
    }
#pragma unroll
    for (int i = 6; i >= 0; i--) {
      T t = y[i];
#pragma unroll
      for (int k = i + 1; k < 7; k++) t = t - L[k][i] * vd[k];
      vd[i] = kdiv(t, L[i][i]);
    }
  }

  // f keeps its Cholesky and substitutions inline (the same operations as chol() and solve(), which the
  // mixed-type stage-Jacobian lanes use): written through the helpers, the rollout kernels of the
  // minimum-time Kuka (MinTime<Kuka>, 15 x 8) were compiled with a broken divergence test — trials
  // with states beyond max_state_value, or NaN costs, came back accepted (round 4; the same source
  // compiled for the host is bit-identical to the oracle). The inline form restores round 3's code.
  template <class T, bool LIT = std::is_same<T, double>::value>
  __host__ __device__ __forceinline__ static void f(T* xd, const T* x, const T* u) {
    const T* q = x;
    const T* qd = x + 7;
    T tau[7], cq[7], sq[7], L[7][7], y[7];
    bias<T, T, LIT>(tau, cq, sq, q, qd);
    mass<T, LIT>(L, cq, sq);
#ifdef TOG_KUKA_HELPER_F  // round 4's helper form (tools/kuka_helper_build.py: the miscompile investigation only)
    chol(L);
    solve(xd + 7, L, u, tau);
#pragma unroll
    for (int i = 0; i < 7; i++) xd[i] = qd[i];
    (void)y;
    return;
#endif
    // Cholesky M = L Lᵀ in place (entry (i,j) of M is read once, before L[i][j] replaces it)
#pragma unroll
    for (int j = 0; j < 7; j++) {
      T s = L[j][j];
#pragma unroll
      for (int k = 0; k < j; k++) s = s - L[j][k] * L[j][k];
      L[j][j] = sqrt_(s);
#pragma unroll
      for (int i = j + 1; i < 7; i++) {
        T t = L[i][j];
#pragma unroll
        for (int k = 0; k < j; k++) t = t - L[i][k] * L[j][k];
        L[i][j] = t / L[j][j];
      }
    }
#pragma unroll
    for (int i = 0; i < 7; i++) {
      T t = u[i] - tau[i];
#pragma unroll
      for (int k = 0; k < i; k++) t = t - L[i][k] * y[k];
      y[i] = t / L[i][i];
    }
#pragma unroll
    for (int i = 6; i >= 0; i--) {
      T t = y[i];
#pragma unroll
      for (int k = i + 1; k < 7; k++) t = t - L[k][i] * xd[7 + k];
      xd[7 + i] = t / L[i][i];
    }
#pragma unroll
    for (int i = 0; i < 7; i++) xd[i] = qd[i];
  }
};

// ---------------------------------------------------------------------------------------------
// add_slack_controls(model) (src/model.jl:761-779): the infeasible-start model. Controls are
// [u (Mb::m); s (Mb::n)], x+ = f_d(x, u) + s. Kernels see it as a model with m = Mb::m + Mb::n;
// discrete_step adds the slacks after the base model's RK step, k_jacobian writes the identity
// slack block directly (the reference's ∇f! copies Diagonal(1.0I, n), it is never differentiated).
// models that define user constraint functions (plugins: static constexpr bool has_con = true and
// template <class T> static void con(int fid, T* c, const T* x, const T* u))
template <class M, class = void>
struct HasCon : std::false_type {};
template <class M>
struct HasCon<M, std::void_t<decltype(M::has_con)>> : std::integral_constant<bool, M::has_con> {};

template <class Mb>
struct Infeasible {
  using Base = Mb;
  static constexpr int n = Mb::n, m = Mb::m + Mb::n, id = Mb::id;
  static constexpr int slack = Mb::n;
  static constexpr bool has_con = HasCon<Mb>::value;  // constraints see the base controls u[1:m]
  template <class T>
  __host__ __device__ __forceinline__ static void con(int fid, T* c, const T* x, const T* u) {
    if constexpr (HasCon<Mb>::value) Mb::con(fid, c, x, u);
  }
};

// add_min_time_controls(model) (src/solvers/altro/minimum_time.jl:83-104): state [x; τ], control
// [u; h], x+ = f_d(x, u, h²), τ+ = h. The time step of every knot is a control (dt_k = h_k², get_dt
// src/problem.jl:300-314); the objective is MinTimeCost (:142-200) and the problem gets the h bounds and
// the h_k = τ_k equalities (mintime_constraints, :125-141).
template <class Mb>
struct MinTime {
  using Base = Mb;
  static constexpr int n = Mb::n + 1, m = Mb::m + 1, id = Mb::id;
  // user constraint functions see the base model's x[1:n], u[1:m] (mintime_constraints'
  // update_constraint_set_jacobians(PC[k], n, n+1, m), minimum_time.jl:125-141): τ and h get zero gradients
  static constexpr bool has_con = HasCon<Mb>::value;
  template <class T>
  __host__ __device__ __forceinline__ static void con(int fid, T* c, const T* x, const T* u) {
    if constexpr (HasCon<Mb>::value) Mb::con(fid, c, x, u);
  }
};

template <class M>
struct ModelTraits {
  using Base = M;
  using Core = M;  // the model inside every wrapper (the one whose dynamics are differentiated)
  static constexpr int slack = 0;
  // implicit integrators instantiated: the small models and the quadrotor (the Kuka arm's are in a unit of
  // their own, KukaImplicit); explicit_ok: the explicit integrators instantiated
  static constexpr bool implicit_ok = M::n <= 4 || M::id == TOG_MODEL_QUADROTOR;
  static constexpr bool explicit_ok = true;
  static constexpr bool min_time = false;
};
template <class Mb>
struct ModelTraits<MinTime<Mb>> {
  using Base = Mb;
  using Core = Mb;
  static constexpr int slack = 0;
  static constexpr bool implicit_ok = false;
  static constexpr bool explicit_ok = true;
  static constexpr bool min_time = true;
};
template <class Mb>
struct ModelTraits<Infeasible<Mb>> {
  using Base = Mb;
  using Core = Mb;
  static constexpr int slack = Mb::n;
  static constexpr bool implicit_ok = false;
  static constexpr bool explicit_ok = true;
  static constexpr bool min_time = false;
};
// altro_problem's infeasible start with tf = :min (altro_methods.jl:98-124): minimum_time_problem of the
// infeasible problem, add_min_time_controls(add_slack_controls(model)): x = [x; τ], u = [u; s; h],
// x+ = f_d(x, u, h²) + s, τ+ = h. discrete_step unwraps MinTime to Infeasible<Mb> (Base); the Jacobian
// differentiates Mb (Core) and writes the slack identity and the h column as the two wrappers' ∇f! do.
template <class Mb>
struct ModelTraits<MinTime<Infeasible<Mb>>> {
  using Base = Infeasible<Mb>;
  using Core = Mb;
  static constexpr int slack = Mb::n;
  static constexpr bool implicit_ok = false;
  static constexpr bool explicit_ok = true;
  static constexpr bool min_time = true;
};
// The Kuka arm under the implicit schemes (midpoint_implicit / rk3_implicit): the same model, its kernels
// instantiated for those two integrators only, in their own translation unit (k_kuka_implicit.hip), so the
// 14-state Newton steps do not double the Kuka unit's build time
struct KukaImplicit : Kuka {};
template <>
struct ModelTraits<KukaImplicit> {
  using Base = KukaImplicit;
  using Core = KukaImplicit;
  static constexpr int slack = 0;
  static constexpr bool implicit_ok = true;
  static constexpr bool explicit_ok = false;
  static constexpr bool min_time = false;
};

// ---------------------------------------------------------------------------------------------
// Implicit integrators (src/integration.jl:44-73 midpoint_implicit, :171-205 rk3_implicit): a
// Newton solve for x+ per step, run while ||g||_2 > 1e-12. Same operations, in the same order, as
// the oracle's implicit_step_dual (oracle/tog_oracle.c): the iterate carries the Jacobian's partials
// when T is a Dual, ∇g is formed at the values (∂f/∂x one Dual<1> column at a time), and
// δy = (-∇g)\g by partial-pivoting LU. rk3_implicit reproduces the reference's aliasing of
// fc1 = fc2 = fc3 (one array), so its residual is y - x - dt/6 F - 4/6 dt F - dt/6 F, F = f(Xm).
// Built for models with n <= 4, the quadrotor and the Kuka arm (ModelTraits::implicit_ok, KukaImplicit; at
// n = 13-14 the real ∇g and its LU live in scratch, several KB per lane: parity, not speed); the reference's
// 1000-iteration error becomes a NaN state (the rollout then fails as diverged).
template <int n>
__host__ __device__ __forceinline__ double jl_norm2(const double* g) {
  double mx = 0.0;
#pragma unroll
  for (int i = 0; i < n; i++) mx = tog_jlmax(mx, fabs(g[i]));
  if (mx != mx || mx == 0.0 || isinf(mx)) return mx;
  if (isfinite((double)n * mx * mx) && mx * mx != 0.0) {
    double s = g[0] * g[0];
#pragma unroll
    for (int i = 1; i < n; i++) s = s + g[i] * g[i];
    return sqrt(s);
  }
  double t = fabs(g[0]) / mx, s = t * t;
#pragma unroll
  for (int i = 1; i < n; i++) {
    t = fabs(g[i]) / mx;
    s = s + t * t;
  }
  return mx * sqrt(s);
}

template <class M, class T>
__host__ __device__ __forceinline__ void jac_x_val(double* A, const T* x, const T* u) {
  constexpr int n = M::n, m = M::m;
#pragma unroll
  for (int j = 0; j < n; j++) {
    Dual<1> X[n], U[m], F[n];
#pragma unroll
    for (int i = 0; i < n; i++) {
      X[i].v = val_(x[i]);
      X[i].g[0] = (i == j) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < m; i++) {
      U[i].v = val_(u[i]);
      U[i].g[0] = 0.0;
    }
    M::f(F, X, U);
#pragma unroll
    for (int i = 0; i < n; i++) A[i + n * j] = F[i].g[0];
  }
}

// b <- (-G) \ b (generic_lufact! + naivesub!, see the oracle's lu_neg_solve)
template <int n, class T>
__host__ __device__ __forceinline__ void lu_neg_solve(const double* G, T* b) {
  double a[n * n];
#pragma unroll
  for (int e = 0; e < n * n; e++) a[e] = -G[e];
  int piv[n];
#pragma unroll
  for (int k = 0; k < n; k++) {
    int kp = k;
    double amax = 0.0;
#pragma unroll
    for (int i = k; i < n; i++) {
      const double ai = fabs(a[i + n * k]);
      if (ai > amax) {
        kp = i;
        amax = ai;
      }
    }
    piv[k] = kp;
    if (a[kp + n * k] != 0.0) {
      if (kp != k) {
#pragma unroll
        for (int j = 0; j < n; j++) {
          // select-based swap keeps the matrix in registers (no dynamic indexing)
#pragma unroll
          for (int i = k + 1; i < n; i++)
            if (i == kp) {
              const double t = a[k + n * j];
              a[k + n * j] = a[i + n * j];
              a[i + n * j] = t;
            }
        }
      }
      const double inv = 1.0 / a[k + n * k];
#pragma unroll
      for (int i = k + 1; i < n; i++) a[i + n * k] = a[i + n * k] * inv;
    }
#pragma unroll
    for (int j = k + 1; j < n; j++)
#pragma unroll
      for (int i = k + 1; i < n; i++) a[i + n * j] = a[i + n * j] - a[i + n * k] * a[k + n * j];
  }
#pragma unroll
  for (int k = 0; k < n; k++) {
#pragma unroll
    for (int i = k + 1; i < n; i++)
      if (piv[k] == i) {
        const T t = b[k];
        b[k] = b[i];
        b[i] = t;
      }
  }
#pragma unroll
  for (int j = 0; j < n; j++)
#pragma unroll
    for (int i = j + 1; i < n; i++) b[i] = b[i] - a[i + n * j] * b[j];
#pragma unroll
  for (int j = n - 1; j >= 0; j--) {
    b[j] = b[j] / a[j + n * j];
#pragma unroll
    for (int i = j - 1; i >= 0; i--) b[i] = b[i] - a[i + n * j] * b[j];
  }
}

template <class M, int INTEG, class T>
__host__ __device__ __forceinline__ void implicit_step(T* y, const T* x, const T* u, double dt) {
  constexpr int n = M::n;
#pragma unroll
  for (int i = 0; i < n; i++) y[i] = x[i];
  double gn = INFINITY;
  int cnt = 0;
  while (gn > 1e-12) {
    if (++cnt > 1000) {  // error("Integration convergence fail")
#pragma unroll
      for (int i = 0; i < n; i++) y[i] = cst_(NAN, x[i]);
      return;
    }
    T g[n], xm[n], F[n];
    double G[n * n], A[n * n];
    if constexpr (INTEG == TOG_MIDPOINT_IMPLICIT) {
#pragma unroll
      for (int i = 0; i < n; i++) xm[i] = 0.5 * (x[i] + y[i]);
      M::f(F, xm, u);
#pragma unroll
      for (int i = 0; i < n; i++) g[i] = (y[i] - x[i]) - dt * F[i];
      jac_x_val<M>(A, xm, u);
      const double h = 0.5 * dt;
#pragma unroll
      for (int j = 0; j < n; j++)
#pragma unroll
        for (int i = 0; i < n; i++) G[i + n * j] = (i == j ? 1.0 : 0.0) - h * A[i + n * j];
    } else {
      T d[n];
      M::f(F, y, u);  // f(fc1, x, u); f(fc3, y, u) -- one array: F = f(y)
#pragma unroll
      for (int i = 0; i < n; i++) d[i] = F[i] - F[i];
      const double dt8 = dt / 8.0;
#pragma unroll
      for (int i = 0; i < n; i++) xm[i] = 0.5 * (x[i] + y[i]) + dt8 * d[i];
      M::f(F, xm, u);  // f(fc2, Xm, u): fc1 = fc2 = fc3 = f(Xm)
      const double dt6 = dt / 6.0, dt46 = (4.0 / 6.0) * dt;
#pragma unroll
      for (int i = 0; i < n; i++) g[i] = (((y[i] - x[i]) - dt6 * F[i]) - dt46 * F[i]) - dt6 * F[i];
      double A2[n * n], M2[n * n];
      jac_x_val<M>(A, xm, u);
      jac_x_val<M>(A2, y, u);
#pragma unroll
      for (int j = 0; j < n; j++)
#pragma unroll
        for (int i = 0; i < n; i++) M2[i + n * j] = (i == j ? 0.5 : 0.0) - dt8 * A2[i + n * j];
#pragma unroll
      for (int j = 0; j < n; j++)
#pragma unroll
        for (int i = 0; i < n; i++) {
          double p = (dt46 * A[i]) * M2[n * j];
#pragma unroll
          for (int k = 1; k < n; k++) p = p + (dt46 * A[i + n * k]) * M2[k + n * j];
          G[i + n * j] = ((i == j ? 1.0 : 0.0) - p) - dt6 * A2[i + n * j];
        }
    }
    double gv[n];
#pragma unroll
    for (int i = 0; i < n; i++) gv[i] = val_(g[i]);
    gn = jl_norm2<n>(gv);
    lu_neg_solve<n>(G, g);
#pragma unroll
    for (int i = 0; i < n; i++) y[i] = y[i] + g[i];
  }
}

// The 13-14 state Newton steps out of line: one copy per (model, scheme, scalar type) instead of one per
// calling kernel (the Kuka unit's build time; the arithmetic is the same call for call)
template <class M, int INTEG, class T>
__host__ __device__ __attribute__((noinline)) void implicit_step_outlined(T* y, const T* x, const T* u, double dt) {
  implicit_step<M, INTEG, T>(y, x, u, dt);
}

// ---------------------------------------------------------------------------------------------
// Explicit Runge-Kutta discretisation with runtime dt (src/integration.jl:115-158). Running-sum
// form keeps the reference's left-to-right association: RK4 ((k1 + 2k2) + 2k3) + k4,
// RK3 (k1 + 4k2) + k3, with RK3's third stage at (x - k1) + 2k2.
template <class M, int INTEG, class T, class TD = double>
__host__ __device__ __forceinline__ void discrete_step(T* xn, const T* x, const T* u, TD dt) {
  if constexpr (ModelTraits<M>::min_time) {
    using Mb = typename ModelTraits<M>::Base;  // f!(x+, x, u, dt): h = u[end]; model.f(x+, x, u, h^2); x+[n̄] = h
    const T h = u[Mb::m];
    discrete_step<Mb, INTEG, T, T>(xn, x, u, h * h);
    xn[Mb::n] = h;
    (void)dt;
  } else if constexpr (ModelTraits<M>::slack > 0) {
    using Mb = typename ModelTraits<M>::Base;
    discrete_step<Mb, INTEG, T, TD>(xn, x, u, dt);  // model.f(x+, x, u[idx.u], dt)
#pragma unroll
    for (int i = 0; i < Mb::n; i++) xn[i] = xn[i] + u[Mb::m + i];  // x+ .+= u[idx.inf]
  } else {
  constexpr int n = M::n;
  if constexpr (INTEG == TOG_MIDPOINT_IMPLICIT || INTEG == TOG_RK3_IMPLICIT) {
    if constexpr (M::n > 4)
      implicit_step_outlined<M, INTEG, T>(xn, x, u, dt);
    else
      implicit_step<M, INTEG, T>(xn, x, u, dt);
    return;
  } else if constexpr (INTEG == TOG_MIDPOINT) {
    // midpoint (src/integration.jl:26-33): ẋ = f(x,u); ẋ .*= dt/2; ẋ = f(x + ẋ, u); x+ = x + ẋ*dt
    T k[n], t[n];
    M::f(k, x, u);
    const TD h = dt / 2.0;
#pragma unroll
    for (int i = 0; i < n; i++) t[i] = x[i] + k[i] * h;
    M::f(k, t, u);
#pragma unroll
    for (int i = 0; i < n; i++) xn[i] = x[i] + k[i] * dt;
    return;
  } else {
  T k[n], s[n], t[n];
  M::f(k, x, u);
#pragma unroll
  for (int i = 0; i < n; i++) k[i] = k[i] * dt;
#pragma unroll
  for (int i = 0; i < n; i++) {
    s[i] = k[i];
    t[i] = x[i] + k[i] / 2.0;
  }
  M::f(k, t, u);
#pragma unroll
  for (int i = 0; i < n; i++) k[i] = k[i] * dt;
  if constexpr (INTEG == TOG_RK4) {
#pragma unroll
    for (int i = 0; i < n; i++) {
      s[i] = s[i] + 2.0 * k[i];
      t[i] = x[i] + k[i] / 2.0;
    }
    M::f(k, t, u);
#pragma unroll
    for (int i = 0; i < n; i++) k[i] = k[i] * dt;
#pragma unroll
    for (int i = 0; i < n; i++) {
      s[i] = s[i] + 2.0 * k[i];
      t[i] = x[i] + k[i];
    }
    M::f(k, t, u);
#pragma unroll
    for (int i = 0; i < n; i++) {
      k[i] = k[i] * dt;
      s[i] = s[i] + k[i];
      xn[i] = x[i] + div6_(s[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < n; i++) {
      t[i] = (x[i] - s[i]) + 2.0 * k[i];  // s == k1 here
      s[i] = s[i] + 4.0 * k[i];
    }
    M::f(k, t, u);
#pragma unroll
    for (int i = 0; i < n; i++) {
      k[i] = k[i] * dt;
      s[i] = s[i] + k[i];
      xn[i] = x[i] + div6_(s[i]);
    }
  }
  }
  }
}

// ---------------------------------------------------------------------------------------------
// Costs (src/cost.jl:171-181), same association as the oracle. The outer loops are kept rolled:
// fully unrolled, the compiler hoists all of Q into registers across the knot loop and spills.
// DC: 0 = the cost's structure from P->diag_cost at run time; 1 = diagonal (the caller knows
// P->diag_cost != 0); 2 = dense. A kernel that inlines only the diagonal form keeps x and u in registers
// (the dense loops index them at run time).
// Stage knot k's QuadraticCost (src/cost.jl:112-157): the problem's, or row k of a time-varying Objective's
// table (DevProblem::kc). Matrices column-major with the compact n, m; cQ, cR the upper Cholesky factors of
// Q dt and R dt (the square-root expansion, src/objective.jl:70-94).
struct CostView {
  const double *Q, *R, *H, *q, *r, *cQ, *cR;
  double c;
};
template <int n, int m>
__host__ __device__ constexpr int kc_stride_of() {
  return 2 * n * n + 2 * m * m + m * n + n + m + 1;
}
template <int n, int m>
__device__ __forceinline__ CostView cost_at(const DevProblem* P, int k) {
  if (!P->kc) return CostView{P->Q, P->R, P->H, P->q, P->r, P->cQ, P->cR, P->c};
  const double* b = P->kc + (size_t)k * kc_stride_of<n, m>();
  constexpr int oR = n * n, oH = oR + m * m, oq = oH + m * n, orr = oq + n, oc = orr + m, ocQ = oc + 1, ocR = ocQ + n * n;
  return CostView{b, b + oR, b + oH, b + oq, b + orr, b + ocQ, b + ocR, b[oc]};
}

template <int n, int m, int DC = 0>
__device__ __forceinline__ double stage_cost_dt(const DevProblem* P, int k, const double* x, const double* u, double dt) {
  const CostView C = cost_at<n, m>(P, k);
  double xQx = 0.0, uRu = 0.0, qx = 0.0, ru = 0.0, uHx = 0.0;
  if (DC == 1 || (DC == 0 && P->diag_cost)) {
#pragma unroll
    for (int j = 0; j < n; j++) xQx = fma((0.5 * x[j]) * C.Q[j + n * j], x[j], xQx);
#pragma unroll
    for (int j = 0; j < m; j++) uRu = fma((0.5 * u[j]) * C.R[j + m * j], u[j], uRu);
  } else {
#pragma unroll 1
    for (int j = 0; j < n; j++) {
      double t = 0.0;
      for (int i = 0; i < n; i++) t = fma(0.5 * x[i], C.Q[i + n * j], t);
      xQx = fma(t, x[j], xQx);
    }
#pragma unroll 1
    for (int j = 0; j < m; j++) {
      double t = 0.0;
      for (int i = 0; i < m; i++) t = fma(0.5 * u[i], C.R[i + m * j], t);
      uRu = fma(t, u[j], uRu);
    }
#pragma unroll 1
    for (int j = 0; j < n; j++) {
      double t = 0.0;
      for (int i = 0; i < m; i++) t = fma(u[i], C.H[i + m * j], t);
      uHx = fma(t, x[j], uHx);
    }
  }
#pragma unroll
  for (int i = 0; i < n; i++) qx = fma(C.q[i], x[i], qx);
#pragma unroll
  for (int i = 0; i < m; i++) ru = fma(C.r[i], u[i], ru);
  return ((((xQx + uRu) + qx) + ru) + C.c + uHx) * dt;
}
template <int n, int m, int DC = 0>
__device__ __forceinline__ double stage_cost(const DevProblem* P, int k, const double* x, const double* u) {
  return stage_cost_dt<n, m, DC>(P, k, x, u, P->dt);
}

template <int n, int DC = 0>
__device__ __forceinline__ double terminal_cost(const DevProblem* P, const double* x) {
  double xQx = 0.0, qx = 0.0;
  if (DC == 1 || (DC == 0 && P->diag_cost)) {
#pragma unroll
    for (int j = 0; j < n; j++) xQx = fma((0.5 * x[j]) * P->Qf[j + n * j], x[j], xQx);
  } else {
#pragma unroll 1
    for (int j = 0; j < n; j++) {
      double t = 0.0;
      for (int i = 0; i < n; i++) t = fma(0.5 * x[i], P->Qf[i + n * j], t);
      xQx = fma(t, x[j], xQx);
    }
  }
#pragma unroll
  for (int i = 0; i < n; i++) qx = fma(P->qf[i], x[i], qx);
  return (xQx + qx) + P->cf;
}

// stage / terminal cost of model M: MinTimeCost for a minimum-time model (minimum_time.jl:148-149:
// stage_cost(cost, x[1:n], u[1:m], h) + R_min_time u[end]^2 with dt = h = u[end]^2, terminal unchanged;
// the zero-padded base matrices give the base cost of the leading parts bit for bit)
template <class M, int DC = 0>
__device__ __forceinline__ double stage_cost_m(const DevProblem* P, int k, const double* x, const double* u) {
  if constexpr (ModelTraits<M>::min_time) {
    const double h = u[M::m - 1];
    return stage_cost_dt<M::n, M::m, DC>(P, k, x, u, h * h) + P->R_min_time * (h * h);
  } else {
    return stage_cost<M::n, M::m, DC>(P, k, x, u);
  }
}
template <class M, int DC = 0>
__device__ __forceinline__ double terminal_cost_m(const DevProblem* P, const double* x) {
  return terminal_cost<M::n, DC>(P, x);
}

// constraint row value (u == nullptr at the terminal knot: only x rows exist there)
// v[i] for a wave-uniform i in [0, NN) without an indexed register read: a chain of selects over
// constant indices, so v stays in registers. An indexed read (s_set_gpr_idx) may read any register, so
// the wait inserted before it drains every outstanding global load of the wave; in the rollouts, which
// keep loads in flight across knots, that exposed a memory round trip per row.
// (The empty asm makes each candidate an opaque value: without it the optimiser folds the chain of
// selects over loads into one load from a selected address, and the array goes to scratch memory.)
template <int NN>
__device__ __forceinline__ double reg_at(const double* v, int i) {
  double r = v[0];
#pragma unroll
  for (int j = 1; j < NN; j++) {
    double t = v[j];
    asm volatile("" : "+v"(t));
    r = (i == j) ? t : r;
  }
  return r;
}
// x[i] / u[i] of a row: an indexed register move (IDX = 0: the backward kernels, which hold no loads in
// flight there), or reg_at over the model's n / m (IDX = n, m: the rollouts)
template <int NX, int NU>
struct RowAt {
  __device__ __forceinline__ static double x(const double* x, int i) {
    if constexpr (NX > 0) return reg_at<NX>(x, i); else return x[i];
  }
  __device__ __forceinline__ static double u(const double* u, int i) {
    if constexpr (NU > 0) return reg_at<NU>(u, i); else return u[i];
  }
};

// SLACK = false compiles the infeasible-start slack row out (plain models never have it; the extra
// case costs the team backward kernel registers)
template <bool SLACK = true, int NX = 0, int NU = 0>
__device__ __forceinline__ double row_value(const ConRow& r, const double* x, const double* u) {
  using A = RowAt<NX, NU>;
  if (SLACK && r.type == ROW_USLACK) return A::u(u, r.idx);
  if (r.type == ROW_MT_EQ) return A::u(u, (int)r.a) - A::x(x, r.idx);
  switch (r.type) {
    case ROW_XMAX: return A::x(x, r.idx) - r.a;
    case ROW_UMAX: return A::u(u, r.idx) - r.a;
    case ROW_XMIN: return r.a - A::x(x, r.idx);
    case ROW_UMIN: return r.a - A::u(u, r.idx);
    case ROW_GOAL: return A::x(x, r.idx) - r.a;
    case ROW_CIRCLE: {
      const double dx = x[0] - r.a, dy = x[1] - r.b;
      return -((dx * dx + dy * dy) - r.r * r.r);
    }
    default: {
      const double dx = x[0] - r.a, dy = x[1] - r.b, dz = x[2] - r.c;
      return -(((dx * dx + dy * dy) + dz * dz) - r.r * r.r);
    }
  }
}
template <bool SLACK = true>
__device__ __forceinline__ bool row_inequality(const ConRow& r) {
  return r.type != ROW_GOAL && r.type != ROW_USER_EQ && r.type != ROW_MT_EQ && (!SLACK || r.type != ROW_USLACK);
}

// The same row seen by every lane of a wave (lanes iterate knots and rows in lockstep over the
// shared row table): make its type and index wave-uniform so that the switch is a scalar branch
// and x[idx] an indexed register move, not a per-lane chain of compares and selects.
__device__ __forceinline__ ConRow uniform_row(ConRow r) {
  ConRow u = r;
  u.type = __builtin_amdgcn_readfirstlane(r.type);
  u.idx = __builtin_amdgcn_readfirstlane(r.idx);
  return u;
}

// d c / d [x; u] of a row: writes up to 3 (index, value) pairs, index in [0, n+m)
template <bool SLACK = true>
__device__ __forceinline__ int row_grad(const ConRow& r, const double* x, int n, int* idx, double* v) {
  if (SLACK && r.type == ROW_USLACK) {
    idx[0] = n + r.idx;
    v[0] = 1.0;
    return 1;
  }
  if (r.type == ROW_MT_EQ) {
    idx[0] = r.idx;
    v[0] = -1.0;
    idx[1] = n + (int)r.a;
    v[1] = 1.0;
    return 2;
  }
  switch (r.type) {
    case ROW_XMAX: idx[0] = r.idx; v[0] = 1.0; return 1;
    case ROW_UMAX: idx[0] = n + r.idx; v[0] = 1.0; return 1;
    case ROW_XMIN: idx[0] = r.idx; v[0] = -1.0; return 1;
    case ROW_UMIN: idx[0] = n + r.idx; v[0] = -1.0; return 1;
    case ROW_GOAL: idx[0] = r.idx; v[0] = 1.0; return 1;
    case ROW_CIRCLE:
      idx[0] = 0; v[0] = -(2.0 * (x[0] - r.a));
      idx[1] = 1; v[1] = -(2.0 * (x[1] - r.b));
      return 2;
    default:
      idx[0] = 0; v[0] = -(2.0 * (x[0] - r.a));
      idx[1] = 1; v[1] = -(2.0 * (x[1] - r.b));
      idx[2] = 2; v[2] = -(2.0 * (x[2] - r.c));
      return 3;
  }
}

// Rows of a model: the built-in row types, plus the user constraint rows of a plugin model. A user
// row evaluates the model's con(fid, c, x, u) (u = zeros at the terminal knot) and takes output idx;
// its gradient over [x; u_base] comes from dual numbers with n + m_base partials (ForwardDiff).
template <class M, bool NOIDX = false>
__device__ __forceinline__ double row_value_m(const ConRow& r, const double* x, const double* u) {
  if constexpr (HasCon<M>::value) {
    if (r.type == ROW_USER_INEQ || r.type == ROW_USER_EQ) {
      using Mb = typename ModelTraits<M>::Base;
      double u0[Mb::m], c[PUSER];
#pragma unroll
      for (int i = 0; i < Mb::m; i++) u0[i] = u ? u[i] : 0.0;
      M::con((int)r.a, c, x, u0);
      return c[r.idx];
    }
  }
  return row_value<(ModelTraits<M>::slack > 0), NOIDX ? M::n : 0, NOIDX ? M::m : 0>(r, x, u);
}
template <class M>
__host__ __device__ constexpr int row_grad_cap() {
  return HasCon<M>::value ? M::n + ModelTraits<M>::Base::m : 3;
}
template <class M>
__device__ __forceinline__ int row_grad_m(const ConRow& r, const double* x, const double* u, int* idx, double* v) {
  if constexpr (HasCon<M>::value) {
    if (r.type == ROW_USER_INEQ || r.type == ROW_USER_EQ) {
      using Mb = typename ModelTraits<M>::Base;
      constexpr int n = M::n, mb = Mb::m, W = n + mb;
      Dual<W> xd[n], ud[mb], c[PUSER];
#pragma unroll
      for (int i = 0; i < n; i++) {
        xd[i].v = x[i];
#pragma unroll
        for (int w = 0; w < W; w++) xd[i].g[w] = (w == i) ? 1.0 : 0.0;
      }
#pragma unroll
      for (int i = 0; i < mb; i++) {
        ud[i].v = u ? u[i] : 0.0;
#pragma unroll
        for (int w = 0; w < W; w++) ud[i].g[w] = (w == n + i) ? 1.0 : 0.0;
      }
      M::con((int)r.a, c, xd, ud);
      const int nz = u ? W : n;  // terminal rows: state gradient only
      for (int w = 0; w < nz; w++) {
        idx[w] = w;
        v[w] = c[r.idx].g[w];
      }
      return nz;
    }
  }
  return row_grad(r, x, M::n, idx, v);
}

// regularization_update! (ilqr_methods.jl:164-176)
template <class St>
__device__ __forceinline__ void reg_increase(const DevProblem* P, St& s) {
  const double f = P->o.bp_reg_increase_factor;
  s.drho = fmax(s.drho * f, f);
  s.rho = fmax(s.rho * s.drho, P->o.bp_reg_min);
  if (s.rho > P->o.bp_reg_max) s.flags |= TOG_TRAJ_MAX_REG;
}
template <class St>
__device__ __forceinline__ void reg_decrease(const DevProblem* P, St& s) {
  const double f = P->o.bp_reg_increase_factor;
  s.drho = fmin(s.drho / f, 1.0 / f);
  const double rd = s.rho * s.drho;
  s.rho = rd * (double)(rd > P->o.bp_reg_min);
}

__device__ __forceinline__ double lapy2(double x, double y) {  // LAPACK dlapy2
  const double xa = fabs(x), ya = fabs(y);
  const double w = fmax(xa, ya), z = fmin(xa, ya);
  if (z == 0.0) return w;
  const double t = z / w;
  return w * sqrt(1.0 + t * t);
}

}  // namespace tog
