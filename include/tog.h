/*
 * tog.h — C ABI of the MI355X-native batched iLQR / AL-iLQR hot path.
 *
 * This is the drop-in boundary for TrajectoryOptimization.jl's inner loop
 * (reference at /root/reference, cited as file:line). Everything here is
 * plain C: fp64 column-major arrays, int32/int64 sizes, int status codes,
 * no exceptions, no torch types. Every entry point is ccall/ctypes friendly.
 *
 * Layout of batched buffers (host side and device side are identical):
 *   x0 : (n, B)            x0[i + n*b]
 *   X  : (n, N, B)         X[i + n*(k + N*b)]          k = 0..N-1 (knot k+1 in Julia)
 *   U  : (m, N-1, B)       U[i + m*(k + (N-1)*b)]
 *   K  : (m, n, N-1, B)    column-major m x n block per knot
 *   d  : (m, N-1, B)
 *   A  : (n, n, N-1, B)    = ∇F[k].xx   (src/model.jl:341 partition :xx)
 *   Bm : (n, m, N-1, B)    = ∇F[k].xu
 *   S  : (n, n, N, B)      cost-to-go Hessian (std) or its upper-triangular
 *                          square-root factor (sqrt), src/solvers/ilqr/ilqr_solver.jl:104
 *   s  : (n, N, B)         cost-to-go gradient S[k].x
 *   lambda, mu, C : (pmax, N, B)  AL multipliers / penalties / constraint values
 */
#ifndef TOG_H
#define TOG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: tog_solve_altro / tog_altro_options, TOG_PROB_TF_MIN, TOG_NKERNELS = 4 (tog_profile_read fills 4
      entries), tog_solve's max_steps <= 0 = the tog_solve_budget default */
/* 4: iteration histories (tog_history_enable, TOG_FIELD_HIST_*), tog_solve_altro_ex / tog_altro_result,
      tog_altro_options.max_steps (was reserved), tog_get_pn_history, tog_batch_stats_begin / _end,
      tog_problem_desc.stage_costs (time-varying objectives) */
#define TOG_ABI_VERSION 4

/* ---------------------------------------------------------------- status */
enum tog_status_code {
  TOG_OK = 0,
  TOG_ERR_ARG = -1,        /* invalid argument (reference: ArgumentError, src/problem.jl:66-68,169-219) */
  TOG_ERR_DEVICE = -2,     /* HIP runtime failure                                                   */
  TOG_ERR_NOMEM = -3,
  TOG_ERR_UNSUPPORTED = -4 /* model / option combination not built                                  */
};

/* per-trajectory status bits (tog_status). Replace the reference's exceptions and @warn. */
enum tog_traj_flag {
  TOG_TRAJ_ACTIVE = 1 << 0,          /* still iterating                                         */
  TOG_TRAJ_CONVERGED = 1 << 1,       /* evaluate_convergence true (ilqr_methods.jl:139-162)     */
  TOG_TRAJ_MAX_ITERS = 1 << 2,       /* stats[:iterations] >= iterations                        */
  TOG_TRAJ_COST_INCREASED = 1 << 3,  /* error("Cost increased") forward_pass.jl:80-82           */
  TOG_TRAJ_COST_BLOWUP = 1 << 4,     /* J > max_cost_value, ilqr_methods.jl:25-28              */
  TOG_TRAJ_MAX_REG = 1 << 5,         /* @warn "Max regularization exceeded" ilqr_methods.jl:169 */
  TOG_TRAJ_SQRT_PD_FAIL = 1 << 6,    /* lowrankdowndate! PosDefException in the sqrt BP: like the
                                        reference's exception it ends the trajectory's solve (with
                                        BP_ABORTED; solve_b raises LinAlgError after the batch) */
  TOG_TRAJ_AL_CONVERGED = 1 << 7,    /* c_max < constraint_tolerance                            */
  TOG_TRAJ_AL_MAX_ITERS = 1 << 8,    /* AL outer loop exhausted                                 */
  TOG_TRAJ_SINGULAR = 1 << 9,        /* zero on the diagonal of the sqrt BP's Q.xx factor (the
                                        reference's SingularException -> pinv path; unreachable
                                        for PD cost Hessians)                     */
  TOG_TRAJ_BP_ABORTED = 1 << 10      /* more than TOG_BP_MAX_RESTARTS regularisation restarts in
                                        one backward pass: the trajectory stops (with MAX_REG).
                                        The reference would keep restarting (backward_pass.jl:52-62,
                                        125-136), e.g. forever on a NaN expansion.              */
};

/* Regularisation restarts one backward pass may take before the trajectory is stopped with
 * TOG_TRAJ_BP_ABORTED | TOG_TRAJ_MAX_REG (same cap in the oracle and every device kernel). The
 * trajectory keeps its X, U; K, d, ΔV of the aborted pass are not used. */
#define TOG_BP_MAX_RESTARTS 1000

/* ---------------------------------------------------------------- models */
enum tog_model_id {
  TOG_MODEL_DOUBLE_INTEGRATOR = 0, /* dynamics/double_integrator.jl:1-4   n=2  m=1 */
  TOG_MODEL_CARTPOLE = 1,          /* dynamics/cartpole.jl:9-36           n=4  m=1 */
  TOG_MODEL_QUADROTOR = 2,         /* dynamics/quadrotor.jl:10-71         n=13 m=4 */
  TOG_MODEL_CAR = 3,               /* dynamics/car.jl:3-8                 n=3  m=2 */
  TOG_MODEL_PENDULUM = 4,          /* dynamics/pendulum.jl:3-12           n=2  m=1 */
  TOG_MODEL_KUKA = 5,              /* src/model.jl:394-431 RBD Model(urdf) n=14 m=7 (include/tog_kuka.h) */
  TOG_MODEL_COUNT = 6,
  /* Model(f!, n, m) (src/model.jl:103-131) with user dynamics: a plugin loaded by tog_model_load,
     passed in tog_problem_desc.user_model */
  TOG_MODEL_USER = 100
};

enum tog_integrator {
  TOG_RK3 = 0, /* src/integration.jl:149-158 */
  TOG_RK4 = 1, /* src/integration.jl:115-125 */
  TOG_MIDPOINT = 2, /* explicit midpoint, src/integration.jl:26-33 (discretize_model(model, :midpoint)) */
  /* implicit schemes: a Newton solve per step to ||g||_2 <= 1e-12 (src/integration.jl:44-73 and
     :171-205); built for models with n <= 4 (double integrator, pendulum, car, cartpole), else
     tog_create returns TOG_ERR_UNSUPPORTED */
  TOG_RK3_IMPLICIT = 3,
  TOG_MIDPOINT_IMPLICIT = 4
};

/* ---------------------------------------------------------------- constraints */
enum tog_constraint_type {
  /* BoundConstraint(n,m; x_min,x_max,u_min,u_max, trim=true), src/constraints.jl:155-188.
     data = [x_max(n), x_min(n), u_max(m), u_min(m)]; ±INFINITY entries are trimmed. */
  TOG_CON_BOUND = 0,
  /* goal_constraint(xf), src/constraints.jl:299-304. Terminal equality. data = xf(count): rows
     x[1:count] - xf (the goal's inds; count 0 = n, count < n for a minimum-time state [x; τ]) */
  TOG_CON_GOAL = 1,
  /* `count` circle_constraint rows (src/utils.jl:140-144) on x[1],x[2]:
     c = -((x1-x0)^2 + (x2-y0)^2 - r^2). data = [x0,y0,r]*count. Stage inequality. */
  TOG_CON_CIRCLES = 2,
  /* `count` sphere_constraint rows (src/utils.jl:150-156) on x[1..3]:
     c = -((x1-x0)^2 + (x2-y0)^2 + (x3-z0)^2 - r^2). data = [x0,y0,z0,r]*count. */
  TOG_CON_SPHERES = 3,
  /* infeasible_constraints(n, m), src/constraints.jl:306-314: the n slack controls of an
     infeasible-start problem must vanish, c = u[m_model + i] (stage equality, n rows, no data).
     Only valid in a TOG_PROB_INFEASIBLE problem. */
  TOG_CON_INFEASIBLE = 4,
  /* Constraint{Inequality|Equality}(c!, n, m, p) with a user function (src/constraints.jl:85-89):
     count = p rows, data = [fid, equality (0/1), where (0 stage knots, 1 terminal knot, 2 both)];
     evaluated by the user model plugin's con(fid, c, x, u), Jacobian by dual numbers */
  TOG_CON_USER = 5,
  /* mintime_equality(n, m) (src/solvers/altro/minimum_time.jl:106-124): h_k - τ_k = 0, stage knots;
     count and data unused (TOG_PROB_MIN_TIME problems) */
  TOG_CON_MIN_TIME_EQ = 6
};

/* problem flags (tog_problem_desc.flags) */
enum tog_problem_flag {
  /* infeasible_problem(prob, R_inf) (src/solvers/altro/infeasible.jl:2-33): the model is
     add_slack_controls(model) (src/model.jl:761-779), x+ = f_d(x, u[1:m]) + u[m+1:m+n], so
     desc.m = m_model + n and R, H, r, the bound data are given for the augmented controls
     (R = blockdiag(R, R_inf I / dt), H and r zero-padded). */
  TOG_PROB_INFEASIBLE = 1,
  /* minimum_time_problem(prob, R_min_time, dt_max, dt_min) (src/solvers/altro/minimum_time.jl:2-34):
     model add_min_time_controls(model) (n = n_base + 1 states [x; τ], m = m_base + 1 controls [u; h],
     dt_k = h_k²), objective MinTimeCost with weight R_min_time (Q, R, H, q, r, Qf, qf the base cost's,
     zero-padded to n, m), constraints from mintime_constraints (h bounds in the BoundConstraint,
     TOG_CON_MIN_TIME_EQ rows). Std backward pass only (there is no sqrt MinTimeCost expansion). */
  TOG_PROB_MIN_TIME = 2,
  /* tf = 0 (src/problem.jl:174-178): the final time is free and dt is the initial time step. Accepted by
     tog_solve_altro only, which solves it as minimum_time_problem (ALTROSolverOptions R_minimum_time,
     dt_max, dt_min); tog_create refuses it. */
  TOG_PROB_TF_MIN = 4
};

typedef struct tog_constraint {
  int32_t type;       /* tog_constraint_type */
  int32_t count;      /* circles / spheres: their number; GOAL: rows x[1:count] (0 = n);
                         BOUND: 0 = trim=true (infinite bounds dropped), 1 = trim=false */
  const double* data; /* see tog_constraint_type */
} tog_constraint;

/* An ordered ConstraintSet (src/constraint_sets.jl:1). Order = order of the
   constraint vector C[k] (labels in insertion order, constraint_sets.jl:64-94). */
typedef struct tog_constraint_set {
  int32_t n_con;
  const tog_constraint* con;
} tog_constraint_set;

/* ---------------------------------------------------------------- problem */
/* Problem{T,Discrete} (src/problem.jl:37-72) with LQR/Quadratic objective
   (src/cost.jl:112-157, src/objective.jl:102-114) and per-knot constraint sets
   (src/constraint_sets.jl:157-206). One problem, B independent trajectories
   that differ in x0 and the initial controls U0. */
typedef struct tog_problem_desc {
  int32_t model;      /* tog_model_id                       */
  int32_t integrator; /* tog_integrator                     */
  int32_t n, m, N;    /* must match the model's n, m (m + n with TOG_PROB_INFEASIBLE) */
  int32_t flags;      /* tog_problem_flag bits (0 = plain problem) */
  int64_t batch;      /* B                                  */
  double dt;          /* prob.dt (tf > 0; min-time is out of scope) */
  /* stage QuadraticCost: 1/2 x'Qx + 1/2 u'Ru + q'x + r'u + c + u'Hx, times dt */
  const double* Q; /* n*n */
  const double* R; /* m*m */
  const double* H; /* m*n */
  const double* q; /* n   */
  const double* r; /* m   */
  double c;
  /* terminal QuadraticCost: 1/2 x'Qf x + qf'x + cf */
  const double* Qf; /* n*n */
  const double* qf; /* n   */
  double cf;
  /* constraints: sets[] table and knot_set[N] (-1 = empty set at that knot).
     knot_set[N-1] is the terminal set (evaluated with the terminal methods). */
  int32_t n_sets;
  int32_t reserved1;
  const tog_constraint_set* sets;
  const int32_t* knot_set;
  /* model == TOG_MODEL_USER: the loaded user model (tog_model_load), else ignored */
  const struct tog_model* user_model;
  /* TOG_PROB_MIN_TIME: MinTimeCost's R_min_time (ALTROSolverOptions.R_minimum_time) */
  double R_min_time;
  /* a time-varying Objective (Objective(costs::Vector{<:CostFunction}), src/objective.jl:12-29): NULL = the
     stage cost Q, R, H, q, r, c above at every stage knot; else (nc, N-1) column-major, per stage knot k
     [Q (n*n); R (m*m); H (m*n); q (n); r (m); c], nc = n*n + m*m + m*n + n + m + 1 (the fields above are
     then unused; the terminal cost stays Qf, qf, cf) */
  const double* stage_costs;
} tog_problem_desc;

/* ---------------------------------------------------------------- options */
/* Live fields of iLQRSolverOptions (src/solvers/ilqr/ilqr_solver.jl:7-81) and
   AugmentedLagrangianSolverOptions (src/solvers/augmented_lagrangian/augmented_lagrangian_solver.jl:8-66).
   tog_default_options() fills the reference defaults. */
typedef struct tog_options {
  double cost_tolerance;          /* 1e-4 */
  double gradient_norm_tolerance; /* 1e-5 */
  int32_t iterations;             /* 300  */
  int32_t dJ_counter_limit;       /* 10   */
  int32_t square_root;            /* 0    */
  int32_t bp_reg_type;            /* 0 = :control, 1 = :state */
  int32_t gradient_type;          /* 0 = :todorov, 1 = :feedforward, 2 = :ℓ2, 3 = :ℓinf */
  int32_t iterations_linesearch;  /* 20   */
  double line_search_lower_bound; /* 1e-8 */
  double line_search_upper_bound; /* 10   */
  double bp_reg_increase_factor;  /* 1.6  */
  double bp_reg_max;              /* 1e8  */
  double bp_reg_min;              /* 1e-8 */
  double bp_reg_fp;               /* 10   */
  double max_cost_value;          /* 1e8  */
  double max_state_value;         /* 1e8  */
  double max_control_value;       /* 1e8  */
  /* augmented Lagrangian */
  double al_cost_tolerance;                       /* 1e-4 */
  double al_cost_tolerance_intermediate;          /* 1e-3 */
  double al_gradient_norm_tolerance;              /* 1e-5 */
  double al_gradient_norm_tolerance_intermediate; /* 1e-5 */
  double constraint_tolerance;                    /* 1e-3 */
  double dual_min;                                /* -1e8 */
  double dual_max;                                /* 1e8  */
  double penalty_max;                             /* 1e8  */
  double penalty_initial;                         /* 1    */
  double penalty_scaling;                         /* 10   */
  int32_t al_iterations;                          /* 30   */
  int32_t kickout_max_penalty;                    /* 0    */
} tog_options;

/* solve modes */
enum tog_mode {
  TOG_MODE_ILQR = 0, /* solve!(prob, iLQRSolverOptions): objective only (ilqr_methods.jl:3-45)   */
  TOG_MODE_AL = 1    /* solve!(prob, AugmentedLagrangianSolverOptions) (augmented_lagrangian_methods.jl:2-31) */
};

/* fields for tog_get / tog_set */
enum tog_field {
  TOG_FIELD_X = 0,      /* (n,N,B)        prob.X                               */
  TOG_FIELD_U = 1,      /* (m,N-1,B)      prob.U                               */
  TOG_FIELD_XBAR = 2,   /* (n,N,B)        solver.X̄                            */
  TOG_FIELD_UBAR = 3,   /* (m,N-1,B)      solver.Ū                            */
  TOG_FIELD_K = 4,      /* (m,n,N-1,B)    solver.K                             */
  TOG_FIELD_D = 5,      /* (m,N-1,B)      solver.d                             */
  TOG_FIELD_A = 6,      /* (n,n,N-1,B)    solver.∇F[k].xx                      */
  TOG_FIELD_B = 7,      /* (n,m,N-1,B)    solver.∇F[k].xu                      */
  TOG_FIELD_S = 8,      /* (n,n,N,B)      solver.S[k].xx (needs TOG_BP_STORE_S) */
  TOG_FIELD_SX = 9,     /* (n,N,B)        solver.S[k].x  (needs TOG_BP_STORE_S) */
  TOG_FIELD_DV = 10,    /* (2,B)          last ΔV                              */
  TOG_FIELD_LAMBDA = 11,/* (pmax,N,B)                                          */
  TOG_FIELD_MU = 12,    /* (pmax,N,B)                                          */
  TOG_FIELD_C = 13,     /* (pmax,N,B)     constraint values at (X,U)           */
  TOG_FIELD_X0 = 14,    /* (n,B)                                               */
  TOG_FIELD_STATS = 15, /* (TOG_NSTATS,B) see tog_stat                         */
  TOG_FIELD_RHO = 16,   /* (2,B)          [ρ, dρ]                              */
  TOG_FIELD_Q = 17,     /* (nq,N,B)       cost expansion Q[k] from tog_cost_expansion, per knot
                           [Q.x (n); Q.u (m); Q.xx (n,n); Q.uu (m,m); Q.ux (m,n)], nq = n+m+n²+m²+mn;
                           the terminal knot has Q.u = Q.uu = Q.ux = 0. Valid until the next
                           backward pass (the buffer doubles as its restart-replay scratch). */
  /* iteration histories (tog_history_enable; read-only). Records are written in solve order since
     tog_solve_init; a record past the capacity is counted but not stored. */
  TOG_FIELD_HIST_INNER = 18, /* (3,cap,B) the iLQR solver's record_iteration! (ilqr_methods.jl:77-89):
                                per record [stats[:cost], stats[:dJ], stats[:gradient]]. In an AL solve the
                                inner solves follow each other (each opens with its (J_prev, Inf) record);
                                TOG_FIELD_HIST_OUTER's iterations_inner splits them (stats_uncon). */
  TOG_FIELD_HIST_OUTER = 19, /* (4,al_iterations+1,B) the AL solver's record_iteration!
                                (augmented_lagrangian_methods.jl:79-97): per outer record
                                [iterations_inner, cost, c_max, penalty_max]; record 0 is the initial one */
  TOG_FIELD_HIST_COUNT = 20  /* (2,B) records written: [inner, outer] */
};

/* per-trajectory statistics row (TOG_FIELD_STATS), all stored as double */
enum tog_stat {
  TOG_STAT_J = 0,           /* current cost (J_prev of the inner loop)              */
  TOG_STAT_DJ = 1,          /* last dJ                                              */
  TOG_STAT_GRADIENT = 2,    /* last gradient (gradient_type's measure)              */
  TOG_STAT_ITERATIONS = 3,  /* iLQR stats[:iterations] (includes initial record)    */
  TOG_STAT_ZERO_COUNT = 4,  /* dJ_zero_counter                                      */
  TOG_STAT_ALPHA = 5,       /* last accepted step (logged 2*alpha)                  */
  TOG_STAT_Z = 6,           /* last line-search ratio                               */
  TOG_STAT_C_MAX = 7,       /* max_violation(solver)                                */
  TOG_STAT_AL_ITER = 8,     /* AL outer iteration counter                           */
  TOG_STAT_TOTAL_STEPS = 9, /* iLQR step!s executed in total                        */
  TOG_STAT_LS_TRIALS = 10,  /* rollouts evaluated in the last forward pass          */
  TOG_STAT_BP_RESTARTS = 11,/* regularisation restarts in the last backward pass    */
  TOG_STAT_FLAGS = 12,      /* tog_traj_flag bits                                   */
  TOG_STAT_PENALTY_MAX = 13,/* max μ                                                */
  TOG_NSTATS = 14
};

/* backward-pass flags */
enum tog_bp_flag {
  TOG_BP_STORE_S = 1 /* write S[k].xx, S[k].x for every knot (test/inspection only) */
};

typedef struct tog_handle tog_handle;

/* ---------------------------------------------------------------- API */
int32_t tog_version(void);

/* ---------------------------------------------------------------- user models (plugins)
   Replaces Model(f!, n, m) (src/model.jl:103-131, continuous dynamics from a user function, its
   Jacobian by ForwardDiff src/model.jl:491-522). The user's f!(ẋ, x, u), written once as a C++
   template over the scalar type (double and the dual numbers of the Jacobian kernel), is compiled
   with hipcc for gfx950 against csrc/tog_plugin.hpp into a shared object that instantiates every
   kernel of the path for it (and for its infeasible-start variant, add_slack_controls
   src/model.jl:761-779). tog_model_load dlopens it and checks its layout fingerprint against
   this library's. */
typedef struct tog_model tog_model;
int32_t tog_model_load(const char* path, tog_model** out);
int32_t tog_model_dims(const tog_model* model, int32_t* n, int32_t* m);
int32_t tog_model_free(tog_model* model); /* after every handle built on it is destroyed */
/* ---------------------------------------------------------------- generic costs (plugins)
   Replaces GenericCost(ℓ, ℓf, n, m) / GenericCost(ℓ, ℓf, grad, hess, n, m) (src/cost.jl:239-287),
   its stage_cost (src/cost.jl:324-325) and cost_expansion! (src/cost.jl:327-345; ForwardDiff gradient
   and Hessian of auto_expansion_function src/cost.jl:289-322). The user's ℓ(x, u) and ℓf(xN), written
   once as C++ templates over the scalar type, are compiled with hipcc for gfx950 against
   csrc/tog_cost_plugin.hpp (TOG_COST_PLUGIN); tog_generic_cost_load dlopens the plugin and checks its
   fingerprint. tog_generic_cost_expand evaluates `count` points at once: X (n, count), U (m, count)
   column-major (U unused when terminal); out J (count) = ℓ, Ex (n, count) = E.x, Eu (m, count) = E.u,
   Exx (n, n, count) = E.xx, Euu (m, m, count) = E.uu, Eux (m, n, count) = E.ux (terminal: J, Ex, Exx;
   the others may be NULL). Host pointers, synchronous on `device`; the _device variant takes device
   pointers and enqueues on `hip_stream` (NULL = the default stream). The reference's solvers never
   call a GenericCost (its stage_cost has no dt method), so it is not a solver cost here either. */
typedef struct tog_generic_cost tog_generic_cost;
int32_t tog_generic_cost_load(const char* path, tog_generic_cost** out);
int32_t tog_generic_cost_dims(const tog_generic_cost* cost, int32_t* n, int32_t* m);
int32_t tog_generic_cost_expand(const tog_generic_cost* cost, int32_t device, int32_t terminal, const double* X, const double* U,
                        int64_t count, double* J, double* Ex, double* Eu, double* Exx, double* Euu, double* Eux);
int32_t tog_generic_cost_expand_device(const tog_generic_cost* cost, int32_t terminal, const double* X, const double* U,
                               int64_t count, double* J, double* Ex, double* Eu, double* Exx, double* Euu,
                               double* Eux, void* hip_stream);
int32_t tog_generic_cost_free(tog_generic_cost* cost);
/* dynamics_bias(state) at x = [q; v] for RBD models (TOG_MODEL_KUKA): c(q, v) into tau[m].
   Replaces RigidBodyDynamics.dynamics_bias as used by hold_trajectory (dynamics/kuka.jl:117-132).
   Host evaluation; TOG_ERR_UNSUPPORTED for analytical models. */
int tog_dynamics_bias(int32_t model, const double* x, double* tau);
int32_t tog_device_count(void);
void tog_default_options(tog_options* opts);

/* AbstractSolver(prob, opts) — src/solvers.jl:47-94, ilqr_solver.jl:118-144,
   augmented_lagrangian_solver.jl:120-140. Allocates every device buffer. */
int32_t tog_create(const tog_problem_desc* desc, const tog_options* opts, int32_t device,
                   tog_handle** out);
/* One handle over several devices (one process driving ndev GPUs, e.g. the single Julia process):
   the batch is split into ndev contiguous slices, one device each (sizes differ by at most one,
   earlier devices take the remainder). Every entry point fans out over the slices and host arrays
   are split/gathered along the batch axis; tog_batch_stats reduces over devices. The per-device
   pointers of tog_get_device_ptr / tog_batch_stats_device and tog_set_stream are
   TOG_ERR_UNSUPPORTED on such a handle. devices may repeat (several slices on one GPU). */
int32_t tog_create_multi(const tog_problem_desc* desc, const tog_options* opts, const int32_t* devices,
                         int32_t ndev, tog_handle** out);
int32_t tog_destroy(tog_handle* h);
/* use an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream */
int32_t tog_set_stream(tog_handle* h, void* hip_stream);
int32_t tog_synchronize(tog_handle* h);

/* initial_controls!/set_x0!/initial_states! (src/problem.jl:149-160).
   X may be NULL: then X is set to NaN (empty_state, src/problem.jl:232). Host pointers. */
int32_t tog_set_state(tog_handle* h, const double* x0, const double* U, const double* X);
/* copy a field host->device / device->host (host pointers, sizes per tog_field) */
int32_t tog_set(tog_handle* h, int32_t field, const double* in);
int32_t tog_get(tog_handle* h, int32_t field, double* out);
/* same, device pointers (no host staging) — for torch / RCCL interop */
int32_t tog_get_device_ptr(tog_handle* h, int32_t field, void** dptr);
int32_t tog_dims(tog_handle* h, int64_t* out6); /* [n, m, N, B, pmax, mode] */
/* Per-trajectory iteration histories: the reference's solver.stats vectors (ilqr_methods.jl:77-89,
   augmented_lagrangian_methods.jl:79-97), recorded on the device as the solve runs (one store per
   iteration) and read with tog_get(TOG_FIELD_HIST_*). capacity = inner records kept per trajectory
   (an AL solve records at most al_iterations x (iterations + 1)); 0 turns recording off (the default). */
int32_t tog_history_enable(tog_handle* h, int32_t capacity);

/* ---- step level (exported because tests and callers use them:
        src/TrajectoryOptimization.jl:82-95, test/sqrt_bp_tests.jl:27-37) ---- */
/* rollout!(prob) src/rollout.jl:25-31: open-loop rollout of trajectories whose X is non-finite */
int32_t tog_rollout_open_loop(tog_handle* h);
/* jacobian!(prob, solver) src/solvers.jl:126 -> src/model.jl:301-306 */
int32_t tog_jacobians(tog_handle* h);
/* update_constraints! + update_active_set! (constraint_sets.jl:221-260) at (X,U) */
int32_t tog_update_constraints(tog_handle* h);
/* cost(obj, X, U, dt) (objective.jl:40-48) or AL cost (augmented_lagrangian_methods.jl:298-313);
   al != 0 selects the AL objective. J_out: (B) host pointer */
int32_t tog_cost(tog_handle* h, int32_t al, double* J_out);
/* cost_expansion! + backwardpass! (ilqr_methods.jl:55-62, backward_pass.jl:1-169).
   sqrt selects _backwardpass_sqrt!; al selects the AL objective; flags = tog_bp_flag.
   Uses and updates the per-trajectory ρ, dρ. dV_out: (2,B) host or NULL. */
int32_t tog_backward_pass(tog_handle* h, int32_t sqrt, int32_t al, int32_t flags, double* dV_out);
/* cost_expansion!(prob, solver) (ilqr_methods.jl:55-62 -> objective.jl:51-94, cost.jl:183-198; AL:
   augmented_lagrangian_methods.jl:186-276) at (X, U) into TOG_FIELD_Q, for inspection and for
   tests that call it apart from the backward pass (test/sqrt_bp_tests.jl:27-37). sqrt selects
   cost_expansion_sqrt (Q.xx, Q.uu hold upper Cholesky factors); al adds the AL terms from the
   constraint values C last evaluated (tog_update_constraints / a cost evaluation). tog_backward_pass
   performs the same expansion fused, knot by knot, and does not read this field. */
int32_t tog_cost_expansion(tog_handle* h, int32_t sqrt, int32_t al);
/* solve!(prob, iLQRSolver) / solve!(prob, AugmentedLagrangianSolver) to completion:
   tog_solve(h, TOG_MODE_ILQR | TOG_MODE_AL, 0), i.e. with the tog_solve_budget step budget */
int32_t tog_solve_ilqr(tog_handle* h);
int32_t tog_solve_al(tog_handle* h);
/* forwardpass! (forward_pass.jl:5-85) from the stored ΔV; J_prev (B) host pointer;
   J_out (B) host or NULL. Writes X̄, Ū. */
int32_t tog_forward_pass(tog_handle* h, int32_t al, const double* J_prev, double* J_out);
/* rollout!(prob, solver, α) (src/rollout.jl:2-23) for every trajectory; ok_out (B) int32 or NULL */
int32_t tog_rollout(tog_handle* h, double alpha, int32_t* ok_out);

/* slack_controls(prob) (src/solvers/altro/infeasible.jl:63-80) for a TOG_PROB_INFEASIBLE handle:
   from x0, the state trajectory X and the model controls U[1:m], writes the slack controls
   U[m+1:m+n] that make X dynamically feasible (x_{k+1} = f_d(x_k, u_k) + s_k). Device side, in
   place; TOG_ERR_ARG on a plain handle. */
int32_t tog_slack_controls(tog_handle* h);

/* ---- solve level ---- */
/* initialise the per-trajectory solve state machine (reset!, λ=0, μ=μ0, initial rollout, J) */
int32_t tog_solve_init(tog_handle* h, int32_t mode);
/* advance every active trajectory by `nsteps` iLQR step!s (AL outer updates happen in between
   on the trajectories whose inner loop converged). Asynchronous: no host sync. */
int32_t tog_solve_step(tog_handle* h, int32_t nsteps);
/* number of trajectories still active + batch sums; blocking. out3 = [n_active, Σ J, max c_max] */
int32_t tog_batch_stats(tog_handle* h, double* out3);
/* batch stats into a device buffer of 3 doubles (stream-ordered, no host sync) */
int32_t tog_batch_stats_device(tog_handle* h, void* dptr3);
/* the stopping check without a device bubble: _begin enqueues the batch statistics and their copy into
   a pinned host buffer on the handle's stream (no wait); _end waits for that copy only, so steps enqueued
   in between keep the device busy while the host waits. One check may be outstanding per handle. Same
   out3 as tog_batch_stats, which also updates the handle's tail-mode hint. */
int32_t tog_batch_stats_begin(tog_handle* h);
int32_t tog_batch_stats_end(tog_handle* h, double* out3);
/* counter of step!s executed since tog_solve_init (device side, read blocking) */
int32_t tog_total_steps(tog_handle* h, int64_t* out);
/* full solves: run until no trajectory is active (or max_steps batch steps; max_steps <= 0: the
   tog_solve_budget default, which lets every trajectory reach its own iteration limit) */
int32_t tog_solve(tog_handle* h, int32_t mode, int32_t max_steps);
/* default batch-step budget of tog_solve: (iterations (x al_iterations) + 1) x the line-search rounds
   an iteration may take when its trials are spread over batch steps (ceil(nc / 8) for batches large
   enough to pend). Returns the budget (> 0) or a negative error code. */
int32_t tog_solve_budget(tog_handle* h, int32_t mode);
/* per-trajectory tog_traj_flag bits; flags_out: (B) int32 */
int32_t tog_status(tog_handle* h, int32_t* flags_out);

/* ---- ALTRO phase 2: projected Newton (src/solvers/direct/projected_newton.jl) ---- */
/* ProjectedNewtonSolverOptions (src/solvers/direct/direct_solvers.jl:14-30); tog_default_pn_options
   fills the reference defaults. solve_type :feasible (the default): newton_step! returns after
   projection_solve! (projected_newton.jl:518-520); :optimal adds multiplier_projection!, solveKKT_Shur and
   line_search (:522-546), not built on minimum-time problems (TOG_ERR_UNSUPPORTED). */
typedef struct tog_pn_options {
  int32_t n_steps;              /* 1                                                          */
  int32_t solve_type;           /* 0 = :feasible, 1 = :optimal                                */
  double active_set_tolerance;  /* 1e-3: inequality rows with c >= -tol are projected         */
  double feasibility_tolerance; /* 1e-6                                                       */
} tog_pn_options;
void tog_default_pn_options(tog_pn_options* opts);

/* per-trajectory projected-Newton statistics row (tog_solve_pn out), all double */
enum tog_pn_stat {
  TOG_PN_VIOL = 0,        /* last viol of projection_solve! (active rows incl. dynamics, Inf norm) */
  TOG_PN_C_MAX = 1,       /* max_violation(prob) after the solve (record_iteration!)           */
  TOG_PN_J = 2,           /* cost(prob) after the solve                                         */
  TOG_PN_PROJECTIONS = 3, /* _projection_solve! calls                                           */
  TOG_PN_LINESEARCHES = 4,/* _projection_linesearch! calls                                      */
  TOG_PN_REFINEMENTS = 5, /* reg_solve refinement iterations, in total                          */
  TOG_PN_STEPS = 6,       /* newton steps taken (solver.stats[:iterations])                     */
  TOG_PN_NSTATS = 7
};
/* The reference's _projection_linesearch! evaluates `count += a` (Int + BitVector, a MethodError)
   when its first trial does not reduce the violation (projected_newton.jl:273-277): such a
   trajectory stops with this flag and keeps the last accepted iterate. */
#define TOG_TRAJ_PN_ERROR (1 << 11)
/* The device's projected Newton blocks hold at most 64 rows (n + the rows active at a knot, a row per lane of
   a wave; the stride is min(n + pmax, 64)): a trajectory whose active set outgrows them stops with
   TOG_TRAJ_PN_ERROR | TOG_TRAJ_PN_BLOCK and keeps its last iterate. A device limit, not the reference's. */
#define TOG_TRAJ_PN_BLOCK (1 << 12)

/* solve!(prob, ProjectedNewtonSolver(prob, opts)) (projected_newton.jl:6-20) on every trajectory's
   current X, U (in place): n_steps newton steps of the feasible projection, each
   projection_solve! -> _projection_solve! (Jacobians of the dynamics and of the active
   constraints, S = Y H⁻¹ Yᵀ with H the diagonal of the cost Hessian, a block-tridiagonal Cholesky
   of S + 1e-2 I, chord-method line searches with reg_solve refinement to |r| < 1e-8).
   out: (TOG_PN_NSTATS, B) host pointer or NULL. */
int32_t tog_solve_pn(tog_handle* h, const tog_pn_options* opts, double* out);
/* solver_pn.stats[:cost] and [:c_max] (record_iteration!, projected_newton.jl:23-29) of the last tog_solve_pn:
   out (2, n_steps, B), per newton step [cost, c_max] (NaN after a trajectory's last step); steps_out (B) the
   records each trajectory made (stats[:iterations]) or NULL. */
int32_t tog_get_pn_history(tog_handle* h, double* out, int32_t* steps_out);

/* ---- ALTRO (src/solvers/altro/altro_methods.jl:2-124) ---- */
/* ALTROSolverOptions (src/solvers/altro/altro_solver.jl:6-65), its live fields; tog_default_altro_options
   fills the reference defaults. opts_al is AugmentedLagrangianSolverOptions with its opts_uncon. */
typedef struct tog_altro_options {
  tog_options opts_al;
  double R_inf;                         /* 1.0   infeasible_problem(prob, R_inf)                      */
  double R_minimum_time;                /* 1.0   minimum_time_problem                                 */
  double dt_max;                        /* 1.0                                                        */
  double dt_min;                        /* 1e-3                                                       */
  double projected_newton_tolerance;    /* 1e-3  AL constraint tolerance before projected Newton      */
  int32_t dynamically_feasible_projection; /* 1 */
  int32_t resolve_feasible_problem;     /* 1 */
  int32_t projected_newton;             /* 0 */
  int32_t max_steps;                    /* batch-step budget of each AL solve (tog_solve's max_steps;
                                           0 = the tog_solve_budget default)                         */
  tog_pn_options opts_pn;
} tog_altro_options;
void tog_default_altro_options(tog_altro_options* opts);
/* solve!(prob, ALTROSolverOptions) (altro_methods.jl:2-53): altro_problem (:98-124) transforms `desc`, the
   original problem (flags 0 or TOG_PROB_TF_MIN), into the infeasible-start problem when X holds an initial
   state trajectory (X not all NaN at the first knot, every trajectory of the batch or none;
   infeasible_problem, infeasible.jl:2-33) or into the minimum-time problem when TOG_PROB_TF_MIN is set
   (minimum_time_problem, minimum_time.jl:2-34); runs the AL solve on `device` (projected Newton after it
   when opts->projected_newton), and process_results! (:56-95) writes the model states and controls back:
   X (n, N, B) in/out (NULL: no initial trajectory), U (m, N-1, B) in/out, h (N-1, B) the time steps of a
   minimum-time solve (dt_k = h_k^2) or NULL. With resolve_feasible_problem the infeasible solve is followed
   by the feasible problem's solve from its controls. stats (TOG_NSTATS, B): the AL phase's statistics
   (the infeasible / minimum-time problem's solve); stats_resolve (TOG_NSTATS, B): the feasible resolve;
   stats_pn (TOG_PN_NSTATS, B): projected Newton; each may be NULL. Host pointers, blocking. A trajectory
   whose forward pass reported TOG_TRAJ_COST_INCREASED (the reference's error) carries the flag in its
   stats row. Projected Newton runs on the infeasible-start problem too (models with n + m + n <= 24). An
   initial state trajectory with TOG_PROB_TF_MIN solves minimum_time_problem(infeasible_problem(prob)) (the
   pendulum, car, double integrator and cartpole), then the feasible minimum-time resolve. Projected Newton
   runs on minimum-time problems too (its H diagonal from MinTimeCost's hessian! at each newton step's X, U;
   models with n + m <= 24 after the transforms, larger ones return TOG_ERR_UNSUPPORTED). */
int32_t tog_solve_altro(const tog_problem_desc* desc, const tog_altro_options* opts, int32_t device,
                        const double* x0, double* X, double* U, double* h, double* stats, double* stats_resolve,
                        double* stats_pn);

/* What solve!(prob, ALTROSolverOptions) returns (altro_methods.jl:40-52, ALTROSolver altro_solver.jl:70-94):
   solver.stats[:time], [:time_al], [:time_pn]; solver.solver_al.stats (the AL phase: the infeasible or
   minimum-time problem's solve) as summary rows and iteration histories; solver.solver_pn.stats. Inputs
   are the capacities and output buffers (each pointer may be NULL); the times and the handle are outputs. */
typedef struct tog_altro_result {
  int32_t inner_capacity;  /* in: inner records per trajectory in hist_inner (0: no histories)            */
  int32_t keep_handle;     /* in: 1 = hand the AL phase's handle (solver_al's buffers: K, d, λ, μ, ...) back
                              in `handle` instead of destroying it; the caller tog_destroys it            */
  double* stats;           /* (TOG_NSTATS, B) AL phase                                                   */
  double* stats_resolve;   /* (TOG_NSTATS, B) the feasible resolve of an infeasible start                */
  double* stats_pn;        /* (TOG_PN_NSTATS, B) projected Newton                                        */
  double* hist_inner;      /* (3, inner_capacity, B) AL phase, TOG_FIELD_HIST_INNER                       */
  double* hist_outer;      /* (4, al_iterations + 1, B) AL phase, TOG_FIELD_HIST_OUTER (AL solves)        */
  double* hist_count;      /* (2, B) TOG_FIELD_HIST_COUNT                                                 */
  double* hist_pn;         /* (2, opts_pn.n_steps, B) solver_pn.stats [:cost, :c_max] per newton step     */
  double time, time_al, time_pn; /* out: seconds (wall clock of the whole call, the AL phase, projected Newton) */
  tog_handle* handle;      /* out: see keep_handle (NULL otherwise)                                       */
} tog_altro_result;
/* tog_solve_altro with the solver's statistics (tog_solve_altro = this with only the three stats rows).
   A trajectory whose AL phase ends with the reference's exceptions (TOG_TRAJ_COST_INCREASED,
   TOG_TRAJ_SQRT_PD_FAIL) is not resolved and not projected: its X, U are what the exception would leave
   (the AL phase's for a feasible start; the caller's inputs for an infeasible or minimum-time start,
   whose AL phase ran on a copy of the problem). */
int32_t tog_solve_altro_ex(const tog_problem_desc* desc, const tog_altro_options* opts, int32_t device,
                           const double* x0, double* X, double* U, double* h, tog_altro_result* res);

/* per-kernel timing with HIP events recorded on the handle's stream around every launch issued by
   tog_solve_step (used by bench.py for the live roofline). */
enum tog_kernel_id {
  TOG_KERNEL_JACOBIAN = 0,
  TOG_KERNEL_BACKWARD = 1,
  TOG_KERNEL_FORWARD = 2,
  TOG_KERNEL_EXPANSION = 3, /* knot-parallel cost expansion ahead of the team backward pass */
  TOG_NKERNELS = 4
};
int32_t tog_profile(tog_handle* h, int32_t enable);
/* blocking: total milliseconds and launch counts per tog_kernel_id since tog_profile(h, 1) */
int32_t tog_profile_read(tog_handle* h, double* total_ms, int64_t* launches);

/* human readable message for the last error on this thread */
const char* tog_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* TOG_H */
