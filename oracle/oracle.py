"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (oracle/tog_oracle.c).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg import this module,
as the checker; the product path (libtog.so) never does.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
LIB_LITERAL = HERE / "liboracle_literal.so"  # -DTOG_ORACLE_LITERAL: the reference's own arithmetic

_pkg = sys.modules.get("trajopt_amd")
if _pkg is None:  # pragma: no cover
    sys.path.insert(0, str(HERE.parent))
    import __graft_entry__  # noqa: E402

    _pkg = __graft_entry__.load_package()
abi = _pkg.abi

_lib = None
_lib_literal = None

FIELDS = {"X": abi.FIELD_X, "U": abi.FIELD_U, "Xbar": abi.FIELD_XBAR, "Ubar": abi.FIELD_UBAR, "K": abi.FIELD_K,
          "d": abi.FIELD_D, "A": abi.FIELD_A, "B": abi.FIELD_B, "S": abi.FIELD_S, "Sx": abi.FIELD_SX,
          "dV": abi.FIELD_DV, "lambda": abi.FIELD_LAMBDA, "mu": abi.FIELD_MU, "C": abi.FIELD_C,
          "x0": abi.FIELD_X0, "stats": abi.FIELD_STATS, "rho": abi.FIELD_RHO, "Q": abi.FIELD_Q}


def lib(literal=False):
    """The contract build (default) or, with ``literal``, the literal-arithmetic build of the oracle."""
    global _lib, _lib_literal
    if literal:
        if _lib_literal is None:
            _lib_literal = _load(LIB_LITERAL)
        return _lib_literal
    if _lib is None:
        _lib = _load(LIB)
    return _lib


def _load(path):
    if not path.exists():
        subprocess.run(["make"], cwd=HERE, check=True, capture_output=True)
    L = C.CDLL(str(path))
    vp, dp = C.c_void_p, C.POINTER(C.c_double)
    L.oc_create.restype = vp
    L.oc_create.argtypes = [C.POINTER(abi.tog_problem_desc), C.POINTER(abi.tog_options)]
    L.oc_destroy.argtypes = [vp]
    L.oc_set_state.argtypes = [vp, dp, dp, dp]
    L.oc_get.argtypes = [vp, C.c_int, dp]
    L.oc_set.argtypes = [vp, C.c_int, dp]
    L.oc_pmax.argtypes = [vp]
    L.oc_rollout_open_loop.argtypes = [vp]
    L.oc_slack_controls.argtypes = [vp]
    L.oc_rollout.argtypes = [vp, C.c_double]
    L.oc_jacobians.argtypes = [vp]
    L.oc_cost_expansion.argtypes = [vp, C.c_int, C.c_int]
    L.oc_backward.argtypes = [vp, C.c_int, dp]
    L.oc_forward.argtypes = [vp, C.c_int, C.c_double]
    L.oc_forward.restype = C.c_double
    L.oc_cost.argtypes = [vp, C.c_int]
    L.oc_cost.restype = C.c_double
    L.oc_cost_bar.argtypes = [vp, C.c_int]
    L.oc_cost_bar.restype = C.c_double
    L.oc_solve_ilqr.argtypes = [vp]
    L.oc_solve_al.argtypes = [vp]
    L.oc_update_constraints.argtypes = [vp]
    L.oc_max_violation.argtypes = [vp]
    L.oc_max_violation.restype = C.c_double
    L.oc_get_trace.argtypes = [vp, dp]
    L.oc_get_history.argtypes = [vp, C.c_int, dp]
    L.oc_discrete_f.argtypes = [C.c_int, C.c_int, dp, dp, dp, C.c_double]
    L.oc_continuous_f.argtypes = [C.c_int, dp, dp, dp]
    L.oc_discrete_jacobian.argtypes = [C.c_int, C.c_int, dp, dp, dp, C.c_double]
    L.oc_cond2.argtypes = [dp, C.c_int]
    L.oc_cond2.restype = C.c_double
    L.oc_qr_R.argtypes = [dp, dp, C.c_int, C.c_int]
    L.oc_solve_pn.argtypes = [vp, C.POINTER(abi.tog_pn_options), dp]
    L.oc_solve_batch.restype = C.c_int64
    L.oc_solve_batch.argtypes = [C.POINTER(abi.tog_problem_desc), C.POINTER(abi.tog_options), C.c_int, dp, dp,
                                 C.c_int64, C.c_int]
    L.oc_solve_batch_timed.restype = C.c_int64
    L.oc_solve_batch_timed.argtypes = [C.POINTER(abi.tog_problem_desc), C.POINTER(abi.tog_options), C.c_int, dp,
                                       dp, C.c_int64, C.c_int, C.POINTER(C.c_double)]
    return L


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def discrete_f(model, integ, x, u, dt):
    n = len(x)
    out = np.empty(n)
    lib().oc_discrete_f(model, integ, _dp(out), _dp(np.ascontiguousarray(x, float)),
                        _dp(np.ascontiguousarray(u, float)), dt)
    return out


def continuous_f(model, x, u):
    out = np.empty(len(x))
    lib().oc_continuous_f(model, _dp(out), _dp(np.ascontiguousarray(x, float)), _dp(np.ascontiguousarray(u, float)))
    return out


def discrete_jacobian(model, integ, x, u, dt):
    """n x (n+m+1) ForwardDiff Jacobian of the discrete map w.r.t. [x; u; dt]."""
    n, m = len(x), len(u)
    S = np.empty((n + m + 1, n))  # column-major n x L
    lib().oc_discrete_jacobian(model, integ, _dp(S), _dp(np.ascontiguousarray(x, float)),
                               _dp(np.ascontiguousarray(u, float)), dt)
    return S.T.copy()


def cond2(A):
    A = np.asfortranarray(A, dtype=float)
    return lib().oc_cond2(A.ctypes.data_as(C.POINTER(C.c_double)), A.shape[0])


def qr_R(P):
    P = np.asfortranarray(P, dtype=float).copy(order="F")
    rows, cols = P.shape
    R = np.zeros((cols, cols), order="F")
    lib().oc_qr_R(R.ctypes.data_as(C.POINTER(C.c_double)), P.ctypes.data_as(C.POINTER(C.c_double)), rows, cols)
    return np.array(R)


class OracleSolver:
    """Single-trajectory oracle solver for trajectory ``b`` of a (possibly batched) Problem."""

    def __init__(self, prob, opts, b=0, literal=False):
        self.L = lib(literal)
        self.prob = prob
        self.n, self.m, self.N = prob.model.n, prob.model.m, prob.N
        self.desc = prob.build_desc()
        self.opts = _pkg.to_tog_options(opts)
        self.al_requested = isinstance(opts, (_pkg.AugmentedLagrangianSolverOptions, _pkg.ALTROSolverOptions))
        self.mode = abi.MODE_AL if (self.al_requested and prob.is_constrained()) else abi.MODE_ILQR
        if self.al_requested and not prob.is_constrained():
            self.opts = _pkg.to_tog_options(opts.opts_uncon if hasattr(opts, "opts_uncon") else opts.opts_al.opts_uncon)
        self.s = self.L.oc_create(C.byref(self.desc.desc), C.byref(self.opts))
        self.pmax = self.L.oc_pmax(self.s)
        X = prob._X[b]
        self.L.oc_set_state(self.s, _dp(np.ascontiguousarray(prob.x0[b])), _dp(np.ascontiguousarray(prob._U[b])),
                           _dp(np.ascontiguousarray(X)) if np.isfinite(X).all() else C.cast(None, C.POINTER(C.c_double)))

    def __del__(self):
        try:
            self.L.oc_destroy(self.s)
        except Exception:
            pass

    def shape(self, name):
        n, m, N, P = self.n, self.m, self.N, max(self.pmax, 1)
        return {"X": (N, n), "U": (N - 1, m), "Xbar": (N, n), "Ubar": (N - 1, m), "K": (N - 1, n, m),
                "d": (N - 1, m), "A": (N - 1, n, n), "B": (N - 1, m, n), "S": (N, n, n), "Sx": (N, n),
                "dV": (2,), "lambda": (N, P), "mu": (N, P), "C": (N, P), "x0": (n,), "stats": (abi.NSTATS,),
                "rho": (2,), "Q": (N, n + m + n * n + m * m + m * n)}[name]

    def get(self, name):
        out = np.empty(self.shape(name))
        self.L.oc_get(self.s, FIELDS[name], _dp(out))
        if name in ("K", "A", "B", "S"):
            out = np.ascontiguousarray(np.swapaxes(out, -1, -2))
        return out

    def set(self, name, v):
        v = np.asarray(v, dtype=float)
        if name in ("K", "A", "B", "S"):
            v = np.swapaxes(v, -1, -2)
        v = np.ascontiguousarray(v.reshape(self.shape(name)))
        self.L.oc_set(self.s, FIELDS[name], _dp(v))

    # step level
    def rollout_open_loop(self):
        self.L.oc_rollout_open_loop(self.s)

    def rollout(self, alpha):
        return bool(self.L.oc_rollout(self.s, alpha))

    def slack_controls(self):
        self.L.oc_slack_controls(self.s)

    def jacobians(self):
        self.L.oc_jacobians(self.s)

    def update_constraints(self):
        self.L.oc_update_constraints(self.s)

    def cost_expansion(self, sqrt=False, al=False):
        return self.L.oc_cost_expansion(self.s, int(sqrt), int(al))

    def backward(self, sqrt=False):
        dV = np.empty(2)
        restarts = self.L.oc_backward(self.s, int(sqrt), _dp(dV))
        return dV, restarts

    def forward(self, J_prev, al=False):
        return self.L.oc_forward(self.s, int(al), float(J_prev))

    def cost(self, al=False):
        return self.L.oc_cost(self.s, int(al))

    def cost_bar(self, al=False):
        """cost of the last rollout's X̄, Ū"""
        return self.L.oc_cost_bar(self.s, int(al))

    def solve(self):
        if self.mode == abi.MODE_AL:
            return self.L.oc_solve_al(self.s)
        return self.L.oc_solve_ilqr(self.s)

    def max_violation(self):
        return self.L.oc_max_violation(self.s)

    def solve_pn(self, pn_opts):
        """solve!(prob, ProjectedNewtonSolver) (projected_newton.jl:6-20) on this trajectory's X, U;
        returns the TOG_PN_NSTATS statistics row."""
        out = np.zeros(abi.PN_NSTATS)
        rc = self.L.oc_solve_pn(self.s, C.byref(_pkg.to_tog_pn_options(pn_opts)), _dp(out))
        if rc != 0:
            raise ValueError(f"oc_solve_pn: unknown solve_type ({rc})")
        return out

    def history(self):
        """The solver.stats vectors of the last solve: inner records (n, 3) [cost, dJ, gradient] (iLQR
        record_iteration!, ilqr_methods.jl:77-89), outer records (n, 4) [iterations_inner, cost, c_max,
        penalty_max] (augmented_lagrangian_methods.jl:79-97), projected Newton records (n, 2) [cost, c_max]."""
        out = []
        for which, w in ((0, 3), (1, 4), (2, 2)):
            k = self.L.oc_get_history(self.s, which, C.cast(None, C.POINTER(C.c_double)))
            a = np.empty((k, w))
            if k:
                self.L.oc_get_history(self.s, which, _dp(a))
            out.append(a)
        return tuple(out)

    def trace(self):
        out = np.empty((4096, 6))
        n = self.L.oc_get_trace(self.s, _dp(out))
        return out[:n]


def solve_batch(prob, opts, nthreads=1, B=None, busy=False):
    """CPU baseline: solve ``B`` trajectories of ``prob`` with ``nthreads`` OpenMP threads.
    Returns the total number of iLQR step!s (and, with ``busy``, the summed per-trajectory solve
    seconds)."""
    desc = prob.build_desc()
    o = _pkg.to_tog_options(opts)
    al = isinstance(opts, (_pkg.AugmentedLagrangianSolverOptions, _pkg.ALTROSolverOptions)) and prob.is_constrained()
    B = prob.B if B is None else B
    x0 = np.ascontiguousarray(prob.x0[:B])
    U0 = np.ascontiguousarray(prob._U[:B])
    bt = C.c_double(0.0)
    steps = int(lib().oc_solve_batch_timed(C.byref(desc.desc), C.byref(o), abi.MODE_AL if al else abi.MODE_ILQR,
                                           _dp(x0), _dp(U0), B, nthreads, C.byref(bt)))
    return (steps, bt.value) if busy else steps


def solve_altro_infeasible(prob, opts, b=0):
    """Oracle restatement of ``solve!(prob, ::ALTROSolverOptions)`` from a given X
    (altro_methods.jl:2-124, infeasible.jl:2-99) for trajectory ``b``; returns (X, U, solver_inf,
    solver_feasible or None). Mirrors ``solvers._solve_altro_infeasible`` step for step."""
    m = prob.model.m
    pinf = _pkg.infeasible_problem(prob, opts.R_inf)
    si = OracleSolver(pinf, opts, b)
    si.slack_controls()
    si.solve()
    if opts.projected_newton:  # altro_methods.jl:31-39: phase 2 on the infeasible problem
        si.solve_pn(opts.opts_pn)
    X = si.get("X")
    U = si.get("U")[:, :m].copy()
    sf = None
    if opts.resolve_feasible_problem:
        p2 = prob.copy()
        p2._X[b] = np.nan if opts.dynamically_feasible_projection else X
        p2._U[b] = U
        sf = OracleSolver(p2, opts.opts_al, b)
        sf.solve()
        X, U = sf.get("X"), sf.get("U")
    return X, U, si, sf


def solve_altro_infeasible_min_time(prob, opts, b=0):
    """Oracle restatement of ``solve!(prob, ::ALTROSolverOptions)`` with an initial state trajectory and
    tf = 0 (altro_methods.jl:98-124): minimum_time_problem(infeasible_problem(prob)) -- the slacks from
    slack_controls on the infeasible problem, the time-step bounds on the first slack control as
    mintime_constraints combines them (minimum_time.jl:125-141) -- then process_results! (:56-95) with
    infeasible_to_feasible_problem (infeasible.jl:37-58: the feasible minimum-time problem, h and τ from the
    infeasible solve, projection! = the open-loop rollout) and the resolve. Returns (X[1:n], U[1:m], h,
    solver_inf, solver_feasible or None). Mirrors ``tog_solve_altro`` (csrc/tog_altro.cpp)."""
    n, m = prob.model.n, prob.model.m
    pinf = _pkg.infeasible_problem(prob, opts.R_inf)
    s0 = OracleSolver(pinf, opts, b)
    s0.slack_controls()
    pinf._U[b] = s0.get("U")
    pmt = _pkg.minimum_time_problem(pinf, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    si = OracleSolver(pmt, opts.opts_al, b)
    si.solve()
    if opts.projected_newton:  # altro_methods.jl:31-39: phase 2 on prob_altro
        si.solve_pn(opts.opts_pn)
    Xi, Ui = si.get("X"), si.get("U")
    X, U, h = Xi[:, :n].copy(), Ui[:, :m].copy(), Ui[:, -1].copy()
    p2 = prob.copy()
    p2._X[b], p2._U[b] = X, U
    pm2 = _pkg.minimum_time_problem(p2, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    pm2._U[b, :, m] = h
    pm2._X[b, :, n] = Xi[:, -1]
    pm2._X[b, 0, n] = 0.0
    if opts.dynamically_feasible_projection:
        pm2._X[b] = np.nan
    sf = None
    if opts.resolve_feasible_problem:
        sf = OracleSolver(pm2, opts.opts_al, b)
        sf.solve()
        Xf, Uf = sf.get("X"), sf.get("U")
        X, U, h = Xf[:, :n].copy(), Uf[:, :m].copy(), Uf[:, m].copy()
    return X, U, h, si, sf


def solve_altro_min_time(prob, opts, b=0):
    """Oracle restatement of ``solve!(prob, ::ALTROSolverOptions)`` for tf = 0 (altro_methods.jl:98-124,
    minimum_time.jl:2-34) for trajectory ``b``: returns (X[1:n], U[1:m], h, solver). Mirrors
    ``solvers._solve_altro_min_time``."""
    n, m = prob.model.n, prob.model.m
    pmt = _pkg.minimum_time_problem(prob, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    s = OracleSolver(pmt, opts.opts_al, b)
    s.solve()
    if opts.projected_newton:  # altro_methods.jl:31-39: phase 2 on the minimum-time problem
        s.solve_pn(opts.opts_pn)
    X, U = s.get("X"), s.get("U")
    return X[:, :n].copy(), U[:, :m].copy(), U[:, m].copy(), s


COST_MYCOST, COST_SOFT_OBSTACLE = 0, 1  # tog_oracle_cost.c example costs


def generic_cost_expand(cost_id, X, U=None, analytic=False):
    """oc_generic_cost_expand (tog_oracle_cost.c): GenericCost ℓ / ℓf and the expansion for count points;
    returns (J, Ex, Eu, Exx, Euu, Eux) with matrices column-major per point (the ABI's layout)."""
    import numpy as np

    L = lib()
    dp = C.POINTER(C.c_double)
    L.oc_generic_cost_expand.argtypes = [C.c_int, C.c_int, C.c_int, dp, dp, C.c_longlong] + [dp] * 6
    n, m = (2, 1) if cost_id == COST_MYCOST else (4, 2)
    X = np.ascontiguousarray(np.atleast_2d(np.asarray(X, dtype=np.float64)))
    cnt = X.shape[0]
    term = U is None
    mm = 0 if term else m
    U = np.zeros((cnt, 1)) if term else np.ascontiguousarray(np.atleast_2d(np.asarray(U, dtype=np.float64)))
    out = [np.zeros(cnt), np.zeros((cnt, n)), np.zeros((cnt, max(mm, 1))), np.zeros((cnt, n * n)),
           np.zeros((cnt, max(mm * mm, 1))), np.zeros((cnt, max(mm * n, 1)))]
    p = lambda a: a.ctypes.data_as(dp)
    rc = L.oc_generic_cost_expand(cost_id, int(analytic), int(term), p(X), p(U), cnt, *[p(a) for a in out])
    if rc != 0:
        raise ValueError("oc_generic_cost_expand failed")
    J, Ex, Eu, Exx, Euu, Eux = out
    Exx = Exx.reshape(cnt, n, n).swapaxes(1, 2)
    if term:
        return J, Ex, np.zeros((cnt, 0)), Exx, np.zeros((cnt, 0, 0)), np.zeros((cnt, 0, n))
    return J, Ex, Eu, Exx, Euu.reshape(cnt, m, m).swapaxes(1, 2), Eux.reshape(cnt, n, m).swapaxes(1, 2)
