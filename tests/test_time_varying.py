"""Time-varying objectives: ``Objective(costs)`` with a cost of its own at every knot (src/objective.jl:15-29;
cost(obj, Z) sums stage_cost(obj[k], x_k, u_k, dt_k) over the knots, src/objective.jl:55-63).

The device reads knot k's [Q; R; H; q; r; c] (and the square-root factors of Q dt, R dt) from the per-knot
table tog_problem_desc.stage_costs (DevProblem::kc, cost_at in csrc/tog_device.hpp); the oracle indexes the
same table (oracle/tog_oracle.c stage_cost / expansion_stage). The oracle is pinned two ways: its cost of a
time-varying objective equals the host formula of src/cost.jl:171-198 summed over the knots, and a table whose
rows are all the shared cost solves bit for bit like the shared cost. The ``gpu`` tests hold libtog.so to the
oracle (X, U within 1e-6 and equal iteration counts; in fact bitwise under the arithmetic contract) for
iLQR (std and sqrt), AL, ALTRO infeasible start (tog_altro.cpp transforms each knot's cost), minimum time and
projected Newton (per-knot Hessian weights, tog_pn.hpp pn_wx / pn_wu).
"""
import math
import os

import numpy as np
import pytest

TOL_SOLVE = 1e-6


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def ramp_objective(tog, Q, R, Qf, xf, N, cross=0.0, seed=0):
    """LQRCost(Q w_k, R v_k, xf) per knot (weights rising along the horizon), optionally with a cross term
    H_k = cross * (random) and a non-diagonal Q_k (then the kernels take the dense-cost path)."""
    rng = np.random.default_rng(seed)
    n, m = Q.shape[0], R.shape[0]
    costs = []
    for k in range(N - 1):
        w = 0.5 + 1.5 * k / (N - 2)
        v = 2.0 - 1.0 * k / (N - 2)
        Qk, Rk = w * Q, v * R
        if cross:
            A = rng.standard_normal((n, n))
            Qk = Qk + cross * (A @ A.T) / n
        c = tog.LQRCost(Qk, Rk, xf)
        if cross:
            H = cross * 0.1 * rng.standard_normal((m, n))
            c = tog.QuadraticCost(c.Q, c.R, H, c.q, c.r, c.c)
        costs.append(c)
    return tog.Objective(costs + [tog.LQRCostTerminal(Qf, xf)])


def with_objective(tog, prob, obj):
    p = tog.Problem(prob.model, obj, prob._U.copy(), constraints=prob.constraints, x0=prob.x0.copy(), xf=prob.xf,
                    N=prob.N, dt=prob.dt)
    p._X[...] = prob._X
    return p


def cartpole_varying(tog, B=4, cross=0.0):
    prob, opts = tog.Problems.config_cartpole(B=B)
    st, term = prob.obj.stage, prob.obj.terminal
    obj = ramp_objective(tog, st.Q, st.R, term.Q, prob.xf, prob.N, cross=cross)
    return with_objective(tog, prob, obj), opts


def quadrotor_varying(tog, B=3):
    prob, opts = tog.Problems.config_quadrotor(B=B)
    st, term = prob.obj.stage, prob.obj.terminal
    obj = ramp_objective(tog, st.Q, st.R, term.Q, prob.xf, prob.N)
    return with_objective(tog, prob, obj), opts


def solve_and_compare(tog, oracle, prob, opts, env=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        gp = prob.copy()
        solver = tog.solve_b(gp, opts)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert rel(gp._X[b], o.get("X")) < TOL_SOLVE and rel(gp._U[b], o.get("U")) < TOL_SOLVE, b
        assert steps == int(solver.stats["iterations_total"][b]), b
    return gp, solver


# ----------------------------------------------------------------------------- CPU: host + oracle


def test_objective_table_layout(tog):
    """An LQRObjective shares one cost (no table); distinct per-knot costs give the (N-1, nc) table with
    each row [vec(Q); vec(R); vec(H); q; r; c], matrices column-major."""
    n, m, N = 3, 2, 6
    xf = np.arange(n, dtype=float)
    assert tog.LQRObjective(np.eye(n), np.eye(m), np.eye(n), xf, N).stage_table(m) is None
    obj = ramp_objective(tog, np.eye(n), np.eye(m), np.eye(n), xf, N, cross=0.5)
    assert obj.varying
    T = obj.stage_table(m)
    assert T.shape == (N - 1, n * n + m * m + m * n + n + m + 1)
    for k in range(N - 1):
        c = obj[k]
        o = 0
        for A in (c.Q, c.R, c.H):
            sz = A.size
            assert np.array_equal(T[k, o:o + sz].reshape(A.shape[::-1]).T, A)
            o += sz
        assert np.array_equal(T[k, o:o + n], c.q) and np.array_equal(T[k, o + n:o + n + m], c.r)
        assert T[k, -1] == c.c
    # the descriptor carries the table
    prob, _ = tog.Problems.config_cartpole(B=1)
    pv = with_objective(tog, prob, ramp_objective(tog, prob.obj.stage.Q, prob.obj.stage.R, prob.obj.terminal.Q,
                                                  prob.xf, prob.N))
    assert bool(pv.build_desc().desc.stage_costs) and not bool(prob.build_desc().desc.stage_costs)


def test_oracle_cost_is_the_sum_over_knots(tog, oracle):
    """cost(obj, Z) (src/objective.jl:55-63) of a time-varying objective: the oracle's J equals the host
    formula stage_cost(obj[k], x, u) dt (src/cost.jl:171-198) summed over the knots, plus the terminal."""
    prob, opts = cartpole_varying(tog, B=1, cross=0.3)
    rng = np.random.default_rng(4)
    X = rng.standard_normal(prob._X[0].shape)
    U = rng.standard_normal(prob._U[0].shape)
    o = oracle.OracleSolver(prob, opts, b=0)
    o.set("X", X)
    o.set("U", U)
    J = o.cost(False)
    ref = sum(prob.obj[k].stage_cost(X[k], U[k], prob.dt) for k in range(prob.N - 1))
    ref += prob.obj.terminal.stage_cost(X[-1])
    assert abs(J - ref) <= 1e-12 * abs(ref)


def test_oracle_equal_rows_solve_like_the_shared_cost(tog, oracle):
    """A table whose rows all hold the shared cost goes through the per-knot path and solves bit for bit
    like the shared cost (the table's indexing, the per-knot square-root factors)."""
    prob, opts = tog.Problems.config_quadrotor(B=1)
    pt = prob.copy()
    pt.obj = tog.Objective(list(prob.obj.cost))
    pt.obj.varying = True  # force the table
    assert pt.obj.stage_table(4).shape[0] == prob.N - 1
    a = oracle.OracleSolver(prob, opts, b=0)
    b = oracle.OracleSolver(pt, opts, b=0)
    assert a.solve() == b.solve()
    assert np.array_equal(a.get("X"), b.get("X")) and np.array_equal(a.get("U"), b.get("U"))


def test_transforms_map_every_knot(tog):
    """infeasible_problem / minimum_time_problem transform each knot's cost (infeasible.jl:2-33,
    minimum_time.jl:2-34)."""
    make, *_ = _pendulum_mt(tog)
    p = make(np.ones((30, 1)), 0.15)
    pinf = tog.infeasible_problem(p, 0.5)
    assert pinf.obj.varying
    for k in (0, 7, p.N - 2):
        R = pinf.obj[k].R
        assert np.array_equal(R[:1, :1], p.obj[k].R) and np.array_equal(R[1:, 1:], 0.5 * np.eye(2) / p.dt)
        assert np.array_equal(pinf.obj[k].Q, p.obj[k].Q)
    pmt = tog.minimum_time_problem(p, 15.0, 0.15, 1e-3)
    for k in (0, 7, p.N - 2):
        assert np.array_equal(pmt.obj[k].Q[:2, :2], p.obj[k].Q) and pmt.obj[k].Q.shape == (3, 3)
        assert np.array_equal(pmt.obj[k].R[:1, :1], p.obj[k].R)


def _pendulum_mt(tog):
    """test/minimum_time_tests.jl:1-63 with ramped per-knot weights."""
    model_d = tog.rk3(tog.Dynamics.pendulum)
    n, m, N = 2, 1, 31
    Q, R = 1e-3 * np.eye(n), 1e-3 * np.eye(m)
    xf, x0 = np.array([math.pi, 0.0]), np.zeros(n)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), iterations=50, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=15.0, dt_max=0.15, dt_min=1.0e-3)

    def make(U, dt, tf=None, X=None):
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=-5.0, u_max=5.0)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += tog.goal_constraint(xf)
        p = tog.Problem(model_d, ramp_objective(tog, Q, R, Q, xf, N), U, constraints=cons, dt=dt, x0=x0, N=N, tf=tf)
        if X is not None:
            p.X = X
        return p

    return make, opts, xf


# ----------------------------------------------------------------------------- GPU: device vs oracle


@pytest.mark.gpu
@pytest.mark.parametrize("sqrt", [False, True])
@pytest.mark.parametrize("tail", ["quad", "team", "full"])
def test_gpu_varying_ilqr(tog, oracle, gpu, sqrt, tail):
    """Cartpole iLQR with a ramped time-varying objective (diagonal costs: the literal-zero path) on each
    backward kernel: the four-wave tail kernel, the one-wave team kernel, full (uncompacted) launches."""
    prob, opts = cartpole_varying(tog, B=4)
    opts.square_root = sqrt
    env = {"quad": {}, "team": {"TOG_BWD_TAIL": "team"}, "full": {"TOG_NO_COMPACT": "1"}}[tail]
    solve_and_compare(tog, oracle, prob, opts, env)


@pytest.mark.gpu
@pytest.mark.parametrize("sqrt", [False, True])
def test_gpu_varying_dense_costs(tog, oracle, gpu, sqrt):
    """Non-diagonal Q_k and cross terms H_k per knot (the dense-cost path of every kernel)."""
    prob, opts = cartpole_varying(tog, B=3, cross=0.2)
    opts.square_root = sqrt
    solve_and_compare(tog, oracle, prob, opts)


@pytest.mark.gpu
def test_gpu_varying_al_quadrotor(tog, oracle, gpu):
    """Config 3's AL solve (square-root backward pass, bounds + goal) under a time-varying objective."""
    prob, opts = quadrotor_varying(tog, B=3)
    gp, solver = solve_and_compare(tog, oracle, prob, opts)
    assert np.all(solver.stats["c_max"] < opts.constraint_tolerance)


@pytest.mark.gpu
def test_gpu_equal_rows_equal_shared_cost(tog, gpu):
    """On the device too, a table of identical rows solves bit for bit like the shared cost."""
    prob, opts = tog.Problems.config_quadrotor(B=4)
    pt = prob.copy()
    pt.obj = tog.Objective(list(prob.obj.cost))
    pt.obj.varying = True
    a, b = prob.copy(), pt.copy()
    sa = tog.solve_b(a, opts)
    sb = tog.solve_b(b, opts)
    assert np.array_equal(a._X, b._X) and np.array_equal(a._U, b._U)
    assert np.array_equal(sa.handle.get(tog.abi.FIELD_STATS), sb.handle.get(tog.abi.FIELD_STATS))


@pytest.mark.gpu
def test_gpu_varying_altro_infeasible(tog, oracle, gpu):
    """test/infeasible_tests.jl's pendulum from a line guess, time-varying objective: tog_altro.cpp's
    infeasible_desc transforms every knot's cost as infeasible_problem does for the oracle."""
    make, opts, xf = _pendulum_mt(tog)
    X = tog.line_trajectory([0.0, 0.0], list(xf), 31)
    prob = make(np.zeros((30, 1)), 0.1, X=X)
    opts = tog.ALTROSolverOptions(opts_al=opts.opts_al, resolve_feasible_problem=True)
    ref = prob.copy()
    solver = tog.solve_b(prob, opts)
    Xo, Uo, si, sf = oracle.solve_altro_infeasible(ref, opts)
    assert rel(prob.X, Xo) < TOL_SOLVE and rel(prob.U, Uo) < TOL_SOLVE
    assert int(solver.stats["iterations_total"][0]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS])


@pytest.mark.gpu
def test_gpu_varying_min_time(tog, oracle, gpu):
    """Minimum time (minimum_time.jl:2-34) with a time-varying objective: each knot's cost zero-padded to
    [x; τ], [u; h] by tog_altro.cpp's min_time_desc, as minimum_time_problem does for the oracle."""
    make, opts, xf = _pendulum_mt(tog)
    p = make(np.ones((30, 1)), 0.15)
    s = oracle.OracleSolver(p, opts.opts_al, 0)
    s.solve()
    pm = make(s.get("U"), 0.075, tf="min")
    ref = pm.copy()
    solver = tog.solve_b(pm, opts)
    Xo, Uo, ho, so = oracle.solve_altro_min_time(ref, opts, 0)
    assert rel(pm._X[0], Xo) < TOL_SOLVE and rel(pm._U[0], Uo) < TOL_SOLVE
    assert np.max(np.abs(pm.h[0] - ho)) <= 1e-6
    assert int(solver.stats["iterations_total"][0]) == int(so.get("stats")[tog.abi.STAT_TOTAL_STEPS])


@pytest.mark.gpu
def test_gpu_varying_projected_newton(tog, oracle, gpu):
    """ALTRO's projected Newton phase weighs each knot with its own Q_k dt, R_k dt (the Hessian
    blocks of projected_newton.jl:97-132): X, U after the projection against the oracle to 1e-13."""
    from test_projected_newton import car_al_opts, car_batch

    p0 = car_batch(tog, 2, seed=11)
    st, term = p0.obj.stage, p0.obj.terminal
    prob = with_objective(tog, p0, ramp_objective(tog, st.Q, st.R, term.Q, p0.xf, p0.N))
    al = car_al_opts(tog, tol=1e-3)
    opts = tog.ALTROSolverOptions(opts_al=al, projected_newton=True, projected_newton_tolerance=1e-2)
    opts.opts_pn.feasibility_tolerance = 1e-10
    opts.opts_pn.active_set_tolerance = 1e-4
    opts.opts_pn.n_steps = 4
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts.opts_al, b=b)
        o.solve()
        o.solve_pn(opts.opts_pn)
        assert rel(gp._X[b], o.get("X")) < 1e-13 and rel(gp._U[b], o.get("U")) < 1e-13, b
    assert solver.stats["time_pn"] > 0.0
