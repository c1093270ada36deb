"""Minimum time: ``minimum_time_problem`` (src/solvers/altro/minimum_time.jl:2-34)
solved by ALTRO's AL phase, on the CPU oracle and on the device.

The augmented model carries the time step as a control: x = [x; τ], u = [u; h], dt_k = h_k²
(add_min_time_controls, :83-104), the objective is MinTimeCost (:142-200) and the constraints gain the h
bounds and h_k = τ_k (mintime_constraints, :125-141). The reference's own thresholds come from
test/minimum_time_tests.jl (pendulum and the box parallel park): the minimum-time solve must at least halve
(pendulum) / cut by a quarter (car) the fixed-time duration, reach the goal to 1e-3 and satisfy the
constraints. The device is held to the oracle: X, U and h within 1e-6 and equal iteration counts.
"""
import math

import numpy as np
import pytest


def pendulum_case(tog):
    """test/minimum_time_tests.jl:1-63."""
    model_d = tog.rk3(tog.Dynamics.pendulum)
    n, m, N = 2, 1, 31
    Q, R = 1e-3 * np.eye(n), 1e-3 * np.eye(m)
    xf, x0 = np.array([math.pi, 0.0]), np.zeros(n)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), iterations=50, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=15.0, dt_max=0.15, dt_min=1.0e-3)

    def make(U, dt, tf=None):
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=-5.0, u_max=5.0)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += tog.goal_constraint(xf)
        return tog.Problem(model_d, tog.LQRObjective(Q, R, Q, xf, N), U, constraints=cons, dt=dt, x0=x0, N=N, tf=tf)

    return make, opts, xf, np.ones((N - 1, m)), 0.15, 0.15 / 2.0, (0.5, 1.0)


def car_case(tog):
    """test/minimum_time_tests.jl:65-121 (box parallel park)."""
    model_d = tog.discretize_model(tog.Dynamics.car, "rk4")
    n, m, N = 3, 2, 51
    x0, xf = np.zeros(3), np.array([0.0, 1.0, 0.0])
    Qf, Q, R = 100.0 * np.eye(n), 1e-2 * np.eye(n), 1e-2 * np.eye(m)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), iterations=30, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=40.0, dt_max=0.2, dt_min=1.0e-3)
    bnd1 = tog.BoundConstraint(n, m, u_min=-2.0, u_max=2.0)
    bnd2 = tog.BoundConstraint(n, m, x_min=[-0.25, -0.001, -math.inf], x_max=[0.25, 1.001, math.inf],
                               u_min=-2.0, u_max=2.0)

    def make(U, dt, tf=None):
        cons = tog.Constraints(N)
        cons[0] += bnd1
        for k in range(1, N - 1):
            cons[k] += bnd2
        cons[N - 1] += tog.goal_constraint(xf)
        return tog.Problem(model_d, tog.LQRObjective(Q, R, Qf, xf, N), U, constraints=cons, dt=dt, x0=x0, N=N, tf=tf)

    return make, opts, xf, np.ones((N - 1, m)), 0.06, 0.06, (0.75, 2.1)


CASES = {"pendulum": pendulum_case, "car": car_case}


def test_mintime_constraint_sets(tog):
    """test/minimum_time_tests.jl:39-47: lengths of mintime_constraints' sets."""
    make, *_ = pendulum_case(tog)
    prob = make(np.ones((30, 1)), 0.15)
    pc = tog.mintime_constraints(prob)
    assert (len(pc[0]), len(pc[1]), len(pc[prob.N - 1])) == (1, 2, 2)
    pmt = tog.minimum_time_problem(prob, 15.0, 0.15, 1e-3)
    assert (pmt.model.n, pmt.model.m, pmt.tf) == (3, 2, 0.0) and pmt.model.min_time
    assert np.all(pmt._U[0, :, 1] == math.sqrt(0.15)) and np.all(pmt._X[0, :, 2] == math.sqrt(0.15))


@pytest.mark.parametrize("case", sorted(CASES))
def test_oracle_min_time_reference_thresholds(tog, oracle, case):
    """The oracle's minimum-time solve meets test/minimum_time_tests.jl's assertions."""
    make, opts, xf, U0, dt, dt_mt, (frac, tmax) = CASES[case](tog)
    p = make(U0, dt)
    s = oracle.OracleSolver(p, opts.opts_al, 0)
    s.solve()
    tt = dt * (p.N - 1)
    pm = make(s.get("U"), dt_mt, tf="min")
    X, U, h, _ = oracle.solve_altro_min_time(pm, opts, 0)
    tt_mt = float(np.sum(h ** 2))
    assert tt_mt < frac * tt and tt_mt < tmax
    assert np.max(np.abs(X[-1] - xf)) < 1e-3
    pm._X[0], pm._U[0] = X, U
    assert tog.max_violation(pm) < opts.opts_al.constraint_tolerance


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_gpu_min_time_equals_oracle(tog, oracle, gpu, case):
    """solve_b(prob, ALTROSolverOptions) with tf = :min on the device vs the oracle: X, U, h within
    1e-6, equal iteration counts, and the reference's thresholds."""
    make, opts, xf, U0, dt, dt_mt, (frac, tmax) = CASES[case](tog)
    p = make(U0, dt)
    s = oracle.OracleSolver(p, opts.opts_al, 0)
    s.solve()
    pm = make(s.get("U"), dt_mt, tf="min")
    ref = pm.copy()
    solver = tog.solve_b(pm, opts)
    Xo, Uo, ho, so = oracle.solve_altro_min_time(ref, opts, 0)
    scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
    assert np.max(np.abs(pm._X[0] - Xo)) <= 1e-6 * scale(Xo)
    assert np.max(np.abs(pm._U[0] - Uo)) <= 1e-6 * scale(Uo)
    assert np.max(np.abs(pm.h[0] - ho)) <= 1e-6
    assert int(solver.stats["iterations_total"][0]) == int(so.get("stats")[tog.abi.STAT_TOTAL_STEPS])
    tt_mt = tog.total_time(pm)
    assert tt_mt < frac * dt * (p.N - 1) and tt_mt < tmax


@pytest.mark.gpu
def test_gpu_min_time_jacobian(tog, oracle, gpu):
    """∇f! of add_min_time_controls on the device (k_jacobian_mt) vs the oracle's, per knot."""
    make, opts, *_ = car_case(tog)
    p = make(np.ones((50, 2)) * 0.3, 0.06)
    pmt = tog.minimum_time_problem(p, 40.0, 0.2, 1e-3)
    h = tog.ALTROSolver(pmt, opts).handle
    h.upload_state(pmt)
    tog.abi.check(h.lib, h.lib.tog_rollout_open_loop(h.h))
    tog.abi.check(h.lib, h.lib.tog_jacobians(h.h))
    A, B = h.get(tog.abi.FIELD_A)[0], h.get(tog.abi.FIELD_B)[0]
    o = oracle.OracleSolver(pmt, opts.opts_al, 0)
    o.rollout_open_loop()
    o.jacobians()
    Ao, Bo = o.get("A"), o.get("B")
    assert np.allclose(A, Ao, rtol=1e-13, atol=1e-15)
    assert np.allclose(B, Bo, rtol=1e-13, atol=1e-15)
    assert np.all(B[:, 3, 2] == 1.0) and np.all(A[:, 3, :] == 0.0)  # τ+ = h


# minimum_time_problem on the remaining built-in models (the reference asserts only that the problem has
# bounds, minimum_time.jl:2-8; its minimum-time tests cover the pendulum and the car, above). The device
# is held to the oracle: equal iteration counts, X and U to the north-star bar. The Kuka case runs a short
# horizon with control bounds added (its notebook problem has only the goal constraint).
def _mt_model_case(tog, name):
    al_opts = dict(opts_uncon=tog.iLQRSolverOptions(iterations=60), iterations=6, penalty_scaling=10.0)
    if name == "quadrotor":
        p = tog.Problems.quadrotor_test("goal+bounds")
        return tog.minimum_time_problem(p, 5.0, 0.1, 1e-3), tog.AugmentedLagrangianSolverOptions(**al_opts)
    if name == "cartpole":
        p = tog.Problems.cartpole(constrained=True)
        return tog.minimum_time_problem(p, 10.0, 0.1, 1e-3), tog.AugmentedLagrangianSolverOptions(**al_opts)
    n, m, N = 14, 7, 11
    base = tog.Problems.kuka(N=N, tf=0.5)
    cons = tog.Constraints(N)
    bnd = tog.BoundConstraint(n, m, u_min=-80.0, u_max=80.0)
    for k in range(N - 1):
        cons[k] += bnd
    cons[N - 1] += tog.goal_constraint(base.xf)
    p = tog.Problem(base.model, base.obj, base._U[0], constraints=cons, x0=base.x0[0], xf=base.xf, N=N, dt=base.dt)
    al_opts["opts_uncon"] = tog.iLQRSolverOptions(iterations=25)
    al_opts["iterations"] = 3
    return tog.minimum_time_problem(p, 1.0, 0.1, 1e-3), tog.AugmentedLagrangianSolverOptions(**al_opts)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["quadrotor", "cartpole", "kuka"])
def test_gpu_min_time_models_equal_oracle(tog, oracle, gpu, name):
    """MinTime<M> for the quadrotor, cartpole and Kuka models (add_min_time_controls, minimum_time.jl:83-104):
    the AL solve of minimum_time_problem on the device (std backward pass, LDS kernel) equals the oracle."""
    from test_gpu_parity import _solve_and_compare

    pmt, opts = _mt_model_case(tog, name)
    assert pmt.model.min_time and pmt.model.n == {"quadrotor": 14, "cartpole": 5, "kuka": 15}[name]
    _solve_and_compare(tog, oracle, pmt, opts)


# ----------------------------------------------------------------------------- infeasible start + minimum time


def _inf_mt_case(tog, resolve=True):
    """test/minimum_time_tests.jl's pendulum from a straight-line state guess with tf = :min: altro_problem
    makes it minimum_time_problem(infeasible_problem(prob)) (altro_methods.jl:98-124)."""
    make, opts, xf, U0, dt, dt_mt, _ = pendulum_case(tog)
    p = make(U0, dt_mt, tf="min")
    p.X = tog.line_trajectory(p.x0[0], xf, p.N)
    opts.resolve_feasible_problem = resolve
    opts.opts_al.iterations = 15
    return p, opts, xf


def test_infeasible_min_time_bounds_quirk(tog):
    """mintime_constraints on the infeasible problem (minimum_time.jl:125-141): combine(bnd, mt_bnd) sizes the
    bound by the infeasible problem's BoundConstraint, which keeps the model's m, so √dt_min <= u[m+1] <=
    √dt_max lands on the first slack control and h (the last control) is unbounded. Reproduced as written."""
    p, opts, _ = _inf_mt_case(tog)
    pinf = tog.infeasible_problem(p, opts.R_inf)
    pmt = tog.minimum_time_problem(pinf, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    n, m = p.model.n, p.model.m
    assert (pmt.model.n, pmt.model.m, pmt.model.slack, pmt.model.min_time) == (n + 1, m + n + 1, n, True)
    bnd = [c for c in pmt.constraints[3] if isinstance(c, tog.BoundConstraint)][0]
    _, _, data = bnd.to_abi(pmt.model.m)
    u_max = data[2 * (n + 1): 2 * (n + 1) + pmt.model.m]
    assert u_max[m] == math.sqrt(opts.dt_max) and np.isinf(u_max[-1])
    labels = [type(c).__name__ for c in pmt.constraints[3]]
    assert labels == ["InfeasibleConstraint", "BoundConstraint", "MinTimeEquality"]


def test_oracle_infeasible_min_time_flow(tog, oracle):
    """The whole flow on the oracle: the infeasible minimum-time AL phase, then the feasible minimum-time
    resolve from its controls and time steps; the resolve meets test/minimum_time_tests.jl's goal threshold."""
    p, opts, xf = _inf_mt_case(tog)
    X, U, h, si, sf = oracle.solve_altro_infeasible_min_time(p, opts, 0)
    assert np.all(np.isfinite(X)) and np.all(np.isfinite(U)) and np.all(h > 0)
    assert sf is not None and np.max(np.abs(X[-1] - xf)) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("resolve", [False, True])
def test_gpu_infeasible_min_time_equals_oracle(tog, oracle, gpu, resolve):
    """solve_b(prob, ALTROSolverOptions) with an initial state trajectory and tf = :min on the device
    (MinTime<Infeasible<Pendulum>>, tog_altro.cpp's transforms) against the oracle's flow: X, U, h within
    1e-6 and equal iteration counts in both phases."""
    p, opts, _ = _inf_mt_case(tog, resolve)
    ref = p.copy()
    solver = tog.solve_b(p, opts)
    Xo, Uo, ho, si, sf = oracle.solve_altro_infeasible_min_time(ref, opts, 0)
    scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
    assert np.max(np.abs(p._X[0] - Xo)) <= 1e-6 * scale(Xo)
    assert np.max(np.abs(p._U[0] - Uo)) <= 1e-6 * scale(Uo)
    assert np.max(np.abs(p.h[0] - ho)) <= 1e-6
    assert int(solver.stats["iterations_total"][0]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS])
    if resolve:
        assert int(solver.stats_feasible["iterations_total"][0]) == int(sf.get("stats")[tog.abi.STAT_TOTAL_STEPS])


def _pn_mt_opts(opts):
    opts.projected_newton = True
    # 1e-2 leaves the pendulum's projection short of 1e-8 in 3 steps: the line search fails and the oracle flags
    # TOG_TRAJ_PN_ERROR (the reference raises), as the device does; from 1e-3 one newton step reaches 6.6e-9
    opts.projected_newton_tolerance = 1e-3
    opts.opts_pn.n_steps = 3
    opts.opts_pn.feasibility_tolerance = 1e-8
    return opts


def test_oracle_min_time_projected_newton(tog, oracle):
    """Projected Newton on the minimum-time problem (altro_methods.jl:31-39 with prob_altro =
    minimum_time_problem): its H is MinTimeCost's hessian! diagonal at the newton step's X, U
    (minimum_time.jl:238-280). After the AL phase stopped at projected_newton_tolerance the projection
    reduces the violation."""
    make, opts, xf, U0, dt, dt_mt, _ = pendulum_case(tog)
    opts = _pn_mt_opts(opts)
    tog.solvers._altro_pn_tolerances(opts)
    p = make(U0, dt_mt, tf="min")
    pmt = tog.minimum_time_problem(p, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    s = oracle.OracleSolver(pmt, opts.opts_al)
    s.solve()
    c_al = s.max_violation()
    st = s.solve_pn(opts.opts_pn)
    assert st[tog.abi.PN_STEPS] >= 1 and s.max_violation() < min(c_al, 1e-8)
    assert not int(s.get("stats")[tog.abi.STAT_FLAGS]) & tog.abi.TRAJ_PN_ERROR


@pytest.mark.gpu
@pytest.mark.parametrize("infeasible,solve_type", [(False, "feasible"), (True, "feasible"), (False, "optimal"),
                                                   (True, "optimal")])
def test_gpu_min_time_projected_newton(tog, oracle, gpu, infeasible, solve_type):
    """solve_b with tf = :min and projected_newton (and an initial state trajectory): the device's projected
    Newton on MinTime<Pendulum> / MinTime<Infeasible<Pendulum>> (per-knot H from X, U: at the newton step's
    point, and under :optimal again at the line search's start and at each projected trial) against the
    oracle's same flow: X, U, h within 1e-6, as the minimum-time AL phase before it."""
    if infeasible:
        p, opts, _ = _inf_mt_case(tog, resolve=False)
    else:
        make, opts, xf, U0, dt, dt_mt, _ = pendulum_case(tog)
        p = make(U0, dt_mt, tf="min")
    opts = _pn_mt_opts(opts)
    opts.opts_pn.solve_type = solve_type
    ref = p.copy()
    try:
        solver, raised = tog.solve_b(p, opts), False
    except tog.ProjectedNewtonError as e:  # the reference raises in _projection_linesearch! for this start
        solver, raised = e.solver, True
    assert solver.stats["time_pn"] > 0.0
    if infeasible:
        Xo, Uo, ho, si, _ = oracle.solve_altro_infeasible_min_time(ref, opts, 0)
    else:
        Xo, Uo, ho, si = oracle.solve_altro_min_time(ref, opts, 0)
    assert raised == bool(int(si.get("stats")[tog.abi.STAT_FLAGS]) & tog.abi.TRAJ_PN_ERROR)
    tol = 1e-6
    scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
    assert np.max(np.abs(p._X[0] - Xo)) <= tol * scale(Xo)
    assert np.max(np.abs(p._U[0] - Uo)) <= tol * scale(Uo)
    assert np.max(np.abs(p.h[0] - ho)) <= tol
    assert int(solver.stats_pn["iterations"][0]) >= 1


def _untrimmed_mt_problem(tog):
    """A minimum-time pendulum built by hand with an untrimmed bound on [x; τ] and [u; h]
    (BoundConstraint(n̄, m̄, trim=false), constraints.jl:155-188): every u row is kept, the time step h's
    √dt bounds included."""
    make, opts, *_ = pendulum_case(tog)
    p = make(np.ones((30, 1)), 0.15)
    pmt = tog.minimum_time_problem(p, 15.0, 0.15, 1e-3)
    n, m, N = pmt.model.n, pmt.model.m, pmt.N
    bnd = tog.BoundConstraint(n, m, x_min=[-10.0, -10.0, -1.0], x_max=[10.0, 10.0, 1.0],
                              u_min=[-5.0, math.sqrt(1e-3)], u_max=[5.0, math.sqrt(0.15)], trim=False)
    cons = tog.Constraints(N)
    for k in range(N):
        cons[k] += bnd
        if 0 < k < N - 1:
            cons[k] += tog.MinTimeEquality()
    q = tog.Problem(pmt.model, pmt.obj, pmt._U[0], constraints=cons, x0=pmt.x0[0], xf=pmt.xf, N=N, dt=pmt.dt)
    q._X[0] = pmt._X[0]
    return q, bnd, opts


def test_oracle_untrimmed_min_time_bound_keeps_h_rows(tog, oracle):
    """An untrimmed bound on a minimum-time problem keeps the rows of h, the last control (advisor r5: they
    were dropped with the slack controls'): the oracle's constraint values equal the host BoundConstraint's."""
    q, bnd, opts = _untrimmed_mt_problem(tog)
    o = oracle.OracleSolver(q, opts.opts_al, 0)
    o.rollout_open_loop()
    o.update_constraints()
    C = o.get("C")
    X, U = o.get("X"), o.get("U")
    assert bnd.length("stage") == 10
    for k in (0, 5, q.N - 2):
        assert np.array_equal(C[k, :10], bnd.evaluate(X[k], U[k])), k
    assert np.array_equal(C[q.N - 1, :6], bnd.evaluate(X[q.N - 1]))


@pytest.mark.gpu
def test_gpu_untrimmed_min_time_bound_rows(tog, oracle, gpu):
    """The device's rows of the untrimmed minimum-time bound (tog_update_constraints) equal the oracle's,
    and an AL solve on it matches the oracle's iteration count and X, U within 1e-6."""
    q, bnd, opts = _untrimmed_mt_problem(tog)
    o = oracle.OracleSolver(q, opts.opts_al, 0)
    o.rollout_open_loop()
    o.update_constraints()
    solver = tog.AugmentedLagrangianSolver(q, opts.opts_al)
    q2 = q.copy()
    q2._X[0] = o.get("X")
    solver.handle.upload_state(q2)
    tog.update_constraints_b(q2, solver)
    C = solver.handle.get(tog.abi.FIELD_C)[0]
    assert np.array_equal(C[:, :11], o.get("C")[:, :11])
    o2 = oracle.OracleSolver(q, opts.opts_al, 0)
    steps = o2.solve()
    gp = q.copy()
    s = tog.solve_b(gp, opts.opts_al)
    assert int(s.stats["iterations_total"][0]) == steps
    scale = max(1.0, float(np.max(np.abs(o2.get("X")))))
    assert np.max(np.abs(gp._X[0] - o2.get("X"))) <= 1e-6 * scale


def _inf_mt_model_case(tog, name):
    """minimum_time_problem(infeasible_problem(prob)) for the quadrotor and the Kuka arm (round 6; the state guess
    a straight line x0 -> xf, short horizons): MinTime<Infeasible<M>> on the LDS backward kernel."""
    if name == "quadrotor":
        n, m, N = 13, 4, 21
        q0 = np.array([1.0, 0.0, 0.0, 0.0])
        x0, xf = np.zeros(n), np.zeros(n)
        x0[3:7] = q0
        xf[0:3] = [0.0, 4.0, 0.0]
        xf[3:7] = q0
        obj = tog.LQRObjective(1e-2 * np.eye(n), 1e-2 * np.eye(m), 100.0 * np.eye(n), xf, N)
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=0.0, u_max=15.0)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += tog.goal_constraint(xf)
        U0 = tog.Problems.HOVER * np.ones((N - 1, m))
        p = tog.Problem(tog.rk4(tog.Dynamics.quadrotor), obj, U0, constraints=cons, x0=x0, xf=xf, N=N, dt=0.1,
                        tf="min")
        dt_max = 0.15
    else:
        n, m, N = 14, 7, 11
        base = tog.Problems.kuka(N=N, tf=0.5)
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=-80.0, u_max=80.0)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += tog.goal_constraint(base.xf)
        x0, xf = base.x0[0], base.xf
        p = tog.Problem(base.model, base.obj, base._U[0], constraints=cons, x0=x0, xf=xf, N=N, dt=base.dt, tf="min")
        dt_max = 0.1
    p.X = np.stack([x0 + (xf - x0) * k / (N - 1) for k in range(N)])
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(iterations=40), iterations=4,
                                              penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=1.0, dt_max=dt_max, dt_min=1e-3, R_inf=1.0,
                                  resolve_feasible_problem=False)
    return p, opts


@pytest.mark.parametrize("name", ["quadrotor", "kuka"])
def test_oracle_infeasible_min_time_models(tog, oracle, name):
    """The oracle's infeasible minimum-time flow runs for the quadrotor and the Kuka arm (finite iterates) with
    the composite model's shapes. (h may go negative: mintime_constraints' quirk leaves it unbounded, dt = h².)"""
    p, opts = _inf_mt_model_case(tog, name)
    X, U, h, si, _ = oracle.solve_altro_infeasible_min_time(p, opts, 0)
    n, m = p.model.n, p.model.m
    assert X.shape == (p.N, n) and U.shape == (p.N - 1, m) and si.m == m + n + 1
    assert np.all(np.isfinite(X)) and np.all(np.isfinite(U)) and np.all(np.isfinite(h))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["quadrotor", "kuka"])
def test_gpu_infeasible_min_time_models(tog, oracle, gpu, name):
    """MinTime<Infeasible<Quadrotor>> and MinTime<Infeasible<Kuka>> (round 6) on the device against the
    oracle's flow: X, U, h within 1e-6 and equal AL iteration counts."""
    p, opts = _inf_mt_model_case(tog, name)
    ref = p.copy()
    solver = tog.solve_b(p, opts)
    Xo, Uo, ho, si, _ = oracle.solve_altro_infeasible_min_time(ref, opts, 0)
    scale = lambda a: max(1.0, float(np.max(np.abs(a))))  # noqa: E731
    assert np.max(np.abs(p._X[0] - Xo)) <= 1e-6 * scale(Xo)
    assert np.max(np.abs(p._U[0] - Uo)) <= 1e-6 * scale(Uo)
    assert np.max(np.abs(p.h[0] - ho)) <= 1e-6
    assert int(solver.stats["iterations_total"][0]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS])


@pytest.mark.gpu
def test_gpu_min_time_kuka_divergent_trials_rejected(tog, oracle, gpu):
    """Regression for round 4's MinTime<Kuka> rollout fault (profiles/r4j_mt_kuka_trials_split_f.txt: written
    through the chol()/solve() helpers, the speculative rollouts accepted trials whose states had passed
    max_state_value; rollout.jl:18-20 rejects them). Replays that case: the line search of step 20 of the
    minimum-time Kuka solve, whose first trials (α = 1 .. 1/32) diverge. Every trial's verdict equals the
    oracle's rollout from the same state, and the accepted trials' costs equal the oracle's bit for bit
    (tog__debug_ls dumps the device's trials)."""
    import ctypes as C
    abi = tog.abi
    prob, opts = _mt_model_case(tog, "kuka")
    s = tog.AbstractSolverFor(prob.copy(), opts)
    h = s.handle
    h.solve_init(abi.MODE_AL)
    for _ in range(19):
        h.solve_step(1)
    st0 = {f: h.get(f, raw=True) for f in (abi.FIELD_X, abi.FIELD_U, abi.FIELD_LAMBDA, abi.FIELD_MU, abi.FIELD_RHO)}
    h.solve_step(1)
    nc = C.c_int32()
    J = np.zeros(64)
    ok = np.zeros(64, dtype=np.int32)
    abi.check(h.lib, h.lib.tog__debug_ls(h.h, J.ctypes.data_as(C.POINTER(C.c_double)),
                                         ok.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(nc)))
    o = oracle.OracleSolver(prob, opts, b=0)
    for f, nm in ((abi.FIELD_X, "X"), (abi.FIELD_U, "U"), (abi.FIELD_LAMBDA, "lambda"), (abi.FIELD_MU, "mu"),
                  (abi.FIELD_RHO, "rho")):
        o.set(nm, st0[f][0])
    o.update_constraints()
    o.jacobians()
    assert o.cost_expansion(False, True) == 0
    o.backward(False)
    diverged = 0
    assert nc.value >= 8
    for j in range(nc.value):
        oko = o.rollout(2.0 ** -j)
        assert bool(ok[j]) == bool(oko), (j, ok[j], oko)
        if oko:
            assert J[j] == o.cost_bar(True), j
        else:
            diverged += 1
    assert diverged >= 1  # the case still exercises the divergence test
