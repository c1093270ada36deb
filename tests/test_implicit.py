"""Implicit integrators: ``midpoint_implicit`` (src/integration.jl:44-73) and
``rk3_implicit`` (:171-205), reached through ``discretize_model(model, :midpoint_implicit)``
(src/model.jl:646-669).

CPU tests pin the oracle's Newton step (oracle/tog_oracle.c implicit_step_dual): the implicit
equation holds to the reference's loop tolerance, the dual Jacobian equals the implicit-function
Jacobian and central differences, and the reference's own test (test/pendulum_tests.jl:9,22-26:
every scheme's ALTRO solve of Problems.pendulum ends with max_violation < constraint_tolerance)
passes on the oracle. The ``gpu`` tests hold the device's Jacobians and solves bit for bit to the
oracle.
"""
import math

import numpy as np
import pytest

TOL_STEP = 1e-13
SCHEMES = ["midpoint_implicit", "rk3_implicit"]
INTEG = {"midpoint_implicit": 4, "rk3_implicit": 3}


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def pendulum_opts(tog):
    """test/pendulum_tests.jl:4-7."""
    il = tog.iLQRSolverOptions()
    return tog.AugmentedLagrangianSolverOptions(opts_uncon=il, iterations=50, penalty_scaling=10.0)


def pendulum_batch(tog, scheme, B, seed=0):
    """Problems.pendulum (problems/pendulum.jl:1-35) under ``scheme``, B starts near x0 = 0."""
    p1 = tog.Problems.pendulum(scheme)
    rng = np.random.default_rng(seed)
    x0 = 0.05 * rng.standard_normal((B, 2))
    x0[0] = 0.0
    U0 = np.ones((B, p1.N - 1, 1)) + 0.1 * rng.standard_normal((B, p1.N - 1, 1))
    U0[0] = 1.0
    return tog.Problem(p1.model, p1.obj, U0, constraints=p1.constraints, x0=x0, xf=p1.xf, N=p1.N, dt=p1.dt)


# ----------------------------------------------------------------------------- CPU: host + oracle


def test_discretize_model_schemes(tog):
    """discretize_model accepts every scheme of test/pendulum_tests.jl:9 and rejects others."""
    for s in ["midpoint", "rk3", "rk4", "rk3_implicit", "midpoint_implicit"]:
        md = tog.discretize_model(tog.Dynamics.pendulum, s)
        assert md.discrete
    assert tog.midpoint_implicit(tog.Dynamics.pendulum).integration == tog.abi.MIDPOINT_IMPLICIT
    assert tog.rk3_implicit(tog.Dynamics.cartpole).integration == tog.abi.RK3_IMPLICIT
    with pytest.raises(ValueError):
        tog.discretize_model(tog.Dynamics.pendulum, "bogus")
    # the device instantiates the Newton step for n <= 4, the quadrotor and the Kuka arm (KukaImplicit)
    assert tog.discretize_model(tog.Dynamics.quadrotor, "midpoint_implicit").integration == tog.abi.MIDPOINT_IMPLICIT
    assert tog.discretize_model(tog.Dynamics.kuka, "rk3_implicit").integration == tog.abi.RK3_IMPLICIT


@pytest.mark.parametrize("scheme", SCHEMES)
@pytest.mark.parametrize("name", ["pendulum", "cartpole", "car", "doubleintegrator"])
def test_oracle_implicit_equation(tog, oracle, scheme, name):
    """x+ solves the implicit equation to the Newton loop's tolerance. midpoint_implicit:
    x+ - x - dt f((x + x+)/2) = 0. rk3_implicit (with the reference's aliased stage buffers):
    x+ - x - (dt/6 + 4/6 dt + dt/6) f((x + x+)/2) = 0."""
    model = getattr(tog.Dynamics, name)
    rng = np.random.default_rng(4)
    dt = 0.1
    for _ in range(5):
        x = 0.5 * rng.standard_normal(model.n)
        u = 0.5 * rng.standard_normal(model.m)
        y = oracle.discrete_f(model.model_id, INTEG[scheme], x, u, dt)
        f = oracle.continuous_f(model.model_id, 0.5 * (x + y), u)
        if scheme == "midpoint_implicit":
            g = y - x - dt * f
        else:
            g = ((y - x - dt / 6 * f) - 4 / 6 * dt * f) - dt / 6 * f
        assert np.linalg.norm(g) < 1e-11


def _jac_x(oracle, model, x, u, h=1e-6):
    n = model.n
    A = np.zeros((n, n))
    for j in range(n):
        e = np.zeros(n)
        e[j] = h
        A[:, j] = (oracle.continuous_f(model.model_id, x + e, u) - oracle.continuous_f(model.model_id, x - e, u)) / (2 * h)
    return A


@pytest.mark.parametrize("scheme", SCHEMES)
@pytest.mark.parametrize("name", ["pendulum", "cartpole", "car"])
def test_oracle_implicit_jacobian(tog, oracle, scheme, name):
    """The dual Jacobian through the Newton loop is the implicit-function Jacobian of
    g(x+, x, u) = 0 (the reference's ForwardDiff through fd!, src/model.jl:491-522, converges to it
    with the loop) and matches central differences of the step."""
    model = getattr(tog.Dynamics, name)
    rng = np.random.default_rng(5)
    dt = 0.1
    n, m = model.n, model.m
    c = 1.0 if scheme == "midpoint_implicit" else ((dt / 6 + 4 / 6 * dt) + dt / 6) / dt
    for _ in range(3):
        x = 0.5 * rng.standard_normal(n)
        u = 0.5 * rng.standard_normal(m)
        S = oracle.discrete_jacobian(model.model_id, INTEG[scheme], x, u, dt)
        y = oracle.discrete_f(model.model_id, INTEG[scheme], x, u, dt)
        xm = 0.5 * (x + y)
        # IFT: (I - c dt/2 Ax) dy = (I + c dt/2 Ax) dx + c dt Bu du, derivatives at xm
        h = 1e-6
        Ax = _jac_x(oracle, model, xm, u)
        Bu = np.zeros((n, m))
        for j in range(m):
            e = np.zeros(m)
            e[j] = h
            Bu[:, j] = (oracle.continuous_f(model.model_id, xm, u + e) - oracle.continuous_f(model.model_id, xm, u - e)) / (2 * h)
        Lm = np.eye(n) - 0.5 * c * dt * Ax
        dydx = np.linalg.solve(Lm, np.eye(n) + 0.5 * c * dt * Ax)
        dydu = np.linalg.solve(Lm, c * dt * Bu)
        assert np.max(np.abs(S[:, :n] - dydx)) < 1e-7
        assert np.max(np.abs(S[:, n:n + m] - dydu)) < 1e-7
        # central differences of the discrete step itself
        for j in range(n + m):
            e = np.zeros(n + m)
            e[j] = h
            yp = oracle.discrete_f(model.model_id, INTEG[scheme], x + e[:n], u + e[n:], dt)
            ym = oracle.discrete_f(model.model_id, INTEG[scheme], x - e[:n], u - e[n:], dt)
            assert np.max(np.abs(S[:, j] - (yp - ym) / (2 * h))) < 1e-6


@pytest.mark.parametrize("scheme", SCHEMES)
def test_oracle_reference_pendulum_schemes(tog, oracle, scheme):
    """test/pendulum_tests.jl:22-26: solve!(prob, opts_altro) under each scheme satisfies
    max_violation(prob) < opts_al.constraint_tolerance (ALTRO with a NaN X0 is its AL phase)."""
    prob = tog.Problems.pendulum(scheme)
    al = pendulum_opts(tog)
    o = oracle.OracleSolver(prob, tog.ALTROSolverOptions(opts_al=al))
    o.solve()
    assert o.max_violation() < al.constraint_tolerance
    X = o.get("X")
    assert np.linalg.norm(X[-1] - prob.xf) < 1e-2


# ----------------------------------------------------------------------------- GPU: device vs oracle


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", SCHEMES)
@pytest.mark.parametrize("name", ["pendulum", "cartpole", "car", "doubleintegrator", "quadrotor", "kuka"])
def test_gpu_implicit_jacobian_parity(tog, oracle, gpu, scheme, name):
    """k_jacobian through the device Newton step vs the oracle's dual restatement, bit for bit."""
    model = getattr(tog.Dynamics, name)
    n, m, N = model.n, model.m, 9
    rng = np.random.default_rng(6)
    B = 4
    md = tog.discretize_model(model, scheme)
    obj = tog.LQRObjective(0.1 * np.eye(n), 0.05 * np.eye(m), 10.0 * np.eye(n), np.zeros(n), N)
    prob = tog.Problem(md, obj, 0.4 * rng.standard_normal((B, N - 1, m)), x0=0.3 * rng.standard_normal((B, n)), N=N,
                       dt=0.08)
    prob._X[...] = 0.5 * rng.standard_normal(prob._X.shape)
    if name == "quadrotor":  # unit quaternions, controls about hover
        prob._X[..., 3:7] = [1.0, 0.0, 0.0, 0.0]
        prob._U[...] += 0.5 * 9.81 / 4
    solver = tog.iLQRSolver(prob, tog.iLQRSolverOptions())
    tog.jacobian_b(prob, solver)
    A = solver.handle.get(tog.abi.FIELD_A)
    Bm = solver.handle.get(tog.abi.FIELD_B)
    for b in range(B):
        for k in range(N - 1):
            S = oracle.discrete_jacobian(model.model_id, INTEG[scheme], prob._X[b, k], prob._U[b, k], prob.dt)
            assert rel(A[b, k], S[:, :n]) < TOL_STEP, (b, k)
            assert rel(Bm[b, k], S[:, n:n + m]) < TOL_STEP, (b, k)


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", SCHEMES)
def test_gpu_implicit_pendulum_solve(tog, oracle, gpu, scheme):
    """The reference's pendulum scheme test on the device (4 starts), X/U and iteration counts equal
    to the oracle's, and its max_violation threshold."""
    prob = pendulum_batch(tog, scheme, 4)
    opts = tog.ALTROSolverOptions(opts_al=pendulum_opts(tog))
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        assert steps == solver.stats["iterations_total"][b]
    assert np.all(solver.stats["c_max"] < opts.opts_al.constraint_tolerance)


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", SCHEMES)
def test_gpu_implicit_quadrotor_solve(tog, oracle, gpu, scheme):
    """The quadrotor (n = 13) under the implicit schemes: a short AL-iLQR solve (u bounds + goal, std
    backward pass) on the device equals the oracle's, iterations included."""
    base = tog.Problems.quadrotor_test("goal+bounds")
    N = 21
    xf = base.xf.copy()
    xf[0:3] = [0.0, 2.0, 0.0]
    n, m = 13, 4
    cons = tog.Constraints(N)
    bnd = tog.BoundConstraint(n, m, u_min=0.0, u_max=15.0)
    for k in range(N - 1):
        cons[k] += bnd
    cons[N - 1] += tog.goal_constraint(xf)
    obj = tog.LQRObjective(1e-2 * np.eye(n), 1e-2 * np.eye(m), 100.0 * np.eye(n), xf, N)
    rng = np.random.default_rng(9)
    U0 = 0.5 * 9.81 / 4 + 0.1 * rng.standard_normal((2, N - 1, m))
    prob = tog.Problem(tog.discretize_model(tog.Dynamics.quadrotor, scheme), obj, U0, constraints=cons,
                       x0=np.tile(base.x0[0], (2, 1)), xf=xf, N=N, dt=0.05)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(iterations=40), iterations=5,
                                                constraint_tolerance=1e-3)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        assert steps == solver.stats["iterations_total"][b]


@pytest.mark.gpu
def test_gpu_implicit_unsupported_model(tog, gpu):
    """tog_create rejects an implicit scheme on a model it is not instantiated for (the minimum-time
    augmentation, whose dt is a control)."""
    prob = tog.Problems.kuka(N=5)
    prob.model = tog.Model(tog.abi.MODEL_KUKA, 15, 8, "kuka_mt", tog.abi.MIDPOINT_IMPLICIT, min_time=True)
    with pytest.raises(Exception):
        tog.iLQRSolver(prob, tog.iLQRSolverOptions())


@pytest.mark.gpu
@pytest.mark.parametrize("scheme", ["midpoint_implicit", "rk3_implicit"])
def test_gpu_implicit_kuka_solve(tog, oracle, gpu, scheme):
    """The Kuka arm (n = 14, RigidBodyDynamics restated) under the implicit schemes
    (src/integration.jl:44-73, :171-205): Newton solves inside every rollout step and the Jacobian through
    the Newton loop; a short AL-iLQR solve on the device equals the oracle's, iterations included."""
    base = tog.Problems.kuka(N=11, tf=0.5)
    model = tog.discretize_model(tog.Dynamics.kuka, scheme)
    rng = np.random.default_rng(21)
    U0 = base._U[0] + 0.1 * rng.standard_normal((2, base.N - 1, 7))
    prob = tog.Problem(model, base.obj, U0, constraints=base.constraints, x0=np.tile(base.x0[0], (2, 1)),
                       xf=base.xf, N=base.N, dt=base.dt)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(iterations=15), iterations=3,
                                                constraint_tolerance=1e-3, penalty_initial=0.01,
                                                penalty_scaling=50.0)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        assert steps == solver.stats["iterations_total"][b]
