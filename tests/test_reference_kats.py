"""The reference's own assertions re-run against the CPU oracle and the host
mirror. These pin the oracle before it is trusted as the GPU parity checker.

Each test cites the reference test it restates. No reference code runs here (there is no Julia);
the inputs and expected values are the ones written in the reference test files.
"""
import math

import numpy as np
import pytest


SQRT_EPS = math.sqrt(np.finfo(float).eps)  # Julia isapprox default rtol


def isapprox(a, b, rtol=SQRT_EPS):
    """Julia ``isapprox`` on arrays: norm(a-b) <= rtol * max(norm(a), norm(b))."""
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    return np.linalg.norm(a - b) <= rtol * max(np.linalg.norm(a), np.linalg.norm(b))


# ------------------------------------------------------------------ constraints (constraint_tests.jl)

def bound_kat_problem(tog):
    """test/constraint_tests.jl:1-16,55-58 setup on the car model (n=3, m=2)."""
    n, m, N = 3, 2, 2
    bnd = tog.BoundConstraint(n, m, x_max=[5, 5, math.inf], x_min=[-10, -5, 0.0], u_min=-10.0, u_max=0.0)
    obj = tog.LQRObjective(np.eye(n), np.eye(m), np.eye(n), np.zeros(n), N)
    cons = tog.Constraints([bnd], N)
    prob = tog.Problem(tog.rk3(tog.Dynamics.car), obj, np.zeros((N - 1, m)), constraints=cons, x0=np.zeros(n),
                       N=N, dt=0.1)
    return prob, bnd


X_KAT = np.array([1.0, 2.0, 3.0])
U_KAT = np.array([-5.0, 5.0])
V_STAGE = [-4, -3, -5, 5, -11, -7, -3, -5, -15]  # constraint_tests.jl:96
V_TERM = [-4, -3, -11, -7, -3]                   # constraint_tests.jl:103


def test_bound_constraint_kat_host(tog):
    """constraint_tests.jl:90-108: trimmed BoundConstraint values, Jacobians and lengths."""
    _, bnd = bound_kat_problem(tog)
    assert bnd.length("stage") == 9 and bnd.length("terminal") == 5
    assert list(bnd.evaluate(X_KAT, U_KAT)) == V_STAGE
    assert list(bnd.evaluate(X_KAT)) == V_TERM
    n, m = 3, 2
    jac = np.vstack([np.eye(n + m)[[True, True, False, True, True]], -np.eye(n + m)])
    assert np.array_equal(bnd.jacobian(X_KAT, U_KAT), jac)
    jac_t = np.vstack([np.eye(n)[[True, True, False]], -np.eye(n)])
    assert np.array_equal(bnd.jacobian(X_KAT), jac_t)


def test_bound_constraint_kat_oracle(tog, oracle):
    """Same KAT through the oracle's constraint rows (row order [x_max; u_max; x_min; u_min])."""
    prob, _ = bound_kat_problem(tog)
    s = oracle.OracleSolver(prob, tog.AugmentedLagrangianSolverOptions())
    s.set("X", np.stack([X_KAT, X_KAT]))
    s.set("U", U_KAT[None, :])
    s.update_constraints()
    C = s.get("C")
    assert list(C[0, :9]) == V_STAGE
    assert list(C[1, :5]) == V_TERM


def test_bound_validation_errors(tog):
    """constraints.jl:276-296: x_max < x_min is an ArgumentError."""
    with pytest.raises(ValueError):
        tog.BoundConstraint(2, 1, x_max=[0.0, 0.0], x_min=[1.0, 1.0])


# ------------------------------------------------------------------ utils (test_utils.jl:81-94)

@pytest.mark.parametrize("x,args,sign", [
    ([0, 0, 0], (1, 0, 1), 0), ([0, 0, 0], (1, 0, 0.5), -1), ([0.75, 0, 0], (1, 0, 0.5), 1),
    ([0, 0, 0], ([1, 0], 1), 0), ([0, 0, 0], ([1, 0], 0.5), -1), ([0.75, 0, 0], ([1, 0], 0.5), 1)])
def test_circle_constraint_signs(tog, x, args, sign):
    v = tog.circle_constraint(np.array(x, float), *args)
    assert np.sign(v) == sign


@pytest.mark.parametrize("x,args,sign", [
    ([0, 0, 0], (1, 0, 0, 1), 0), ([0, 0, 0], (1, 0, 0, 0.5), -1), ([0.75, 0, 0], (1, 0, 0, 0.5), 1),
    ([0, 0, 0], ([1, 0, 0], 1), 0), ([0, 0, 0], ([1, 0, 0], 0.5), -1), ([0.75, 0, 0], ([1, 0, 0], 0.5), 1)])
def test_sphere_constraint_signs(tog, x, args, sign):
    v = tog.sphere_constraint(np.array(x, float), *args)
    assert np.sign(v) == sign


def test_circle_sphere_rows_oracle(tog, oracle):
    """The oracle's circle/sphere rows equal the utils.jl formulas (quadrotor state, stage knot)."""
    n, m, N = 13, 4, 2
    circles = [(1.0, 0.0, 1.0), (1.0, 0.0, 0.5), (0.2, -0.3, 0.7)]
    spheres = [(1.0, 0.0, 0.0, 1.0), (1.0, 0.0, 0.0, 0.5), (0.1, 0.2, 0.3, 2.0)]
    cons = tog.Constraints(N)
    cons[0] += tog.CircleConstraints(n, m, circles)
    cons[0] += tog.SphereConstraints(n, m, spheres)
    obj = tog.LQRObjective(np.eye(n), np.eye(m), np.eye(n), np.zeros(n), N)
    prob = tog.Problem(tog.rk4(tog.Dynamics.quadrotor), obj, np.zeros((N - 1, m)), constraints=cons,
                       x0=np.zeros(n), N=N, dt=0.1)
    s = oracle.OracleSolver(prob, tog.AugmentedLagrangianSolverOptions())
    x = np.zeros(n)
    x[:3] = [0.75, 0.1, -0.2]
    s.set("X", np.stack([x, x]))
    s.set("U", np.zeros((1, m)))
    s.update_constraints()
    C = s.get("C")[0]
    want = [tog.circle_constraint(x, *c) for c in circles] + [tog.sphere_constraint(x, *sp) for sp in spheres]
    np.testing.assert_allclose(C[:6], want, rtol=0, atol=1e-15)


# ------------------------------------------------------------------ costs (cost_tests.jl:40-95)

def test_lqr_cost_constructors(tog):
    """cost_tests.jl:49-58: LQRCost q = -Q xf, LQRCostTerminal q = -Qf xf."""
    rng = np.random.default_rng(3)
    n, m = 4, 2
    Q, R, Qf = np.diag(rng.random(n)), np.diag(rng.random(m)), np.diag(rng.random(n))
    xf = rng.random(n)
    c = tog.LQRCost(Q, R, xf)
    assert np.array_equal(c.q, -Q @ xf)
    assert np.isclose(c.c, 0.5 * xf @ Q @ xf)
    ct = tog.LQRCostTerminal(Qf, xf)
    assert np.array_equal(ct.Q, Qf)
    assert np.array_equal(ct.q, -Qf @ xf)


def test_stage_and_terminal_cost_oracle(tog, oracle):
    """cost_tests.jl:61-64: stage_cost == ½(x'Qx + u'Ru)dt (xf = 0), terminal ≈ ½(x-xf)'Qf(x-xf);
    evaluated by the oracle's cost() on a 2-knot trajectory."""
    rng = np.random.default_rng(4)
    n, m, N = 3, 2, 2
    Q, R, Qf = np.diag(rng.random(n) + 0.1), np.diag(rng.random(m) + 0.1), np.diag(rng.random(n) + 0.1)
    x, u, xN = rng.random(n), rng.random(m), rng.random(n)
    xf = rng.random(n)
    dt = float(rng.random())
    obj = tog.Objective(tog.QuadraticCost(Q, R), tog.LQRCostTerminal(Qf, xf), N=N)
    prob = tog.Problem(tog.rk3(tog.Dynamics.car), obj, u[None, :], x0=x, N=N, dt=dt)
    s = oracle.OracleSolver(prob, tog.iLQRSolverOptions())
    s.set("X", np.stack([x, xN]))
    s.set("U", u[None, :])
    J = s.cost()
    want = 0.5 * (x @ Q @ x + u @ R @ u) * dt + 0.5 * (xN - xf) @ Qf @ (xN - xf)
    assert J == pytest.approx(want, rel=1e-13)


# ------------------------------------------------------------------ dynamics Jacobians (model_tests.jl)

def fd_jacobian(oracle, model, integ, x, u, dt, h=1e-6):
    z = np.concatenate([x, u])
    n = len(x)
    J = np.zeros((n, len(z)))
    for i in range(len(z)):
        zp, zm = z.copy(), z.copy()
        zp[i] += h
        zm[i] -= h
        fp = oracle.discrete_f(model.model_id, integ, zp[:n], zp[n:], dt)
        fm = oracle.discrete_f(model.model_id, integ, zm[:n], zm[n:], dt)
        J[:, i] = (fp - fm) / (2 * h)
    return J


@pytest.mark.parametrize("name", ["doubleintegrator", "pendulum", "car", "cartpole", "quadrotor"])
@pytest.mark.parametrize("integ", ["rk3", "rk4"])
def test_dual_jacobian_vs_finite_differences(tog, oracle, name, integ):
    """model_tests.jl:108-157,193-208 pin the ForwardDiff Jacobian of the discrete map; here the
    oracle's dual-number Jacobian is checked against central differences of the same map."""
    model = getattr(tog.Dynamics, name)
    ig = tog.abi.RK4 if integ == "rk4" else tog.abi.RK3
    rng = np.random.default_rng(5)
    x = 0.5 * rng.standard_normal(model.n)
    if name == "quadrotor":
        x[3:7] = [1, 0.1, -0.2, 0.05]
    u = 0.5 * rng.standard_normal(model.m)
    S = oracle.discrete_jacobian(model.model_id, ig, x, u, 0.05)
    J = fd_jacobian(oracle, model, ig, x, u, 0.05)
    np.testing.assert_allclose(S[:, :model.n + model.m], J, rtol=1e-6, atol=1e-7)


def test_double_integrator_jacobian_exact(tog, oracle):
    """A linear map: the dual-number Jacobian equals the closed form of RK3 on ẋ=[x2; u] exactly."""
    dt = 0.1
    S = oracle.discrete_jacobian(tog.Dynamics.doubleintegrator.model_id, tog.abi.RK3, np.array([0.3, -0.2]),
                                 np.array([0.7]), dt)
    # RK3 of a double integrator: x1+ = x1 + dt x2 + dt²/2 u, x2+ = x2 + dt u
    A = np.array([[1.0, dt], [0.0, 1.0]])
    Bm = np.array([[dt * dt / 2], [dt]])
    np.testing.assert_allclose(S[:, :2], A, rtol=0, atol=1e-15)
    np.testing.assert_allclose(S[:, 2:3], Bm, rtol=0, atol=1e-15)


# ------------------------------------------------------------------ sqrt backward pass (sqrt_bp_tests.jl)

def _bp(tog, oracle, prob, sqrt, al):
    ilqr = tog.iLQRSolverOptions(square_root=sqrt)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr) if al else ilqr
    s = oracle.OracleSolver(prob, opts)
    s.rollout_open_loop()
    if al:
        s.update_constraints()
    s.jacobians()
    assert s.cost_expansion(sqrt=sqrt, al=al) == 0
    dV, _ = s.backward(sqrt=sqrt)
    S = s.get("S")
    if sqrt:
        S = np.einsum("kji,kjl->kil", S, S)  # S.xx = Ssqrt' Ssqrt
    return dV, s.get("K"), s.get("d"), S, s.get("Sx")


@pytest.mark.parametrize("constrained", [False, True])
def test_sqrt_backward_pass_equivalence(tog, oracle, constrained):
    """sqrt_bp_tests.jl:1-85 — the reference's single most important parity pin: std and sqrt
    backward passes agree (isapprox, rtol √eps) on ΔV, K, d, S.xx (= S'S) and S.x, unconstrained and
    with bounds ±5 + goal under AL."""
    prob = tog.Problems.car_sqrt_bp(constrained=constrained)
    a = _bp(tog, oracle, prob, False, constrained)
    b = _bp(tog, oracle, prob, True, constrained)
    assert isapprox(b[0], a[0])
    assert isapprox(b[1], a[1])
    assert isapprox(b[2], a[2])
    for k in range(prob.N):
        assert isapprox(b[3][k], a[3][k]), k
        assert isapprox(b[4][k], a[4][k]), k


# ------------------------------------------------------------------ end-to-end thresholds

def _solve(tog, oracle, prob, opts):
    s = oracle.OracleSolver(prob, opts)
    s.solve()
    return s


QUAD_OPTS = dict(cost_tolerance=1e-5)


def _quad_opts(tog):
    ilqr = tog.iLQRSolverOptions(**QUAD_OPTS)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr, constraint_tolerance=1e-3, cost_tolerance=1e-5,
                                              cost_tolerance_intermediate=1e-4)
    return ilqr, al


def test_quadrotor_ilqr_reaches_goal(tog, oracle):
    """quadrotor_tests.jl:38-43: unconstrained iLQR, ‖X_N - xf‖ < 5e-3."""
    ilqr, _ = _quad_opts(tog)
    prob = tog.Problems.quadrotor_test("none")
    s = _solve(tog, oracle, prob, ilqr)
    assert np.linalg.norm(s.get("X")[-1] - prob.xf) < 5e-3


@pytest.mark.parametrize("cons", ["goal", "goal+bounds", "goal+bounds+obs"])
def test_quadrotor_al_constraint_tolerance(tog, oracle, cons):
    """quadrotor_tests.jl:45-84: AL with goal / goal+bounds u∈[0,15] / + 3 spheres reaches
    max_violation < constraint_tolerance and the goal within it."""
    _, al = _quad_opts(tog)
    prob = tog.Problems.quadrotor_test(cons)
    s = _solve(tog, oracle, prob, al)
    X = s.get("X")
    assert s.max_violation() < al.constraint_tolerance
    assert np.linalg.norm(X[-1] - prob.xf, np.inf) < al.constraint_tolerance
    if cons == "goal+bounds":
        assert np.linalg.norm(X[-1] - prob.xf) < al.constraint_tolerance


def test_car_parallel_park(tog, oracle):
    """car_tests.jl:28-32: parallel park, iLQR (cost_tolerance 1e-5), ‖X_N - xf‖ < 1e-3."""
    prob = tog.Problems.car_parallel_park()
    s = _solve(tog, oracle, prob, tog.iLQRSolverOptions(cost_tolerance=1e-5))
    assert np.linalg.norm(s.get("X")[-1] - prob.xf) < 1e-3


@pytest.mark.parametrize("integ", ["midpoint", "rk3", "rk4"])
def test_pendulum_altro(tog, oracle, integ):
    """pendulum_tests.jl:23-27 (the explicit schemes :midpoint, :rk3, :rk4): AL (ALTRO phase 1) with
    penalty_scaling=10, 50 outer iterations reaches max_violation < constraint_tolerance."""
    ilqr = tog.iLQRSolverOptions()
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr, iterations=50, penalty_scaling=10.0)
    prob = tog.Problems.pendulum(integ)
    s = _solve(tog, oracle, prob, tog.ALTROSolverOptions(opts_al=al))
    assert s.max_violation() < al.constraint_tolerance


def test_doubleintegrator_altro(tog, oracle):
    """Config 1 (README quick-start, problems/doubleintegrator.jl): ALTRO defaults converge."""
    prob, opts = tog.Problems.config_doubleintegrator()
    s = _solve(tog, oracle, prob, opts)
    assert s.max_violation() < opts.opts_al.constraint_tolerance


def test_undefined_integration_raises(tog):
    """pendulum_tests.jl:30: Problem(model, obj, integration=:bogus) throws ArgumentError."""
    prob = tog.Problems.pendulum()
    with pytest.raises(ValueError):
        tog.Problem(tog.Dynamics.pendulum, prob.obj, integration="bogus", N=prob.N, dt=prob.dt)
    # the implicit Newton step is instantiated for models with n <= 4, the quadrotor and the Kuka arm
    # (csrc/tog_device.hpp implicit_step, KukaImplicit), not for user plugin models with n > 4
    assert tog.discretize_model(tog.Dynamics.pendulum, "midpoint_implicit").integration == tog.abi.MIDPOINT_IMPLICIT
    with pytest.raises(NotImplementedError):
        tog.discretize_model(tog.Model(tog.abi.MODEL_USER, 5, 2, "user5"), "midpoint_implicit")


def test_midpoint_jacobian_matches_central_differences(tog, oracle):
    """The dual-number midpoint Jacobian (src/integration.jl:26-33 under ForwardDiff) equals
    central differences of the oracle's midpoint step, for every model."""
    rng = np.random.default_rng(5)
    for mid in range(tog.abi.MODEL_KUKA):
        n, m = tog.abi.MODEL_NM[mid]
        x, u = 0.3 * rng.standard_normal(n), 0.3 * rng.standard_normal(m)
        if mid == tog.abi.MODEL_QUADROTOR:
            x[3:7] = [1, 0.1, -0.2, 0.05]
        S = oracle.discrete_jacobian(mid, tog.abi.MIDPOINT, x, u, 0.05)
        z = np.concatenate([x, u])
        for j in range(n + m):
            e = np.zeros(n + m)
            e[j] = 1e-6
            fp = oracle.discrete_f(mid, tog.abi.MIDPOINT, (z + e)[:n], (z + e)[n:], 0.05)
            fm = oracle.discrete_f(mid, tog.abi.MIDPOINT, (z - e)[:n], (z - e)[n:], 0.05)
            assert np.allclose(S[:, j], (fp - fm) / 2e-6, rtol=1e-6, atol=1e-7), (mid, j)


def _notebook_quadrotor(tog):
    """examples/quadrotor/Quadrotor.ipynb cells 3-11: rk3(Dynamics.quadrotor), N = 101, dt = 0.1,
    Q = R = 1e-2 I, Qf = 1000 I, x0 at the origin, xf = (0, 50, 0), hover controls, no constraints."""
    n, m, N = 13, 4, 101
    q0 = np.array([1.0, 0.0, 0.0, 0.0])
    x0 = np.zeros(n)
    x0[3:7] = q0
    xf = np.zeros(n)
    xf[0:3] = [0.0, 50.0, 0.0]
    xf[3:7] = q0
    obj = tog.LQRObjective(1e-2 * np.eye(n), 1e-2 * np.eye(m), 1000.0 * np.eye(n), xf, N)
    U = 0.5 * 9.81 / 4.0 * np.ones((N - 1, m))
    return tog.Problem(tog.rk3(tog.Dynamics.quadrotor), obj, U, x0=x0, xf=xf, N=N, dt=0.1)


def test_quadrotor_notebook_final_cost(tog, oracle):
    """The reference's own output for the quadrotor model: Quadrotor.ipynb cell 13 logs the converged
    iLQR cost 18.17292526 (solve!(prob, iLQRSolverOptions{T}(verbose=true))). The oracle reaches
    18.17294801 in 58 steps: 1.25e-6 relative. The notebook ran an older snapshot of the package (its
    last logged step has α = 0.25, dJ = 2.36e-5, against α = 0.5, dJ = 5.9e-5 here), so iteration
    counts are not comparable; the converged cost is, to within the cost tolerance's last step
    (cost_tolerance = 1e-4 stops when 0 < dJ < 1e-4, i.e. within ~5.5e-6 relative of 18.17)."""
    prob = _notebook_quadrotor(tog)
    s = oracle.OracleSolver(prob, tog.iLQRSolverOptions())
    s.solve()
    J = s.get("stats")[tog.abi.STAT_J]
    assert abs(J - 18.17292526) / 18.17292526 < 5e-6


@pytest.mark.gpu
def test_quadrotor_notebook_device(tog, gpu, oracle):
    """The same notebook problem on the device equals the oracle (and so the notebook's cost)."""
    prob = _notebook_quadrotor(tog)
    s = oracle.OracleSolver(prob, tog.iLQRSolverOptions())
    steps = s.solve()
    gp = prob.copy()
    solver = tog.solve_b(gp, tog.iLQRSolverOptions())
    assert solver.stats["iterations_total"][0] == steps
    assert np.abs(gp.X - s.get("X")).max() / max(1.0, np.abs(s.get("X")).max()) < 1e-6
    assert np.abs(gp.U - s.get("U")).max() / max(1.0, np.abs(s.get("U")).max()) < 1e-6
    assert abs(solver.stats["cost"][0] - 18.17292526) / 18.17292526 < 5e-6


# Untrimmed bounds (BoundConstraint(trim=false), src/constraints.jl:182-186). The reference's own KAT for
# them is commented out in test/constraint_tests.jl:65-78; its values are the ones below.
V_STAGE_UNTRIM = [-4, -3, -math.inf, -5, 5, -11, -7, -3, -5, -15]
V_TERM_UNTRIM = [-4, -3, -math.inf, -11, -7, -3]


def untrimmed_kat_problem(tog):
    n, m, N = 3, 2, 2
    bnd = tog.BoundConstraint(n, m, x_max=[5, 5, math.inf], x_min=[-10, -5, 0.0], u_min=-10.0, u_max=0.0, trim=False)
    obj = tog.LQRObjective(np.eye(n), np.eye(m), np.eye(n), np.zeros(n), N)
    cons = tog.Constraints([bnd], N)
    prob = tog.Problem(tog.rk3(tog.Dynamics.car), obj, np.zeros((N - 1, m)), constraints=cons, x0=np.zeros(n),
                       N=N, dt=0.1)
    return prob, bnd


def test_untrimmed_bound_kat_host(tog):
    _, bnd = untrimmed_kat_problem(tog)
    n, m = 3, 2
    assert bnd.length("stage") == 2 * (n + m) and bnd.length("terminal") == 2 * n
    assert list(bnd.evaluate(X_KAT, U_KAT)) == V_STAGE_UNTRIM
    assert list(bnd.evaluate(X_KAT)) == V_TERM_UNTRIM
    jac = bnd.jacobian(X_KAT, U_KAT)
    assert np.array_equal(jac[:, :n], np.vstack([np.eye(n), np.zeros((m, n)), -np.eye(n), np.zeros((m, n))]))
    assert np.array_equal(jac[:, n:], np.vstack([np.zeros((n, m)), np.eye(m), np.zeros((n, m)), -np.eye(m)]))


def test_untrimmed_bound_kat_oracle(tog, oracle):
    """The oracle keeps every row of an untrimmed bound (tog_constraint count = 1)."""
    prob, _ = untrimmed_kat_problem(tog)
    s = oracle.OracleSolver(prob, tog.AugmentedLagrangianSolverOptions())
    s.set("X", np.stack([X_KAT, X_KAT]))
    s.set("U", U_KAT[None, :])
    s.update_constraints()
    C = s.get("C")
    assert list(C[0, :10]) == V_STAGE_UNTRIM
    assert list(C[1, :6]) == V_TERM_UNTRIM
    # an infinite bound's row makes the AL cost NaN (λ'c with λ = 0, c = -Inf), as in the reference
    assert math.isnan(s.cost(al=True))


def test_untrimmed_finite_bounds_solve_like_trimmed(tog, oracle):
    """With every bound finite, trim=false changes nothing: the oracle's solves agree bit for bit."""
    out = []
    for trim in (True, False):
        p = tog.Problems.pendulum("rk3")
        n, m = p.model.n, p.model.m
        cons = tog.Constraints(p.N)
        bnd = tog.BoundConstraint(n, m, x_min=[-10.0, -10.0], x_max=[10.0, 10.0], u_min=-3.0, u_max=3.0, trim=trim)
        for k in range(p.N - 1):
            cons[k] += bnd
        cons[p.N - 1] += tog.goal_constraint(p.xf)
        q = tog.Problem(p.model, p.obj, p._U[0], constraints=cons, x0=p.x0[0], xf=p.xf, N=p.N, dt=p.dt)
        o = oracle.OracleSolver(q, tog.AugmentedLagrangianSolverOptions(iterations=5), b=0)
        steps = o.solve()
        out.append((steps, o.get("X"), o.get("U")))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])


@pytest.mark.gpu
def test_gpu_untrimmed_bound_rows(tog, oracle, gpu):
    """Device constraint values of the untrimmed KAT equal the oracle's (tog_update_constraints)."""
    prob, _ = untrimmed_kat_problem(tog)
    solver = tog.AugmentedLagrangianSolver(prob, tog.AugmentedLagrangianSolverOptions())
    prob._X[0] = np.stack([X_KAT, X_KAT])
    prob._U[0] = U_KAT[None, :]
    solver.handle.upload_state(prob)
    tog.update_constraints_b(prob, solver)
    C = solver.handle.get(tog.abi.FIELD_C)[0]
    assert list(C[0, :10]) == V_STAGE_UNTRIM
    assert list(C[1, :6]) == V_TERM_UNTRIM
