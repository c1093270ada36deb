"""User models: ``Model(f!, n, m)`` (src/model.jl:103-131) as libtog plugins (csrc/tog_plugin.hpp).

A plugin instantiates every kernel of the path for the user's dynamics; libtog loads it with
``tog_model_load`` and dispatches through the same ModelOps table as its built-in models.

* ``plugins/user_pendulum.hip`` restates the reference's pendulum (dynamics/pendulum.jl:3-12) through
  the plugin API. Its solves must equal the built-in model's bit for bit, and the CPU oracle's.
* ``problems.UNICYCLE_F`` is a model the library does not have, compiled from source by
  ``user_model`` (build() fills the in-tree cache). Its dual-number Jacobians are checked against
  central differences of the device rollout, and its AL solve must reach the goal.
"""
import ctypes as C
import pathlib

import numpy as np
import pytest

PLUG = pathlib.Path(__file__).resolve().parents[1] / "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd" / "csrc" / "plugins"


def test_plugin_load_and_dims(tog):
    m = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    assert (m.n, m.m, m.model_id) == (2, 1, tog.abi.MODEL_USER)
    u = tog.Model.from_plugin(PLUG / "user_unicycle.so")
    assert (u.n, u.m) == (5, 2)
    # discretisation and slack controls keep the plugin (src/model.jl:607-615, 761-779)
    d = tog.add_slack_controls(tog.rk3(u))
    assert d.plugin is u.plugin and (d.n, d.m, d.slack) == (5, 7, 5)


def test_plugin_errors(tog):
    lib = tog.abi.load_library()
    h = C.c_void_p()
    assert lib.tog_model_load(b"/nonexistent/plugin.so", C.byref(h)) == tog.abi.ERR_ARG and not h.value
    # a shared object without the TOG_PLUGIN symbols (libtog itself) is refused
    assert lib.tog_model_load(str(tog.abi.LIB_PATH).encode(), C.byref(h)) == tog.abi.ERR_ARG
    assert b"TOG_PLUGIN" in lib.tog_last_error()
    # a user-model problem without a loaded model is refused at tog_create
    prob = tog.Problems.pendulum(model=tog.Model.from_plugin(PLUG / "user_pendulum.so"))
    b = prob.build_desc()
    b.desc.user_model = None
    o = tog.to_tog_options(tog.AugmentedLagrangianSolverOptions())
    assert lib.tog_create(C.byref(b.desc), C.byref(o), 0, C.byref(h)) in (tog.abi.ERR_UNSUPPORTED, tog.abi.ERR_DEVICE)


def test_user_model_source_generation(tog):
    """user_model() compiles a generated plugin once per source (hash-keyed in-tree cache)."""
    m1 = tog.Problems.unicycle_model()
    m2 = tog.Problems.unicycle_model()
    assert m1.plugin is m2.plugin and (m1.n, m1.m) == (5, 2)
    assert pathlib.Path(m1.plugin.path).parent == PLUG and pathlib.Path(m1.plugin.path).name.startswith("gen_Unicycle_")


@pytest.mark.gpu
@pytest.mark.parametrize("integration", ["rk3", "rk4"])
def test_user_pendulum_equals_builtin_and_oracle(tog, oracle, gpu, integration):
    user = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    opts = tog.AugmentedLagrangianSolverOptions()
    p_user = tog.Problems.pendulum(integration, model=user)
    p_builtin = tog.Problems.pendulum(integration)
    s_user = tog.solve_b(p_user, opts)
    s_builtin = tog.solve_b(p_builtin, opts)
    assert np.array_equal(p_user._X, p_builtin._X) and np.array_equal(p_user._U, p_builtin._U)
    assert np.array_equal(s_user.stats["iterations_total"], s_builtin.stats["iterations_total"])
    ref = oracle.OracleSolver(tog.Problems.pendulum(integration), opts, b=0)
    ref.solve()
    X, U = ref.get("X"), ref.get("U")
    assert np.max(np.abs(p_user._X[0] - X)) <= 1e-6 * max(1.0, np.max(np.abs(X)))
    assert np.max(np.abs(p_user._U[0] - U)) <= 1e-6 * max(1.0, np.max(np.abs(U)))


@pytest.mark.gpu
def test_user_pendulum_jacobians_equal_builtin(tog, gpu):
    user = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    out = []
    for model in (user, None):
        prob = tog.Problems.pendulum("rk4", model=model)
        solver = tog.AugmentedLagrangianSolver(prob, tog.AugmentedLagrangianSolverOptions())
        h = solver.handle
        h.upload_state(prob)
        tog.abi.check(h.lib, h.lib.tog_rollout_open_loop(h.h))
        tog.abi.check(h.lib, h.lib.tog_jacobians(h.h))
        out.append(h.get(tog.abi.FIELD_A).copy())
    assert np.array_equal(out[0], out[1])


@pytest.mark.gpu
def test_user_unicycle_jacobian_and_solve(tog, gpu):
    model = tog.Problems.unicycle_model()
    B = 8
    prob = tog.Problems.unicycle(model, B=B)
    opts = tog.AugmentedLagrangianSolverOptions()
    solver = tog.AugmentedLagrangianSolver(prob, opts)
    h = solver.handle
    h.upload_state(prob)
    tog.abi.check(h.lib, h.lib.tog_rollout_open_loop(h.h))
    tog.abi.check(h.lib, h.lib.tog_jacobians(h.h))
    A, Bm = h.get(tog.abi.FIELD_A), h.get(tog.abi.FIELD_B)
    X = h.get(tog.abi.FIELD_X)
    n, m, N, dt = 5, 2, prob.N, prob.dt
    # central differences of the discrete step (rk3 of the same f, evaluated on the host)
    def f(x, u):
        return np.array([x[3] * np.cos(x[2]), x[3] * np.sin(x[2]), x[4], u[0] - 0.1 * x[3], u[1] - 0.2 * x[4]])

    def step(x, u):
        k1 = f(x, u) * dt
        k2 = f(x + k1 / 2, u) * dt
        k3 = f(x - k1 + 2 * k2, u) * dt
        return x + (k1 + 4 * k2 + k3) / 6

    U = prob._U
    for b in (0, 5):
        for k in (0, 17, N - 2):
            x, u = X[b, k], U[b, k]
            assert np.allclose(step(x, u), X[b, k + 1], rtol=1e-12, atol=1e-12)
            eps = 1e-6
            Jx = np.stack([(step(x + eps * e, u) - step(x - eps * e, u)) / (2 * eps) for e in np.eye(n)], 1)
            Ju = np.stack([(step(x, u + eps * e) - step(x, u - eps * e)) / (2 * eps) for e in np.eye(m)], 1)
            assert np.allclose(A[b, k], Jx, rtol=1e-6, atol=1e-8)
            assert np.allclose(Bm[b, k], Ju, rtol=1e-6, atol=1e-8)
    s = tog.solve_b(prob, opts)
    flags = s.stats["flags"]
    assert np.all(flags & tog.abi.TRAJ_AL_CONVERGED)
    assert np.all(np.abs(prob._X[:, -1] - np.array([2.0, 1.0, 0, 0, 0])) < 1e-2)


def test_user_constraint_rows_cpu(tog):
    """UserConstraint marshals as TOG_CON_USER; a model without con() is refused at tog_create."""
    uc = tog.UserConstraint(2, 1, 1, fid=0, label="obstacle")
    t, cnt, data = uc.to_abi()
    assert (t, cnt, list(data)) == (tog.abi.CON_USER, 1, [0.0, 0.0, 0.0])
    assert uc.length("stage") == 1 and uc.length("terminal") == 0
    assert np.isnan(uc.evaluate(np.zeros(2), np.zeros(1))).all()
    prob = tog.Problems.pendulum(stage_constraints=(uc,))  # built-in pendulum: no con()
    lib = tog.abi.load_library()
    b = prob.build_desc()
    o = tog.to_tog_options(tog.AugmentedLagrangianSolverOptions())
    h = C.c_void_p()
    rc = lib.tog_create(C.byref(b.desc), C.byref(o), 0, C.byref(h))
    assert rc in (tog.abi.ERR_ARG, tog.abi.ERR_DEVICE) and not h.value


@pytest.mark.gpu
def test_user_circle_constraint_equals_builtin_and_oracle(tog, oracle, gpu):
    """A circle obstacle as a user constraint function (plugin con, fid 0; dense dual Jacobian, LDS
    backward kernel) against the built-in circle rows (team backward kernel) and the oracle."""
    user = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    opts = tog.AugmentedLagrangianSolverOptions()
    circ = tog.CircleConstraints(2, 1, [[1.2, 2.5, 0.6]])
    p_user = tog.Problems.pendulum(model=user, stage_constraints=(tog.UserConstraint(2, 1, 1, fid=0),))
    p_builtin = tog.Problems.pendulum(stage_constraints=(circ,))
    s_user = tog.solve_b(p_user, opts)
    s_builtin = tog.solve_b(p_builtin, opts)
    assert np.array_equal(p_user._X, p_builtin._X) and np.array_equal(p_user._U, p_builtin._U)
    assert np.array_equal(s_user.stats["iterations_total"], s_builtin.stats["iterations_total"])
    ref = oracle.OracleSolver(tog.Problems.pendulum(stage_constraints=(circ,)), opts, b=0)
    ref.solve()
    X, U = ref.get("X"), ref.get("U")
    assert np.max(np.abs(p_user._X[0] - X)) <= 1e-6 * max(1.0, np.max(np.abs(X)))
    assert np.max(np.abs(p_user._U[0] - U)) <= 1e-6 * max(1.0, np.max(np.abs(U)))


@pytest.mark.gpu
def test_user_constraints_unicycle_solve(tog, gpu):
    """State (obstacle) and control-dependent (traction a·v <= 1) user rows on a user model."""
    model = tog.Problems.unicycle_model()
    prob = tog.Problems.unicycle(model, B=8, user_constraints=True)
    opts = tog.AugmentedLagrangianSolverOptions()
    s = tog.solve_b(prob, opts)
    assert np.all(s.stats["flags"] & tog.abi.TRAJ_AL_CONVERGED)
    cmax = tog.max_violation(prob)
    assert np.all(cmax < opts.constraint_tolerance)
    assert np.all(np.abs(prob._X[:, -1] - np.array([2.0, 1.0, 0, 0, 0])) < 1e-2)


@pytest.mark.gpu
def test_user_pendulum_min_time_equals_builtin(tog, gpu):
    """minimum_time_problem on a user model (the plugin's MinTime<M>, add_min_time_controls
    minimum_time.jl:83-104): ALTRO with tf = :min on the user pendulum equals the same solve on the built-in
    pendulum bit for bit (X, U, the time steps h, every statistic); the built-in one is held to the oracle
    by tests/test_minimum_time.py."""
    import math

    user = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    n, m, N = 2, 1, 31
    Q, R = 1e-3 * np.eye(n), 1e-3 * np.eye(m)
    xf, x0 = np.array([math.pi, 0.0]), np.zeros(n)

    def make(model):
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=-5.0, u_max=5.0)
        for k in range(N - 1):
            cons[k] += bnd
        cons[N - 1] += tog.goal_constraint(xf)
        U0 = np.ones((N - 1, m)) + 0.1 * np.sin(np.arange(N - 1))[:, None]
        return tog.Problem(tog.rk3(model), tog.LQRObjective(Q, R, Q, xf, N), U0, constraints=cons, dt=0.075,
                           x0=x0, N=N, tf="min")

    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), iterations=50, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=15.0, dt_max=0.15, dt_min=1.0e-3)
    pu, pb = make(user), make(tog.Dynamics.pendulum)
    su = tog.solve_b(pu, opts.copy())
    sb = tog.solve_b(pb, opts.copy())
    assert np.array_equal(pu._X, pb._X) and np.array_equal(pu._U, pb._U)
    assert np.array_equal(pu.h, pb.h)
    for key in ("iterations_total", "flags", "cost", "c_max"):
        assert np.array_equal(su.stats[key], sb.stats[key]), key
    assert 0.0 < tog.total_time(pu) < math.inf


@pytest.mark.gpu
def test_user_constraint_min_time_equals_builtin_and_oracle(tog, oracle, gpu):
    """Minimum time with user constraint rows (round 6; mintime_constraints keeps every constraint over the base
    model's x, u, minimum_time.jl:125-141): tf = :min on the user pendulum with its circle as a user function
    (MinTime<M>::con) equals the built-in pendulum with CircleConstraints bit for bit, and that one equals the
    oracle's minimum-time flow within 1e-6."""
    import math

    user = tog.Model.from_plugin(PLUG / "user_pendulum.so")
    n, m, N = 2, 1, 31
    Q, R = 1e-3 * np.eye(n), 1e-3 * np.eye(m)
    xf, x0 = np.array([math.pi, 0.0]), np.zeros(n)

    def make(model, con):
        cons = tog.Constraints(N)
        bnd = tog.BoundConstraint(n, m, u_min=-5.0, u_max=5.0)
        for k in range(N - 1):
            cons[k] += bnd
            cons[k] += con
        cons[N - 1] += tog.goal_constraint(xf)
        U0 = np.ones((N - 1, m)) + 0.1 * np.sin(np.arange(N - 1))[:, None]
        return tog.Problem(tog.rk3(model), tog.LQRObjective(Q, R, Q, xf, N), U0, constraints=cons, dt=0.075,
                           x0=x0, N=N, tf="min")

    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), iterations=30, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al, R_minimum_time=15.0, dt_max=0.15, dt_min=1.0e-3)
    circ = tog.CircleConstraints(2, 1, [[1.2, 2.5, 0.6]])
    pu = make(user, tog.UserConstraint(2, 1, 1, fid=0))
    pb = make(tog.Dynamics.pendulum, circ)
    ref = pb.copy()
    su = tog.solve_b(pu, opts.copy())
    sb = tog.solve_b(pb, opts.copy())
    assert np.array_equal(pu._X, pb._X) and np.array_equal(pu._U, pb._U) and np.array_equal(pu.h, pb.h)
    for key in ("iterations_total", "flags", "cost", "c_max"):
        assert np.array_equal(su.stats[key], sb.stats[key]), key
    Xo, Uo, ho, so = oracle.solve_altro_min_time(ref, opts.copy(), 0)
    assert np.max(np.abs(pb._X[0] - Xo)) <= 1e-6 * max(1.0, np.max(np.abs(Xo)))
    assert np.max(np.abs(pb._U[0] - Uo)) <= 1e-6 * max(1.0, np.max(np.abs(Uo)))
    assert np.max(np.abs(pb.h[0] - ho)) <= 1e-6
