"""Infeasible start: ``infeasible_problem`` + slack controls + the ALTRO
infeasible-start flow (src/solvers/altro/infeasible.jl:2-99, altro_methods.jl:2-124,
src/model.jl:761-779, src/constraints.jl:306-314).

CPU tests pin the oracle on the reference's own assertions (test/infeasible_tests.jl,
test/constraint_tests.jl:189-194); the ``gpu`` tests hold libtog.so (Infeasible<M> kernels, through
the C ABI) bit-for-bit to the oracle, and solves to the north-star 1e-6 with equal iteration counts.
"""
import numpy as np
import pytest

TOL_SOLVE = 1e-6
TOL_STEP = 1e-13


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def pendulum_opts(tog, resolve):
    """test/infeasible_tests.jl:11-19."""
    opts_ilqr = tog.iLQRSolverOptions()
    opts_al = tog.AugmentedLagrangianSolverOptions(constraint_tolerance=1e-5, cost_tolerance=1e-5,
                                                   cost_tolerance_intermediate=1e-5, opts_uncon=opts_ilqr,
                                                   iterations=30, penalty_scaling=10.0)
    return tog.ALTROSolverOptions(opts_al=opts_al, R_inf=1.0, resolve_feasible_problem=resolve)


def pendulum_line(tog, constrained_variant=False):
    """test/infeasible_tests.jl:21-45: Problems.pendulum with X0 = line_trajectory(x0, xf, N)."""
    prob = tog.Problems.pendulum()
    if constrained_variant:  # Constraints([bnd], N); constraints[N] += goal
        n, m, N = 2, 1, prob.N
        bnd = tog.BoundConstraint(n, m, u_min=-3.0, u_max=3.0)
        cons = tog.Constraints([bnd], N)
        cons[N - 1] = cons[N - 1] + tog.goal_constraint(prob.xf)
        prob = tog.Problem(prob.model, prob.obj, prob.U, constraints=cons, x0=prob.x0[0], xf=prob.xf, N=N,
                           dt=prob.dt)
    prob.X = tog.line_trajectory(prob.x0[0], prob.xf, prob.N)
    return prob


def quad_line_batch(tog, B=3, N=31, seed=7):
    """Quadrotor (test/quadrotor_tests.jl:4-35 model and costs, u in [0, 15] + goal), N shortened,
    batched random starts with a straight-line state guess x0 -> xf per trajectory (the
    quadrotor_maze initial-guess path, problems/quadrotor_maze.jl:107-114). Not line_trajectory:
    that one is slope*t without the x0 offset (infeasible.jl:82-90), which zeroes the quaternion."""
    p0 = tog.Problems.quadrotor_test("goal+bounds")
    n, m = 13, 4
    rng = np.random.default_rng(seed)
    x0 = np.tile(p0.x0[0], (B, 1))
    x0[:, 0:3] += rng.standard_normal((B, 3))
    U0 = 0.5 * 9.81 / 4 + 0.1 * rng.standard_normal((B, N - 1, m))
    xf = p0.xf
    cons = tog.Constraints(N)
    bnd = tog.BoundConstraint(n, m, u_min=0.0, u_max=15.0)
    for k in range(N - 1):
        cons[k] += bnd
    cons[N - 1] += tog.goal_constraint(xf)
    obj = tog.LQRObjective(p0.obj.stage.Q, p0.obj.stage.R, p0.obj.terminal.Q, xf, N)
    prob = tog.Problem(p0.model, obj, U0, x0=x0, xf=xf, N=N, dt=0.05, constraints=cons)
    t = np.linspace(0.0, 1.0, N)[None, :, None]
    prob.X = x0[:, None, :] + (xf - x0)[:, None, :] * t
    return prob


# ----------------------------------------------------------------------------- CPU: host + oracle


def test_infeasible_constraint_kat(tog):
    """test/constraint_tests.jl:189-194: con_inf.c(v, x, u_inf[inds[2]]) == [5, -5, 10]."""
    n, m = 3, 2
    con = tog.infeasible_constraints(n, m)
    u_inf = np.concatenate([[0.3, -0.7], [5.0, -5.0, 10.0]])
    assert np.array_equal(con.evaluate(np.zeros(n), u_inf), [5.0, -5.0, 10.0])
    assert con.length("stage") == n and con.length("terminal") == 0 and not con.inequality
    J = con.jacobian(np.zeros(n), u_inf)
    assert J.shape == (n, 2 * n + m) and np.array_equal(J[:, n + m:], np.eye(n)) and not J[:, :n + m].any()
    # C_inf = [..., bnd, con_inf]: the stage vector is the plain one followed by the slacks (:196-202)
    bnd = tog.BoundConstraint(n, m, u_min=-1.0, u_max=1.0, x_max=2.0)
    x = np.array([0.5, 3.0, -1.0])
    v_stage = bnd.evaluate(x, u_inf[:m])
    v_inf = np.concatenate([bnd.evaluate(x, u_inf), con.evaluate(x, u_inf)])
    assert np.array_equal(v_inf, np.concatenate([v_stage, [5.0, -5.0, 10.0]]))


def test_infeasible_problem_structure(tog):
    """infeasible_problem (infeasible.jl:2-33): augmented R, zero-padded H/r, bounds moved after the
    other constraints (update_constraint_set_jacobians, constraint_sets.jl:135-150), slack
    equality appended at the stage knots only, controls [U; 0]."""
    prob = tog.Problems.quad_obs(N=21)
    n, m, N = 13, 4, prob.N
    prob.X = np.zeros((N, n))
    pinf = tog.infeasible_problem(prob, 0.5)
    assert pinf.model.m == m + n and pinf.model.slack == n and pinf.model.model_id == prob.model.model_id
    R = pinf.obj.stage.R
    assert np.array_equal(R[:m, :m], prob.obj.stage.R)
    assert np.array_equal(R[m:, m:], 0.5 * np.eye(n) / prob.dt) and not R[:m, m:].any()
    assert pinf.obj.stage.H.shape == (m + n, n) and not pinf.obj.stage.H[m:].any()
    for k in range(N - 1):
        kinds = [type(c).__name__ for c in pinf.constraints[k]]
        assert kinds[-1] == "InfeasibleConstraint"
        nb = [i for i, t in enumerate(kinds) if t == "BoundConstraint"]
        assert all(i > j for i in nb for j, t in enumerate(kinds[:-1]) if t != "BoundConstraint")
    assert all(type(c).__name__ != "InfeasibleConstraint" for c in pinf.constraints[N - 1])
    assert np.array_equal(pinf.U[:, :m], prob.U) and not pinf.U[:, m:].any()
    d = pinf.build_desc().desc
    assert d.flags == tog.abi.PROB_INFEASIBLE and d.m == m + n


def test_line_trajectory(tog):
    """line_trajectory (infeasible.jl:82-90): t = range(0, N, length=N), slope (xf-x0)/N."""
    X = tog.line_trajectory([0.0, 0.0], [np.pi, 0.0], 31)
    assert X.shape == (31, 2) and np.array_equal(X[0], [0, 0]) and np.array_equal(X[-1], [np.pi, 0])
    t = np.linspace(0, 31, 31)
    assert np.allclose(X[1:-1, 0], (np.pi / 31) * t[1:-1], rtol=0, atol=1e-15)


def test_oracle_slack_controls_and_jacobian(tog, oracle):
    """slack_controls (infeasible.jl:63-80) and the slack model (src/model.jl:761-779) in the oracle
    against a numpy restatement over the oracle's plain model."""
    prob = pendulum_line(tog)
    pinf = tog.infeasible_problem(prob, 1.0)
    o = oracle.OracleSolver(pinf, pendulum_opts(tog, False))
    o.slack_controls()
    U = o.get("U")
    X = prob.X
    x = prob.x0[0].copy()
    for k in range(prob.N - 1):
        xn = oracle.discrete_f(tog.abi.MODEL_PENDULUM, tog.abi.RK3, x, prob.U[k], prob.dt)
        s = X[k + 1] - xn
        assert np.array_equal(U[k, 1:], s), k
        assert np.array_equal(U[k, :1], prob.U[k])
        x = xn + s
    # the open-loop rollout of the slack model reproduces X (to rounding of x + (X - x))
    o.set("X", np.full((prob.N, 2), np.nan))
    o.rollout_open_loop()
    assert np.allclose(o.get("X"), X, rtol=0, atol=1e-14)
    o.jacobians()
    A, Bm = o.get("A"), o.get("B")
    for k in range(prob.N - 1):
        S = oracle.discrete_jacobian(tog.abi.MODEL_PENDULUM, tog.abi.RK3, o.get("X")[k], U[k, :1], prob.dt)
        assert np.array_equal(A[k], S[:, :2])
        assert np.array_equal(Bm[k][:, :1], S[:, 2:3])
        assert np.array_equal(Bm[k][:, 1:], np.eye(2))


@pytest.mark.parametrize("variant", [False, True])
def test_reference_infeasible_pendulum_oracle(tog, oracle, variant):
    """test/infeasible_tests.jl:23-55 on the oracle: ‖X_N − xf‖ < 1e-3 (first case),
    max_violation < constraint_tolerance (second), resolve ≈ no resolve to 1e-5."""
    Xend = {}
    for resolve in (False, True):
        prob = pendulum_line(tog, variant)
        opts = pendulum_opts(tog, resolve)
        X, U, si, sf = oracle.solve_altro_infeasible(prob, opts)
        Xend[resolve] = X[-1]
        if not variant:
            assert np.linalg.norm(X[-1] - prob.xf) < 1e-3
        else:
            p = prob.copy()
            p.X, p.U = X, U
            assert tog.max_violation(p) < opts.opts_al.constraint_tolerance
    assert np.linalg.norm(Xend[False] - Xend[True]) < 1e-5


# ----------------------------------------------------------------------------- GPU parity


@pytest.mark.gpu
def test_gpu_slack_controls_and_rollout(tog, oracle, gpu):
    """tog_slack_controls + Infeasible<Quadrotor> rollout / Jacobians vs the oracle, bitwise."""
    prob = quad_line_batch(tog, B=4, N=21)
    pinf = tog.infeasible_problem(prob, 1.0)
    opts = tog.ALTROSolverOptions()
    solver = tog.ALTROSolver(pinf, opts)
    h = solver.handle
    h.slack_controls()
    U = h.get(tog.abi.FIELD_U)
    for b in range(prob.B):
        o = oracle.OracleSolver(pinf, opts, b)
        o.slack_controls()
        assert rel(U[b], o.get("U")) == 0.0, b
    pinf._U[...] = U
    pinf._X[...] = np.nan
    h.upload_state(pinf)
    h.rollout_open_loop()
    h.jacobians()
    X, A, Bm = h.get(tog.abi.FIELD_X), h.get(tog.abi.FIELD_A), h.get(tog.abi.FIELD_B)
    for b in range(prob.B):
        o = oracle.OracleSolver(pinf, opts, b)
        o.rollout_open_loop()
        o.jacobians()
        assert rel(X[b], o.get("X")) < TOL_STEP, b
        assert rel(A[b], o.get("A")) < TOL_STEP, b
        assert rel(Bm[b], o.get("B")) < TOL_STEP, b
        assert np.array_equal(Bm[b][:, :, 4:], np.broadcast_to(np.eye(13), (20, 13, 13)))


@pytest.mark.gpu
@pytest.mark.parametrize("sqrt", [False, True])
def test_gpu_infeasible_backward_pass(tog, oracle, gpu, sqrt):
    """cost_expansion! + backwardpass! of the infeasible quadrotor under AL (slack equality rows,
    m = 17: the LDS backward kernel) vs the oracle."""
    prob = quad_line_batch(tog, B=3, N=21, seed=3)
    pinf = tog.infeasible_problem(prob, 1.0)
    il = tog.iLQRSolverOptions(square_root=sqrt)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=il)
    solver = tog.AugmentedLagrangianSolver(pinf, opts)
    h = solver.handle
    h.slack_controls()
    h.update_constraints()
    h.jacobians()
    dV = h.backward_pass(sqrt=sqrt, al=True)
    K, d = h.get(tog.abi.FIELD_K), h.get(tog.abi.FIELD_D)
    U = h.get(tog.abi.FIELD_U)
    for b in range(prob.B):
        p = pinf.copy()
        p._U[b] = U[b]
        o = oracle.OracleSolver(p, opts, b)
        o.update_constraints()
        o.jacobians()
        assert o.cost_expansion(sqrt, True) == 0
        dVo, _ = o.backward(sqrt)
        assert rel(K[b], o.get("K")) < TOL_STEP, b
        assert rel(d[b], o.get("d")) < TOL_STEP, b
        assert rel(dV[b], dVo) < TOL_STEP, b


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [False, True])
def test_gpu_reference_infeasible_pendulum(tog, oracle, gpu, variant):
    """test/infeasible_tests.jl through solve_b(prob, ALTROSolverOptions) on the device: the
    reference's thresholds, and the same X, U and iteration counts as the oracle."""
    Xend = {}
    for resolve in (False, True):
        prob = pendulum_line(tog, variant)
        opts = pendulum_opts(tog, resolve)
        ref = prob.copy()
        solver = tog.solve_b(prob, opts)
        Xo, Uo, si, sf = oracle.solve_altro_infeasible(ref, opts)
        assert rel(prob.X, Xo) < TOL_SOLVE and rel(prob.U, Uo) < TOL_SOLVE
        assert int(solver.stats["iterations_total"][0]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS])
        Xend[resolve] = prob.X[-1]
        if not variant:
            assert np.linalg.norm(prob.X[-1] - prob.xf) < 1e-3
        else:
            assert tog.max_violation(prob) < opts.opts_al.constraint_tolerance
    assert np.linalg.norm(Xend[False] - Xend[True]) < 1e-5


@pytest.mark.gpu
def test_gpu_infeasible_quadrotor_batch(tog, oracle, gpu):
    """A batch of infeasible-start quadrotor solves (resolve + projection) vs the oracle per
    trajectory: final X, U within 1e-6 and equal iteration counts in both phases."""
    prob = quad_line_batch(tog, B=3, N=31, seed=11)
    opts = tog.ALTROSolverOptions()
    ref = prob.copy()
    solver = tog.solve_b(prob, opts)
    for b in range(prob.B):
        Xo, Uo, si, sf = oracle.solve_altro_infeasible(ref, opts, b)
        assert rel(prob._X[b], Xo) < TOL_SOLVE, b
        assert rel(prob._U[b], Uo) < TOL_SOLVE, b
        assert int(solver.stats["iterations_total"][b]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS]), b
        assert int(solver.stats_feasible["iterations_total"][b]) == int(sf.get("stats")[tog.abi.STAT_TOTAL_STEPS]), b


def maze_opts(tog, resolve=False):
    """test/infeasible_tests.jl:57-76 (the reference's commented-out maze case)."""
    il = tog.iLQRSolverOptions(iterations=300)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=il, iterations=40, cost_tolerance=1e-5,
                                              cost_tolerance_intermediate=1e-4, constraint_tolerance=1e-3,
                                              penalty_scaling=10.0, penalty_initial=1.0)
    return tog.ALTROSolverOptions(resolve_feasible_problem=resolve, opts_al=al, R_inf=0.001)


def test_quadrotor_maze_problem(tog):
    """problems/quadrotor_maze.jl: 44 cylinders (+ r_quad), bnd1 at knot 1, bnd2 + maze at 2..N-1,
    bnd_xf at N; the interpolated state guess starts at x0, ends at xf and keeps q = q0."""
    p = tog.Problems.quadrotor_maze()
    nc = p.constraints.num_constraints()
    assert nc[0] == 8 and all(c == 56 for c in nc[1:-1]) and nc[-1] == 18
    assert np.allclose(p.X[0], p.x0[0]) and np.allclose(p.X[-1], p.xf)
    assert np.allclose(p.X[:, 3:7], [1, 0, 0, 0])
    pinf = tog.infeasible_problem(p, 0.001)
    nci = pinf.constraints.num_constraints()
    assert nci[0] == 8 + 13 and all(c == 56 + 13 for c in nci[1:-1]) and nci[-1] == 18


@pytest.mark.gpu
def test_gpu_quadrotor_maze_infeasible(tog, oracle, gpu):
    """The quadrotor_maze infeasible-start AL solve (69 rows per knot: the LDS backward kernel)
    on the device equals the oracle: X, U and the iteration count."""
    p = tog.Problems.quadrotor_maze()
    opts = maze_opts(tog, resolve=False)
    ref = p.copy()
    solver = tog.solve_b(p, opts)
    Xo, Uo, si, _ = oracle.solve_altro_infeasible(ref, opts)
    assert rel(p.X, Xo) < TOL_SOLVE and rel(p.U, Uo) < TOL_SOLVE
    assert int(solver.stats["iterations_total"][0]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS])
    # the reference's (commented-out) assertion, infeasible_tests.jl:69-70
    assert tog.max_violation(p) < opts.opts_al.constraint_tolerance


@pytest.mark.gpu
@pytest.mark.parametrize("sqrt", [False, True])
def test_gpu_quadrotor_maze_step_level(tog, oracle, gpu, sqrt):
    """One AL step of the maze's infeasible problem (69 rows per knot, more than a wave's lanes;
    the sqrt expansion's [Q.uu; √Iμ cu] QR is 86 x 17): constraint values, AL cost, Jacobians,
    gains and ΔV bit-identical to the oracle, then the forward pass picks the same α and J."""
    p = tog.Problems.quadrotor_maze()
    pinf = tog.infeasible_problem(p, 0.001)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(square_root=sqrt))
    h = tog.AugmentedLagrangianSolver(pinf, opts).handle
    o = oracle.OracleSolver(pinf, opts)
    h.slack_controls()
    o.slack_controls()
    h.update_constraints()
    o.update_constraints()
    assert rel(h.get(tog.abi.FIELD_C)[0], o.get("C")) == 0.0
    J0 = o.cost(True)
    assert h.cost(al=True)[0] == J0
    h.jacobians()
    o.jacobians()
    dV = h.backward_pass(sqrt=sqrt, al=True)[0]
    assert o.cost_expansion(sqrt, True) == 0
    dVo, _ = o.backward(sqrt)
    assert rel(h.get(tog.abi.FIELD_K)[0], o.get("K")) < TOL_STEP
    assert rel(h.get(tog.abi.FIELD_D)[0], o.get("d")) < TOL_STEP
    assert rel(dV, dVo) < TOL_STEP
    assert h.forward_pass(J0, al=True)[0] == o.forward(J0, True)


@pytest.mark.gpu
def test_gpu_infeasible_error_paths(tog, gpu):
    """slack_controls on a plain handle and a slack constraint in a plain problem fail loudly through
    the ABI (no silent fallback)."""
    prob, opts = tog.Problems.config_quadrotor(B=2)
    h = tog.AugmentedLagrangianSolver(prob, opts).handle
    with pytest.raises(RuntimeError, match="TOG_PROB_INFEASIBLE"):
        h.slack_controls()
    bad = prob.copy()
    bad.constraints[0] = bad.constraints[0] + tog.infeasible_constraints(13, 4)
    with pytest.raises(RuntimeError, match="TOG_CON_INFEASIBLE"):
        tog.AugmentedLagrangianSolver(bad, opts)


@pytest.mark.gpu
def test_gpu_infeasible_kuka(tog, oracle, gpu):
    """add_slack_controls on the Kuka RBD model (src/model.jl:761-779 over src/model.jl:394-447): m = 7 +
    14 slack controls (LDS backward kernel). Infeasible-start AL solves from a straight-line joint
    guess x0 -> xf, against the oracle per trajectory (final X, U within 1e-6, equal iteration counts)."""
    pk, ok = tog.Problems.config_kuka(B=2)
    N = pk.N
    t = np.linspace(0.0, 1.0, N)[None, :, None]
    pk.X = pk.x0[:, None, :] + (pk.xf - pk.x0)[:, None, :] * t
    opts = tog.ALTROSolverOptions(opts_al=ok, resolve_feasible_problem=False)
    ref = pk.copy()
    solver = tog.solve_b(pk, opts)
    for b in range(pk.B):
        Xo, Uo, si, _ = oracle.solve_altro_infeasible(ref, opts, b)
        assert rel(pk._X[b], Xo) < TOL_SOLVE, b
        assert rel(pk._U[b], Uo) < TOL_SOLVE, b
        assert int(solver.stats["iterations_total"][b]) == int(si.get("stats")[tog.abi.STAT_TOTAL_STEPS]), b


def _pn_opts(tog, resolve):
    opts = pendulum_opts(tog, resolve)
    opts.projected_newton = True
    opts.projected_newton_tolerance = 1e-2
    opts.opts_pn.n_steps = 4
    opts.opts_pn.feasibility_tolerance = 1e-8
    return opts


def test_oracle_infeasible_projected_newton(tog, oracle):
    """ALTRO phase 2 on the infeasible-start problem (altro_methods.jl:31-39 runs solve!(prob_altro,
    solver_pn) on the infeasible problem): after the AL phase stopped at projected_newton_tolerance, the
    projection drives the infeasible problem's violation (the slack rows included) below the AL phase's."""
    prob = pendulum_line(tog, True)
    opts = _pn_opts(tog, False)
    tog.solvers._altro_pn_tolerances(opts)
    pinf = tog.infeasible_problem(prob, opts.R_inf)
    si = oracle.OracleSolver(pinf, opts)
    si.slack_controls()
    si.solve()
    c_al = si.max_violation()
    st = si.solve_pn(opts.opts_pn)
    assert st[tog.abi.PN_STEPS] >= 1
    assert si.max_violation() < c_al


@pytest.mark.gpu
@pytest.mark.parametrize("resolve", [False, True])
def test_gpu_infeasible_projected_newton(tog, oracle, gpu, resolve):
    """solve_b(prob, ALTROSolverOptions(projected_newton=true)) from an initial state trajectory: the
    device's AL phase, projected Newton on Infeasible<Pendulum> (k_pn_*), process_results! and the resolve
    against the oracle's same flow: X, U to the projected Newton tolerance of test_projected_newton.py
    (1e-13) without the resolve, 1e-6 with it."""
    prob = pendulum_line(tog, True)
    opts = _pn_opts(tog, resolve)
    ref = prob.copy()
    solver = tog.solve_b(prob, opts)
    assert solver.stats["time_pn"] > 0.0
    Xo, Uo, si, sf = oracle.solve_altro_infeasible(ref, opts)
    tol = TOL_SOLVE if resolve else TOL_STEP
    assert rel(prob.X, Xo) < tol and rel(prob.U, Uo) < tol
    assert int(solver.stats_pn["iterations"][0]) >= 1


def _pendulum_line_bound(tog, trim):
    """pendulum_line's constrained variant with a finite state bound as well, trimmed or not."""
    prob = tog.Problems.pendulum()
    n, m, N = 2, 1, prob.N
    bnd = tog.BoundConstraint(n, m, x_min=[-20.0, -20.0], x_max=[20.0, 20.0], u_min=-3.0, u_max=3.0, trim=trim)
    cons = tog.Constraints([bnd], N)
    cons[N - 1] = cons[N - 1] + tog.goal_constraint(prob.xf)
    prob = tog.Problem(prob.model, prob.obj, prob.U, constraints=cons, x0=prob.x0[0], xf=prob.xf, N=N, dt=prob.dt)
    prob.X = tog.line_trajectory(prob.x0[0], prob.xf, prob.N)
    return prob


def test_oracle_infeasible_untrimmed_bound(tog, oracle):
    """BoundConstraint(trim=false) on an infeasible-start problem (built since round 6): the bound keeps the
    model's m (update_constraint_set_jacobians, constraint_sets.jl:135-150), so with every entry finite the
    untrimmed solve equals the trimmed one bit for bit."""
    opts = pendulum_opts(tog, False)
    out = []
    for trim in (True, False):
        prob = _pendulum_line_bound(tog, trim)
        pinf = tog.infeasible_problem(prob, opts.R_inf)
        assert pinf.constraints[0][0].to_abi(pinf.model.m)[1] == (0 if trim else 1)
        X, U, si, _ = oracle.solve_altro_infeasible(prob, opts, 0)
        out.append((X, U, si.history()[1]))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2], out[1][2])


@pytest.mark.gpu
def test_gpu_infeasible_untrimmed_bound(tog, oracle, gpu):
    """The untrimmed infeasible-start case on the device equals the oracle (X, U to 1e-6, AL records)."""
    opts = pendulum_opts(tog, True)
    prob = _pendulum_line_bound(tog, False)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    X, U, si, sf = oracle.solve_altro_infeasible(prob, opts, 0)
    assert rel(gp._X[0], X) < TOL_SOLVE and rel(gp._U[0], U) < TOL_SOLVE
    assert solver.solver_al.traj_stats(0)["iterations"] == len(si.history()[1])
