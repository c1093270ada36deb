"""GPU parity: libtog.so (HIP, gfx950) vs the CPU oracle on identical inputs.

Bar (north star): fp64 states / controls / gains within 1e-6 relative of the CPU solve. Under the
arithmetic contract the kernels are bit-identical to the oracle, so step-level
results are held to 1e-13 and solves must also take the same number of iterations. Every call goes
through the C ABI (include/tog.h).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_SOLVE = 1e-6  # north-star bar; the arithmetic contract makes GPU == oracle bitwise
TOL_STEP = 1e-13


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def lqr_problem(tog, model, integ, N=21, dt=0.05, B=4, seed=0, constraints=None):
    rng = np.random.default_rng(seed)
    n, m = model.n, model.m
    md = tog.discretize_model(model, integ)
    xf = rng.standard_normal(n)
    if model.name == "quadrotor":
        xf[3:7] = [1, 0, 0, 0]
    obj = tog.LQRObjective(0.1 * np.eye(n), 0.05 * np.eye(m), 10.0 * np.eye(n), xf, N)
    x0 = 0.3 * rng.standard_normal((B, n))
    U0 = 0.2 * rng.standard_normal((B, N - 1, m))
    if model.name == "quadrotor":
        x0[:, 3:7] = [1, 0, 0, 0]
        U0 += 0.5 * 9.81 / 4
    return tog.Problem(md, obj, U0, x0=x0, N=N, dt=dt, constraints=constraints)


MODELS = [("doubleintegrator", "rk3"), ("cartpole", "rk3"), ("quadrotor", "rk4"), ("quadrotor", "rk3"),
          ("car", "rk4"), ("pendulum", "rk3"), ("quadrotor", "midpoint"), ("cartpole", "midpoint")]
INTEG = {"rk3": 0, "rk4": 1, "midpoint": 2}


@pytest.mark.parametrize("name,integ", MODELS)
def test_jacobian_parity(tog, oracle, gpu, name, integ):
    """jacobian!(prob, solver) (src/model.jl:301-306) vs the oracle's ForwardDiff restatement."""
    model = getattr(tog.Dynamics, name)
    prob = lqr_problem(tog, model, integ, N=11, B=5, seed=1)
    rng = np.random.default_rng(2)
    prob._X[...] = 0.5 * rng.standard_normal(prob._X.shape)
    if name == "quadrotor":
        prob._X[..., 3:7] += np.array([1.0, 0, 0, 0])
    solver = tog.iLQRSolver(prob, tog.iLQRSolverOptions())
    tog.jacobian_b(prob, solver)
    A = solver.handle.get(tog.abi.FIELD_A)
    Bm = solver.handle.get(tog.abi.FIELD_B)
    ig = INTEG[integ]
    for b in range(prob.B):
        for k in range(prob.N - 1):
            S = oracle.discrete_jacobian(model.model_id, ig, prob._X[b, k], prob._U[b, k], prob.dt)
            n = model.n
            assert rel(A[b, k], S[:, :n]) < TOL_STEP, (b, k)
            assert rel(Bm[b, k], S[:, n:n + model.m]) < TOL_STEP, (b, k)


def _oracle_bp(oracle, prob, opts, b, sqrt, al):
    o = oracle.OracleSolver(prob, opts, b=b)
    o.rollout_open_loop()
    if al:
        o.update_constraints()
    o.jacobians()
    assert o.cost_expansion(sqrt, al) == 0
    dV, restarts = o.backward(sqrt)
    return o, dV


@pytest.mark.parametrize("sqrt", [False, True])
@pytest.mark.parametrize("al", [False, True])
@pytest.mark.parametrize("which", ["car", "quadrotor"])
def test_backward_pass_parity(tog, oracle, gpu, sqrt, al, which):
    """cost_expansion! + backwardpass! (std and sqrt, plain and AL objective): K, d, ΔV, S, s."""
    if which == "car":
        prob = tog.Problems.car_sqrt_bp(constrained=al)
        B = 1
    else:
        prob, _ = tog.Problems.config_quadrotor(B=3)
        if not al:
            prob.constraints = tog.Constraints(prob.N)
        B = prob.B
    il = tog.iLQRSolverOptions(square_root=sqrt)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=il) if al else il
    solver = tog.AbstractSolverFor(prob, opts)
    h = solver.handle
    h.rollout_open_loop()
    h.jacobians()
    dV = h.backward_pass(sqrt=sqrt, al=al, store_S=True)
    K, d = h.get(tog.abi.FIELD_K), h.get(tog.abi.FIELD_D)
    S, Sx = h.get(tog.abi.FIELD_S), h.get(tog.abi.FIELD_SX)
    for b in range(B):
        o, dV_ref = _oracle_bp(oracle, prob, opts, b, sqrt, al)
        assert rel(dV[b], dV_ref) < TOL_STEP
        assert rel(K[b], o.get("K")) < TOL_STEP
        assert rel(d[b], o.get("d")) < TOL_STEP
        Sref = o.get("S")
        for k in range(prob.N):
            if sqrt:  # compare S'S (A.8: R factors are unique up to row signs)
                assert rel(S[b, k].T @ S[b, k], Sref[k].T @ Sref[k]) < TOL_STEP, k
            else:
                assert rel(S[b, k], Sref[k]) < TOL_STEP, k
        assert rel(Sx[b], o.get("Sx")) < TOL_STEP


@pytest.mark.parametrize("constrained", [False, True])
def test_std_sqrt_equivalence_on_gpu(tog, gpu, constrained):
    """test/sqrt_bp_tests.jl:17-44 and :46-85 run on the GPU kernels."""
    prob = tog.Problems.car_sqrt_bp(constrained=constrained)
    res = {}
    for sq in (False, True):
        il = tog.iLQRSolverOptions(square_root=sq)
        opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=il) if constrained else il
        s = tog.AbstractSolverFor(prob, opts)
        s.handle.rollout_open_loop()
        s.handle.jacobians()
        dV = s.handle.backward_pass(sqrt=sq, al=constrained, store_S=True)
        res[sq] = (dV[0], s.K[0], s.d[0], s.handle.get(tog.abi.FIELD_S)[0], s.handle.get(tog.abi.FIELD_SX)[0])
    (dV, K, d, S, Sx), (dV2, K2, d2, S2, Sx2) = res[False], res[True]
    assert np.allclose(dV, dV2, rtol=1.5e-8)
    assert np.allclose(K, K2, rtol=1.5e-8, atol=1e-12)
    assert np.allclose(d, d2, rtol=1.5e-8, atol=1e-12)
    for k in range(prob.N):
        assert np.allclose(S[k], S2[k].T @ S2[k], rtol=1.5e-8, atol=1e-10)
        assert np.allclose(Sx[k], Sx2[k], rtol=1.5e-8, atol=1e-10)


@pytest.mark.parametrize("al", [False, True])
def test_forward_pass_parity(tog, oracle, gpu, al):
    """forwardpass! (forward_pass.jl:5-85) from identical gains: J, X̄, Ū, α."""
    prob, opts_al = tog.Problems.config_quadrotor(B=3)
    opts = opts_al if al else opts_al.opts_uncon
    solver = tog.AbstractSolverFor(prob, opts)
    h = solver.handle
    h.rollout_open_loop()
    h.jacobians()
    dV = h.backward_pass(sqrt=True, al=al)
    J0 = h.cost(al=al)
    J = h.forward_pass(J0, al=al)
    Xb, Ub = h.get(tog.abi.FIELD_XBAR), h.get(tog.abi.FIELD_UBAR)
    for b in range(prob.B):
        o, dV_ref = _oracle_bp(oracle, prob, opts, b, True, al)
        Jref0 = o.cost(al)
        assert rel(J0[b], Jref0) < TOL_STEP
        Jref = o.forward(Jref0, al)
        assert rel(J[b], Jref) < TOL_STEP
        assert rel(Xb[b], o.get("Xbar")) < TOL_STEP
        assert rel(Ub[b], o.get("Ubar")) < TOL_STEP


def test_rollout_alpha_and_divergence(tog, oracle, gpu):
    """rollout!(prob, solver, α) incl. the divergence check (src/rollout.jl:18-20)."""
    prob = lqr_problem(tog, tog.Dynamics.cartpole, "rk3", N=31, B=4, seed=5)
    solver = tog.iLQRSolver(prob, tog.iLQRSolverOptions())
    h = solver.handle
    h.rollout_open_loop()
    rng = np.random.default_rng(0)
    K = rng.standard_normal(h.shape(tog.abi.FIELD_K))
    K[0] *= 1e9  # trajectory 0 must diverge
    d = rng.standard_normal(h.shape(tog.abi.FIELD_D))
    h.set(tog.abi.FIELD_K, np.swapaxes(K, -1, -2))
    h.set(tog.abi.FIELD_D, d)
    X = h.get(tog.abi.FIELD_X)
    X[:, 1:, :] += 0.01  # make δx non-zero
    h.set(tog.abi.FIELD_X, X)
    ok = h.rollout(0.5)
    Xb = h.get(tog.abi.FIELD_XBAR)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, tog.iLQRSolverOptions(), b=b)
        o.set("X", X[b])
        o.set("K", np.swapaxes(K[b], -1, -2))
        o.set("d", d[b])
        ok_ref = o.rollout(0.5)
        assert ok[b] == ok_ref
        if ok_ref:
            assert rel(Xb[b], o.get("Xbar")) < TOL_STEP
    assert not ok[0]


def _solve_and_compare(tog, oracle, prob, opts, tol=TOL_SOLVE):
    gpu_prob = prob.copy()
    solver = tog.solve_b(gpu_prob, opts)
    st = solver.stats
    out = []
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        X, U = o.get("X"), o.get("U")
        eX, eU = rel(gpu_prob._X[b], X), rel(gpu_prob._U[b], U)
        out.append((eX, eU, steps, int(st["iterations_total"][b])))
        assert eX < tol and eU < tol, (b, eX, eU, steps, st["iterations_total"][b])
        assert steps == st["iterations_total"][b]
    return solver, out


def test_solve_cartpole_ilqr(tog, oracle, gpu):
    """Config 2 shape (cartpole swing-up, unconstrained iLQR), small batch."""
    prob, opts = tog.Problems.config_cartpole(B=6)
    _solve_and_compare(tog, oracle, prob, opts)


def test_solve_quadrotor_al_sqrt(tog, oracle, gpu):
    """Config 3 shape (quadrotor AL-iLQR, u in [0,15] + goal, sqrt BP), small batch."""
    prob, opts = tog.Problems.config_quadrotor(B=4)
    solver, _ = _solve_and_compare(tog, oracle, prob, opts)
    assert np.all(solver.stats["c_max"] < opts.constraint_tolerance)


def test_solve_double_integrator_altro(tog, oracle, gpu):
    """Config 1 (double integrator block move, ALTRO defaults = AL phase)."""
    prob, opts = tog.Problems.config_doubleintegrator()
    _solve_and_compare(tog, oracle, prob, opts)
    assert tog.max_violation(prob) >= 0.0


@pytest.mark.parametrize("cons,sq", [("none", False), ("goal", False), ("goal+bounds", True)])
def test_solve_quadrotor_tests(tog, oracle, gpu, cons, sq):
    """test/quadrotor_tests.jl:38-66 problems; plus the reference's own thresholds."""
    prob = tog.Problems.quadrotor_test(cons)
    il = tog.iLQRSolverOptions(cost_tolerance=1e-5, square_root=sq)
    opts = il if cons == "none" else tog.AugmentedLagrangianSolverOptions(
        opts_uncon=il, constraint_tolerance=1e-3, cost_tolerance=1e-5, cost_tolerance_intermediate=1e-4)
    _solve_and_compare(tog, oracle, prob, opts)
    xf = prob.xf
    gp = prob.copy()
    tog.solve_b(gp, opts)
    if cons == "none":
        assert np.linalg.norm(gp.X[-1] - xf) < 5e-3
    else:
        assert np.linalg.norm(gp.X[-1] - xf, np.inf) < 1e-3
        assert tog.max_violation(gp) < 1e-3


def test_solve_quad_obs(tog, oracle, gpu):
    """Config 4 constraint set (bounds + cylinders + spheres, N=101) on two starts."""
    prob, opts = tog.Problems.config_quad_maze(B=2, N=101)
    _solve_and_compare(tog, oracle, prob, opts)


def test_batch_stats_and_status(tog, gpu):
    prob, opts = tog.Problems.config_cartpole(B=16)
    solver = tog.iLQRSolver(prob, opts)
    h = solver.handle
    h.solve_init(tog.abi.MODE_ILQR)
    h.solve_step(3)
    st = h.batch_stats()
    assert st[0] == 16
    assert h.total_steps() == 48
    flags = h.status()
    assert np.all(flags & tog.abi.TRAJ_ACTIVE)


@pytest.mark.parametrize("integ", ["midpoint", "rk3"])
def test_solve_pendulum_altro(tog, oracle, gpu, integ):
    """pendulum_tests.jl:23-27 over the explicit schemes: the device AL solve equals the oracle's
    and meets the reference's max_violation < constraint_tolerance."""
    ilqr = tog.iLQRSolverOptions()
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr, iterations=50, penalty_scaling=10.0)
    opts = tog.ALTROSolverOptions(opts_al=al)
    prob = tog.Problems.pendulum(integ)
    _solve_and_compare(tog, oracle, prob, opts)
    gp = prob.copy()
    tog.solve_b(gp, opts)
    assert tog.max_violation(gp) < al.constraint_tolerance


@pytest.mark.gpu
def test_batch_stats_begin_end(tog, gpu):
    """tog_batch_stats_begin / _end (the pipelined stopping check) return what the blocking
    tog_batch_stats returns at the same point of the stream; one check may be outstanding."""
    prob, opts = tog.Problems.config_quadrotor(B=16)
    h = tog.AbstractSolverFor(prob, opts).handle
    h.solve_init(tog.abi.MODE_AL)
    h.solve_step(3)
    h.batch_stats_begin()
    with pytest.raises(RuntimeError):
        h.batch_stats_begin()
    a = h.batch_stats_end()
    with pytest.raises(RuntimeError):
        h.batch_stats_end()
    b = h.batch_stats()
    assert np.array_equal(a, b)
    h.batch_stats_begin()
    h.solve_step(2)  # enqueued behind the check: the check sees the state after 3 steps
    c = h.batch_stats_end()
    assert np.array_equal(c, a)
