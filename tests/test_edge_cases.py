"""Edge cases of the device path against the oracle: the smallest horizon (N = 2, one stage knot),
a single trajectory, a batch that does not fill the last wave's teams, and a horizon above the team
kernel's knot cap (N > TEAM_MAX_KNOTS = 1024 routes the backward pass to the LDS kernel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_SOLVE = 1e-6
TOL_STEP = 1e-13


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def _solve_vs_oracle(tog, oracle, prob, opts):
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert rel(gp._X[b], o.get("X")) < TOL_SOLVE, b
        assert rel(gp._U[b], o.get("U")) < TOL_SOLVE, b
        assert steps == solver.stats["iterations_total"][b], b
    return gp, solver


def _quad(tog, N, B, seed):
    rng = np.random.default_rng(seed)
    p0 = tog.Problems.quadrotor_test("goal+bounds")
    n, m = 13, 4
    x0 = np.tile(p0.x0[0], (B, 1))
    x0[:, :3] += 0.3 * rng.standard_normal((B, 3))
    xf = p0.xf.copy()
    xf[:3] = [0.0, 2.0, 0.0]
    cons = tog.Constraints(N)
    bnd = tog.BoundConstraint(n, m, u_min=0.0, u_max=15.0)
    for k in range(N - 1):
        cons[k] += bnd
    cons[N - 1] += tog.goal_constraint(xf)
    obj = tog.LQRObjective(p0.obj.stage.Q, p0.obj.stage.R, p0.obj.terminal.Q, xf, N)
    U0 = 0.5 * 9.81 / 4 + 0.1 * rng.standard_normal((B, N - 1, m))
    return tog.Problem(p0.model, obj, U0, x0=x0, xf=xf, N=N, dt=0.05, constraints=cons)


@pytest.mark.parametrize("sqrt", [False, True])
def test_two_knot_horizon(tog, oracle, gpu, sqrt):
    """N = 2: one stage knot, the terminal goal, AL; std and sqrt backward passes."""
    prob = _quad(tog, N=2, B=3, seed=1)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(square_root=sqrt))
    _solve_vs_oracle(tog, oracle, prob, opts)


def test_single_trajectory_and_ragged_batch(tog, oracle, gpu):
    """B = 1 and B = 5 (the last wave's four-trajectory teams half empty) give the oracle's solves."""
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(square_root=True))
    _solve_vs_oracle(tog, oracle, _quad(tog, N=21, B=1, seed=2), opts)
    _solve_vs_oracle(tog, oracle, _quad(tog, N=21, B=5, seed=3), opts)


def test_long_horizon_lds_backward(tog, oracle, gpu):
    """N = 1100 > TEAM_MAX_KNOTS: one backward pass on the LDS kernel equals the oracle's (K, d, ΔV)."""
    prob, opts = tog.Problems.config_cartpole(B=2)
    N = 1100
    obj = tog.LQRObjective(1e-2 * np.eye(4), 1e-1 * np.eye(1), 100.0 * np.eye(4), prob.xf, N)
    U0 = 0.01 + 0.5 * np.random.default_rng(4).standard_normal((2, N - 1, 1))
    p = tog.Problem(prob.model, obj, U0, x0=np.zeros((2, 4)), xf=prob.xf, N=N, dt=0.005)
    s = tog.iLQRSolver(p, tog.iLQRSolverOptions())
    h = s.handle
    h.rollout_open_loop()
    h.jacobians()
    dV = h.backward_pass(sqrt=False, al=False)
    K, d = h.get(tog.abi.FIELD_K), h.get(tog.abi.FIELD_D)
    for b in range(2):
        o = oracle.OracleSolver(p, tog.iLQRSolverOptions(), b=b)
        o.rollout_open_loop()
        o.jacobians()
        assert o.cost_expansion(False, False) == 0
        dVo, _ = o.backward(False)
        assert rel(K[b], o.get("K")) < TOL_STEP and rel(d[b], o.get("d")) < TOL_STEP
        assert rel(dV[b], dVo) < TOL_STEP
