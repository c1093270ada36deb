"""The square-root backward pass's PosDefException (backward_pass.jl:186-192: chol_minus ->
lowrankdowndate!, which throws when a downdate leaves the factor indefinite).

In the reference the exception ends the solve. Here the trajectory stops where the exception would be
thrown (TRAJ_SQRT_PD_FAIL | TRAJ_BP_ABORTED, no forward pass, its X and U as they were), the rest of
the batch finishes, and solve_b then raises PosDefException (a numpy LinAlgError). The cases: a cost
with a cross term H large enough that the Schur complement R - H Q⁻¹ H' of the stage Hessian is
indefinite — at the first backward pass (h = 2) or after one accepted iteration (quadrotor, h = 1.1);
h = 1 converges. The device (every backward kernel: the bulk team kernel, and the tail's quad, trio, duo
and one-wave team kernels) must stop at the same step as the oracle with the same X, U and flags."""
import os

import numpy as np
import pytest

def _di_problem(tog, hval, N=21):
    n, m = 2, 1
    H = np.array([[hval, hval]])
    obj = tog.Objective(tog.QuadraticCost(np.eye(n), np.eye(m), H=H), tog.LQRCostTerminal(10 * np.eye(n), np.zeros(n)),
                        N=N)
    return tog.Problem(tog.rk3(tog.Dynamics.doubleintegrator), obj, np.zeros((N - 1, m)), x0=np.array([1.0, 0.0]),
                       N=N, dt=0.1)


def _quad_problem(tog, hval, B=None, N=31):
    n, m = 13, 4
    H = np.zeros((m, n))
    H[:, 7:11] = hval * np.eye(4)
    x0 = np.zeros(n)
    x0[3] = 1.0
    xf = x0.copy()
    xf[0] = 1.0
    obj = tog.Objective(tog.QuadraticCost(np.eye(n), np.eye(m), H=H), tog.LQRCostTerminal(10 * np.eye(n), xf), N=N)
    U0 = np.full((N - 1, m), 0.5 * 9.81 / 4 * 0.5)
    if B is not None:  # a batch: x0[1:3] jittered per trajectory
        rng = np.random.default_rng(11)
        x0 = np.tile(x0, (B, 1))
        x0[:, :3] += 0.05 * rng.standard_normal((B, 3))
        U0 = np.tile(U0, (B, 1, 1))
    return tog.Problem(tog.rk3(tog.Dynamics.quadrotor), obj, U0, x0=x0, N=N, dt=0.05)


def _flags(S, abi):
    return int(S[abi.STAT_FLAGS])


@pytest.mark.parametrize("hval,fail,steps", [(0.5, False, 2), (2.0, True, 0)])
def test_oracle_downdate_failure_stops_the_solve(tog, oracle, hval, fail, steps):
    abi = tog.abi
    prob = _di_problem(tog, hval)
    o = oracle.OracleSolver(prob, tog.iLQRSolverOptions(square_root=True, iterations=50))
    assert o.solve() == steps
    f = _flags(o.get("stats"), abi)
    want = abi.TRAJ_SQRT_PD_FAIL | abi.TRAJ_BP_ABORTED
    assert (f & want == want) if fail else (f & want == 0)


def test_posdef_exception_is_a_linalg_error(tog):
    e = tog.PosDefException([3, 5])
    assert isinstance(e, np.linalg.LinAlgError) and e.trajectories == [3, 5]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [None, "trio", "duo", "team"])
@pytest.mark.parametrize("model,hval", [("di", 2.0), ("quad", 1.1), ("quad", 2.0)])
def test_device_stops_like_the_oracle(tog, gpu, oracle, kind, model, hval):
    abi = tog.abi
    old = os.environ.get("TOG_BWD_TAIL")
    if kind:
        os.environ["TOG_BWD_TAIL"] = kind
    try:
        prob = _di_problem(tog, hval) if model == "di" else _quad_problem(tog, hval)
        opts = tog.iLQRSolverOptions(square_root=True, iterations=50)
        ref = oracle.OracleSolver(prob, opts)
        steps = ref.solve()
        dev = prob.copy()
        with pytest.raises(tog.PosDefException) as ei:
            tog.solve_b(dev, opts)
    finally:
        if old is None:
            os.environ.pop("TOG_BWD_TAIL", None)
        else:
            os.environ["TOG_BWD_TAIL"] = old
    assert ei.value.trajectories == [0]
    assert steps == (1 if hval == 1.1 else 0)
    assert np.array_equal(dev.X, ref.get("X"))
    assert np.array_equal(dev.U, ref.get("U"))


@pytest.mark.gpu
def test_bulk_team_kernel_stops_like_the_oracle(tog, gpu, oracle):
    """B = 4096 > the tail threshold: the first steps run the bulk team kernel."""
    abi = tog.abi
    prob = _quad_problem(tog, 1.1, B=4096)
    opts = tog.iLQRSolverOptions(square_root=True, iterations=50)
    dev = prob.copy()
    with pytest.raises(tog.PosDefException) as ei:
        tog.solve_b(dev, opts)
    bad = ei.value.trajectories
    assert len(bad) > 0
    for b in sorted({0, bad[0], bad[-1]}):
        ref = oracle.OracleSolver(prob, opts, b=b)
        ref.solve()
        assert bool(_flags(ref.get("stats"), abi) & abi.TRAJ_SQRT_PD_FAIL) == (b in bad)
        assert np.array_equal(dev._X[b], ref.get("X"))
        assert np.array_equal(dev._U[b], ref.get("U"))
