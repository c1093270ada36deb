"""Step-level Python API (the reference's exported step functions, src/TrajectoryOptimization.jl:
82-95) and the backward pass's failure paths.

* ``test/sqrt_bp_tests.jl:27-37,58-85`` mirrored call for call through the Python API:
  ``rollout_b`` → (AL: ``update_constraints_b``) → ``jacobian_b`` → ``cost_expansion_b`` →
  ``backwardpass_b``. The device expansion (``solver.Q``) and the gains equal the oracle's bitwise,
  and std ≡ sqrt within the reference's isapprox tolerance.
* The regularisation-restart cap (``TOG_BP_MAX_RESTARTS``, include/tog.h): a trajectory whose
  expansion is NaN can never pass ``isposdef`` (backward_pass.jl:52-62; the reference loops
  forever). Oracle and device both stop it after the same number of restarts with
  ``MAX_REG | BP_ABORTED``, without disturbing the other trajectories of the batch.
* NaN constraint values propagate into ``max_violation`` as Julia's ``max`` does
  (augmented_lagrangian_methods.jl:171-184), on the oracle and on the device.
"""
import numpy as np
import pytest

RTOL = np.sqrt(np.finfo(float).eps)  # Julia isapprox default


def isapprox(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.linalg.norm(a - b) <= RTOL * max(np.linalg.norm(a), np.linalg.norm(b))


def _opts(tog, sqrt, constrained):
    il = tog.iLQRSolverOptions(square_root=sqrt)
    return tog.AugmentedLagrangianSolverOptions(opts_uncon=il) if constrained else il


def _device_steps(tog, prob, sqrt, constrained):
    """sqrt_bp_tests.jl call sequence on the device, through the Python mirror."""
    p = prob.copy()
    tog.rollout_b(p)  # rollout!(prob)
    solver = tog.AbstractSolverFor(p, _opts(tog, sqrt, constrained))
    if constrained:
        tog.update_constraints_b(p, solver)  # update_constraints! + update_active_set!
    tog.jacobian_b(p, solver)
    Q = tog.cost_expansion_b(p, solver)
    dV = tog.backwardpass_b(p, solver, square_root=sqrt)
    h = solver.handle
    S = h.get(tog.abi.FIELD_S)[0]
    if sqrt:
        S = np.einsum("kji,kjl->kil", S, S)  # S.xx = Ssqrt' Ssqrt
    return dict(Q=Q, Qflat=h.get(tog.abi.FIELD_Q)[0], dV=dV, K=solver.K[0], d=solver.d[0], S=S,
                Sx=h.get(tog.abi.FIELD_SX)[0])


def _oracle_steps(oracle, tog, prob, sqrt, constrained):
    s = oracle.OracleSolver(prob, _opts(tog, sqrt, constrained))
    s.rollout_open_loop()
    if constrained:
        s.update_constraints()
    s.jacobians()
    assert s.cost_expansion(sqrt=sqrt, al=constrained) == 0
    Q = s.get("Q")
    dV, _ = s.backward(sqrt=sqrt)
    return dict(Qflat=Q, dV=dV, K=s.get("K"), d=s.get("d"))


@pytest.mark.gpu
@pytest.mark.parametrize("constrained", [False, True])
def test_sqrt_bp_step_by_step_python_api(tog, oracle, gpu, constrained):
    prob = tog.Problems.car_sqrt_bp(constrained=constrained)
    std = _device_steps(tog, prob, False, constrained)
    sq = _device_steps(tog, prob, True, constrained)
    for sqrt, dev in ((False, std), (True, sq)):
        ref = _oracle_steps(oracle, tog, prob, sqrt, constrained)
        assert np.array_equal(dev["Qflat"], ref["Qflat"])  # cost_expansion! itself
        assert np.array_equal(dev["dV"], ref["dV"])
        assert np.array_equal(dev["K"], ref["K"]) and np.array_equal(dev["d"], ref["d"])
    # solver.Q is the reference's Expansion: sqrt factors reproduce the std expansion (:38-44)
    n, m = prob.model.n, prob.model.m
    assert std["Q"].xx.shape == (1, prob.N, n, n) and std["Q"].ux.shape == (1, prob.N, m, n)
    UtU = np.einsum("...ki,...kj->...ij", sq["Q"].xx, sq["Q"].xx)
    assert np.allclose(UtU, std["Q"].xx, rtol=RTOL, atol=1e-12)
    assert np.array_equal(sq["Q"].x, std["Q"].x) and np.array_equal(sq["Q"].u, std["Q"].u)
    # the reference's assertions (sqrt_bp_tests.jl:39-44 / 79-85)
    assert isapprox(sq["dV"], std["dV"])
    assert isapprox(sq["K"], std["K"]) and isapprox(sq["d"], std["d"])
    for k in range(prob.N):
        assert isapprox(sq["S"][k], std["S"][k]), k
        assert isapprox(sq["Sx"][k], std["Sx"][k]), k


def _nan_batch(tog, B=3, bad=1):
    prob, opts = tog.Problems.config_quadrotor(B=B)
    opts.opts_uncon.square_root = False  # isposdef path (backward_pass.jl:52-62)
    prob.x0[bad, 3] = np.nan  # quaternion: A, B and so Q.uu are NaN
    return prob, opts


def test_oracle_restart_cap_stops_nan_trajectory(tog, oracle):
    prob, opts = _nan_batch(tog)
    s = oracle.OracleSolver(prob, opts, b=1)
    s.solve()
    st = s.get("stats")
    flags = int(st[tog.abi.STAT_FLAGS])
    assert flags & tog.abi.TRAJ_BP_ABORTED and flags & tog.abi.TRAJ_MAX_REG
    assert int(st[tog.abi.STAT_BP_RESTARTS]) == tog.abi.BP_MAX_RESTARTS + 1
    assert int(st[tog.abi.STAT_TOTAL_STEPS]) == 0
    assert np.isnan(s.max_violation())  # NaN constraint values propagate (Julia max)


def test_oracle_max_violation_nan_propagates(tog, oracle):
    prob, opts = tog.Problems.config_quadrotor(B=1)
    s = oracle.OracleSolver(prob, opts)
    s.rollout_open_loop()
    s.update_constraints()
    assert np.isfinite(s.max_violation())
    prob.x0[0, 5] = np.nan
    s = oracle.OracleSolver(prob, opts)
    s.rollout_open_loop()
    s.update_constraints()
    assert np.isnan(s.max_violation())


@pytest.mark.gpu
def test_device_restart_cap_matches_oracle(tog, oracle, gpu):
    prob, opts = _nan_batch(tog, B=3, bad=1)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    flags = solver.stats["flags"]
    assert flags[1] & tog.abi.TRAJ_BP_ABORTED and flags[1] & tog.abi.TRAJ_MAX_REG
    assert not flags[1] & tog.abi.TRAJ_ACTIVE
    for b in (0, 2):  # the healthy trajectories are untouched, bit for bit
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert not flags[b] & tog.abi.TRAJ_BP_ABORTED
        assert np.array_equal(gp._X[b], o.get("X")) and np.array_equal(gp._U[b], o.get("U"))
        assert steps == solver.stats["iterations_total"][b]
    assert solver.stats["iterations_total"][1] == 0
    assert np.isnan(solver.stats["c_max"][1])
    assert np.isnan(solver.handle.batch_stats()[2])  # the batch max violation propagates NaN too


def test_as_dp_rejects_wrong_dtype(tog):
    with pytest.raises(TypeError):
        tog.abi.as_dp(np.zeros(4, dtype=np.float32))
    with pytest.raises(TypeError):
        tog.abi.as_dp(np.zeros((4, 4))[:, ::2])
    tog.abi.as_dp(np.zeros((3, 2), order="F"))
