"""BASELINE config 4 at its own horizon: quad_obs (problems/quad_obs.jl:1-88; bounds, 4 cylinders and
3 "spheres" with the radius quirk A.6), N=201, dt=0.025, 19 stage rows per knot.

* Oracle ≡ committed golden (tests/golden/quad_maze_n201.npz, made by make_golden.py) — CPU.
* Device ≡ golden bit for bit on the same 4 seeded starts: X, U, iteration counts, flags — GPU.
* Step level at N=201: K, d, ΔV, S, s of one backward pass (std and sqrt, AL) at 1e-13 — GPU.
* Full size (one GPU's shard, B=8192): finite results, converged trajectories within the
  constraint tolerance, consistent status flags, the first 4 trajectories equal to the golden — GPU.
"""
import pathlib

import numpy as np
import pytest

GOLD = pathlib.Path(__file__).resolve().parent / "golden" / "quad_maze_n201.npz"
TOL_STEP = 1e-13


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b))))


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_golden_inputs_are_the_config(tog, gold):
    prob, _ = tog.Problems.config_quad_maze(B=4, N=201)
    assert np.array_equal(prob.x0, gold["x0"]) and np.array_equal(prob._U, gold["U0"])
    st = gold["stats"]
    conv = (st[:, tog.abi.STAT_FLAGS].astype(int) & tog.abi.TRAJ_AL_CONVERGED) != 0
    assert conv.sum() == 2  # two starts converge, two exhaust the AL iterations
    assert np.all(st[conv, tog.abi.STAT_C_MAX] < 1e-3)


def test_oracle_matches_golden(tog, oracle, gold):
    """One converging start (the cheapest, ~25 s): the oracle reproduces its committed solve."""
    prob, opts = tog.Problems.config_quad_maze(B=4, N=201)
    b = 3
    s = oracle.OracleSolver(prob, opts, b)
    steps = s.solve()
    assert steps == int(gold["stats"][b, tog.abi.STAT_TOTAL_STEPS])
    assert np.array_equal(s.get("X"), gold["X"][b]) and np.array_equal(s.get("U"), gold["U"][b])


@pytest.mark.gpu
def test_device_solve_matches_golden(tog, gpu, gold):
    prob, opts = tog.Problems.config_quad_maze(B=4, N=201)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    st = solver.stats
    g = gold["stats"]
    for b in range(4):
        assert np.array_equal(gp._X[b], gold["X"][b]), b
        assert np.array_equal(gp._U[b], gold["U"][b]), b
        assert st["iterations_total"][b] == int(g[b, tog.abi.STAT_TOTAL_STEPS]), b
        assert st["flags"][b] & ~tog.abi.TRAJ_ACTIVE == int(g[b, tog.abi.STAT_FLAGS]), b
        assert st["c_max"][b] == g[b, tog.abi.STAT_C_MAX], b


@pytest.mark.gpu
@pytest.mark.parametrize("sqrt", [False, True])
def test_step_level_backward_at_n201(tog, oracle, gpu, sqrt):
    prob, _ = tog.Problems.config_quad_maze(B=2, N=201)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(square_root=sqrt))
    solver = tog.AbstractSolverFor(prob, opts)
    h = solver.handle
    h.rollout_open_loop()
    h.update_constraints()
    h.jacobians()
    dV = h.backward_pass(sqrt=sqrt, al=True, store_S=True)
    K, d = h.get(tog.abi.FIELD_K), h.get(tog.abi.FIELD_D)
    S, Sx = h.get(tog.abi.FIELD_S), h.get(tog.abi.FIELD_SX)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        o.rollout_open_loop()
        o.update_constraints()
        o.jacobians()
        assert o.cost_expansion(sqrt, True) == 0
        dV_ref, _ = o.backward(sqrt)
        assert rel(dV[b], dV_ref) < TOL_STEP
        assert rel(K[b], o.get("K")) < TOL_STEP and rel(d[b], o.get("d")) < TOL_STEP
        Sref = o.get("S")
        for k in range(prob.N):
            if sqrt:
                assert rel(S[b, k].T @ S[b, k], Sref[k].T @ Sref[k]) < TOL_STEP, k
            else:
                assert rel(S[b, k], Sref[k]) < TOL_STEP, k
        assert rel(Sx[b], o.get("Sx")) < TOL_STEP


@pytest.mark.gpu
def test_full_size_shard_properties(tog, gpu, gold):
    """B=8192, N=201 (one GPU's shard of the 65536-start job): size-independent properties."""
    prob, opts = tog.Problems.config_quad_maze(B=8192, N=201)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    st = solver.stats
    f = st["flags"]
    A = tog.abi
    assert not np.any(f & A.TRAJ_ACTIVE)  # every trajectory finished
    done = f & (A.TRAJ_AL_CONVERGED | A.TRAJ_AL_MAX_ITERS | A.TRAJ_COST_INCREASED | A.TRAJ_BP_ABORTED)
    assert np.all(done != 0)
    conv = (f & A.TRAJ_AL_CONVERGED) != 0
    assert conv.mean() > 0.3
    assert np.all(st["c_max"][conv] < opts.constraint_tolerance)
    assert np.all(np.isfinite(gp._X[conv])) and np.all(np.isfinite(gp._U[conv]))
    # converged: the terminal state is within the terminal box of quad_obs.jl:35-41 ± tolerance
    assert np.all(np.abs(gp._X[conv, -1, 1] - 60.0) < 1.0)
    # batching does not change a trajectory: the first 4 starts equal the committed solves
    for b in range(4):
        assert np.array_equal(gp._X[b], gold["X"][b]) and np.array_equal(gp._U[b], gold["U"][b]), b
        assert st["iterations_total"][b] == int(gold["stats"][b, A.STAT_TOTAL_STEPS]), b


@pytest.mark.gpu
def test_pattern_loop_equals_general_loop(tog, gpu, monkeypatch):
    """The std AL expansion's row loop over the Q.xx entries a stage row can change (DevProblem::qpat: for
    config 4, the x-y-z block of the cylinders and spheres and the bounded states' diagonal) adds the same
    terms in the same order as the general loop over all n entries: a solve with it equals one with the
    general loop (TOG_DENSE_RECORDS=1) bit for bit."""
    prob, opts = tog.Problems.config_quad_maze(B=24, N=201)
    out = []
    for dense in (False, True):
        if dense:
            monkeypatch.setenv("TOG_DENSE_RECORDS", "1")
        gp = prob.copy()
        s = tog.solve_b(gp, opts)
        out.append((gp._X, gp._U, s.handle.get(tog.abi.FIELD_STATS)))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
