"""The three line-search schedules of the device forward pass give the same solve, bit for bit.

forwardpass! (src/solvers/ilqr/forward_pass.jl:5-85) is evaluated speculatively (trial j at α = 2⁻ʲ)
and decided by replaying the reference's sequential acceptance loop. How the trials are scheduled
must not change any result:

* pending (default for batches above 65536 / 21 trajectories): one round of 8 trials per batch step;
  a trajectory left undecided continues its line search in the next batch step, skipping that step's
  Jacobians and backward pass. The accepted rollout is copied from its trial's candidate slot.
* two rounds (``TOG_LS_NOPEND=1``): trials [0, 8) then [8, 21) for the undecided, in the same step.
* replay (``TOG_LS=replay``): the accepted α is rolled out again in place (k_ls_commit).

The batches are large enough to take the pending path; tog_solve's periodic n_active readback also
switches the tail to single 21-trial rounds, so all three schedules meet in one solve. Trajectories
0 and 1 are also checked against the CPU oracle.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(tog, prob, opts, mode, env):
    saved = {k: os.environ.get(k) for k in ("TOG_LS", "TOG_LS_NOPEND")}
    for k in saved:
        os.environ.pop(k, None)
    os.environ.update(env)
    try:
        p = prob.copy()
        solver = tog.AbstractSolverFor(p, opts, device=0)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    h = solver.handle
    h.solve(mode, max_steps=3000)
    h.download_state(p)
    return p, h.stats_dict(), h.status()


@pytest.mark.parametrize("case", ["quadrotor_al", "cartpole_ilqr"])
def test_line_search_schedules_agree(tog, oracle, gpu, case):
    if case == "quadrotor_al":
        prob, opts = tog.Problems.config_quadrotor(B=4096)
        opts.iterations = 3  # three AL outer iterations keep the solve short
        mode = tog.abi.MODE_AL
    else:
        prob, opts = tog.Problems.config_cartpole(B=4096)
        mode = tog.abi.MODE_ILQR
    ref = _solve(tog, prob, opts, mode, {})
    for env in ({"TOG_LS_NOPEND": "1"}, {"TOG_LS": "replay"}):
        got = _solve(tog, prob, opts, mode, env)
        assert np.array_equal(ref[0]._X, got[0]._X), env
        assert np.array_equal(ref[0]._U, got[0]._U), env
        assert np.array_equal(ref[1]["iterations_total"], got[1]["iterations_total"]), env
        assert np.array_equal(ref[2], got[2]), env
    for b in (0, 1):
        o = oracle.OracleSolver(prob, opts, b=b)
        o.solve()
        X, U = o.get("X"), o.get("U")
        assert np.max(np.abs(ref[0]._X[b] - X)) <= 1e-6 * max(1.0, np.max(np.abs(X)))
        assert np.max(np.abs(ref[0]._U[b] - U)) <= 1e-6 * max(1.0, np.max(np.abs(U)))


def test_default_budget_covers_pending_rounds(tog, oracle, gpu):
    """in pending mode an iteration can take ceil(nc / 8) batch steps, so the default
    step budget (tog_solve_budget) must let every trajectory reach its own iteration limits. The old
    budget of one iteration per step (iterations x al_iterations + 1) stops trajectories whose line
    searches pended while they are still active; the default budget ends them all with their
    iteration flags, as the reference's solve! loops (augmented_lagrangian_solve.jl / ilqr_solve.jl)
    do, and matches the oracle. The maze's AL line searches backtrack past 8 trials as the penalties
    grow; B = 8192 keeps the batch in pending mode for most of the solve."""
    prob, opts = tog.Problems.config_quad_maze(B=8192)
    il = opts.opts_uncon
    il.iterations = 2                  # small caps that every trajectory reaches: dJ never
    il.cost_tolerance = 0.0            # converges an inner solve, the constraints never converge
    il.gradient_norm_tolerance = 0.0   # the AL solve: 15 outer iterations of one iLQR step each,
    opts.iterations = 15               # the later ones backtracking past 8 trials (oracle: 19 of
    opts.cost_tolerance = 0.0          # the first 32 trajectories need more than 31 batch steps)
    opts.cost_tolerance_intermediate = 0.0
    opts.constraint_tolerance = 0.0
    mode = tog.abi.MODE_AL
    old_budget = il.iterations * opts.iterations + 1

    p_old = prob.copy()
    s_old = tog.AbstractSolverFor(p_old, opts, device=0)
    s_old.handle.solve(mode, max_steps=old_budget)
    st_old = s_old.handle.status()
    short = np.flatnonzero(st_old & tog.abi.TRAJ_ACTIVE)
    assert short.size > 0, "no trajectory outlived the old budget: the case does not exercise it"

    p = prob.copy()
    solver = tog.solve_b(p, opts)
    h = solver.handle
    assert h.solve_budget(mode) == old_budget * -(-(il.iterations_linesearch + 1) // 8)
    flags = solver.stats["flags"]
    assert not np.any(flags & tog.abi.TRAJ_ACTIVE)
    assert np.all(flags & (tog.abi.TRAJ_AL_MAX_ITERS | tog.abi.TRAJ_AL_CONVERGED))
    for b in (int(short[0]), int(short[-1])):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        assert steps == int(solver.stats["iterations_total"][b]), b
        assert int(o.get("stats")[tog.abi.STAT_FLAGS]) == int(flags[b]), b
        X, U = o.get("X"), o.get("U")
        assert np.max(np.abs(p._X[b] - X)) <= 1e-6 * max(1.0, np.max(np.abs(X))), b
        assert np.max(np.abs(p._U[b] - U)) <= 1e-6 * max(1.0, np.max(np.abs(U))), b
