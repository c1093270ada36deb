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
