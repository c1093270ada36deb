"""Configs 2 and 5 at their full benchmark sizes (BASELINE.json configs[1] and configs[4], SURVEY.md
§8(d)), solved to completion on the device exactly as bench.py's solve leg runs them (tog_solve with
the default budget: pending line searches, compacted tail launches, the tail kernels):

* config 2: cartpole swing-up, unconstrained iLQR, B = 1024 (problems/cartpole.jl:1-18);
* config 5: Kuka iiwa, AL-iLQR with the terminal goal and the notebook's options, B = 4096
  (examples/kuka_iiwa/Kuka iiwa.ipynb cells 7-16).

Properties over the whole batch: nothing left active, finite X/U, x0 kept, every converged trajectory
within its tolerance. Against the CPU oracle (oracle/tog_oracle.c): trajectories 0-3, the slowest one
and up to three that end without convergence: X/U within the north star's 1e-6 relative, iteration
counts and status flags exact. config 3's full batch is tests/test_config3_full.py."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_SOLVE = 1e-6


def full_batch_check(tog, oracle, prob, opts, converged_bit, cmax_tol=None):
    abi = tog.abi
    p = prob.copy()
    solver = tog.solve_b(p, opts)
    S = solver.handle.get(abi.FIELD_STATS)
    flags = S[:, abi.STAT_FLAGS].astype(np.int64)
    it = S[:, abi.STAT_TOTAL_STEPS].astype(np.int64)

    assert not np.any(flags & abi.TRAJ_ACTIVE)
    assert np.isfinite(p._X).all() and np.isfinite(p._U).all()
    assert np.array_equal(p._X[:, 0, :], prob.x0)
    conv = (flags & converged_bit) != 0
    assert conv.mean() > 0.9, conv.mean()
    if cmax_tol is not None:
        assert np.all(S[conv, abi.STAT_C_MAX] <= cmax_tol)

    picks = [0, 1, 2, 3, int(np.argmax(it))]
    nonconv = np.flatnonzero(~conv)
    picks += [int(b) for b in nonconv[:3]]
    picks = list(dict.fromkeys(picks))

    def run(b):
        o = oracle.OracleSolver(prob, opts, b=b)
        steps = o.solve()
        return b, steps, o.get("X"), o.get("U"), o.get("stats")

    with ThreadPoolExecutor(max_workers=len(picks)) as ex:
        results = list(ex.map(run, picks))
    for b, steps, X, U, st in results:
        assert steps == int(it[b]), (b, steps, int(it[b]))
        assert int(st[abi.STAT_FLAGS]) == int(flags[b]), b
        assert np.abs(p._X[b] - X).max() / max(1.0, np.abs(X).max()) < TOL_SOLVE, b
        assert np.abs(p._U[b] - U).max() / max(1.0, np.abs(U).max()) < TOL_SOLVE, b
    return it, nonconv, picks


@pytest.mark.timeout(600)
def test_config2_cartpole_full_batch_against_oracle(tog, gpu, oracle):
    prob, opts = tog.Problems.config_cartpole(B=1024)
    it, nonconv, picks = full_batch_check(tog, oracle, prob, opts, tog.abi.TRAJ_CONVERGED)
    print(f"config 2 full batch: max iterations {it.max()} (trajectory {int(np.argmax(it))}), "
          f"{len(nonconv)} not converged, oracle-checked {picks}")


@pytest.mark.timeout(900)
def test_config5_kuka_full_batch_against_oracle(tog, gpu, oracle):
    prob, opts = tog.Problems.config_kuka(B=4096)
    it, nonconv, picks = full_batch_check(tog, oracle, prob, opts, tog.abi.TRAJ_AL_CONVERGED,
                                          cmax_tol=opts.constraint_tolerance)
    print(f"config 5 full batch: max iterations {it.max()} (trajectory {int(np.argmax(it))}), "
          f"{len(nonconv)} not AL-converged, oracle-checked {picks}")
