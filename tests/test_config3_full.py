"""Config 3 at its full benchmark size (BASELINE.json configs[1]): the quadrotor
AL-iLQR batch of B = 8192 trajectories solved to completion on the device, exactly as bench.py's
solve leg runs it (tog_solve with the default budget, every tail mode: pending line searches,
compacted launches, k_bwd_quad).

Properties over the whole batch: no trajectory left active, finite X/U, x0 kept, every AL-converged
trajectory within the constraint tolerance. Against the CPU oracle (oracle/tog_oracle.c, the
restatement of augmented_lagrangian_solver.jl / ilqr_solve.jl): trajectories 0-3, the slowest one and
three that end without AL convergence, X/U to 1e-6 relative, iteration counts and flags exact
(VERDICT r2 #3). The oracle runs in threads: ctypes releases the GIL."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL_SOLVE = 1e-6


@pytest.mark.timeout(900)
def test_config3_full_batch_against_oracle(tog, gpu, oracle):
    abi = tog.abi
    prob, opts = tog.Problems.config_quadrotor(B=8192)
    p = prob.copy()
    solver = tog.solve_b(p, opts)
    S = solver.handle.get(abi.FIELD_STATS)
    flags = S[:, abi.STAT_FLAGS].astype(np.int64)
    it = S[:, abi.STAT_TOTAL_STEPS].astype(np.int64)

    assert not np.any(flags & abi.TRAJ_ACTIVE)
    assert np.isfinite(p._X).all() and np.isfinite(p._U).all()
    assert np.array_equal(p._X[:, 0, :], prob.x0)
    conv = (flags & abi.TRAJ_AL_CONVERGED) != 0
    assert conv.mean() > 0.9
    assert np.all(S[conv, abi.STAT_C_MAX] <= opts.constraint_tolerance)

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
        assert steps == int(it[b]), b
        assert int(st[abi.STAT_FLAGS]) == int(flags[b]), b
        assert np.abs(p._X[b] - X).max() / max(1.0, np.abs(X).max()) < TOL_SOLVE, b
        assert np.abs(p._U[b] - U).max() / max(1.0, np.abs(U).max()) < TOL_SOLVE, b
    print(f"config 3 full batch: max iterations {it.max()} (trajectory {int(np.argmax(it))}), "
          f"{len(nonconv)} not AL-converged, oracle-checked {picks}")
