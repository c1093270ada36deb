"""The convergence-tail launch modes are numerically invisible (DESIGN.md §5 "tail"):

* compacted launches: once the host has read back n_active <= 2048, tog_solve_step lists the active
  trajectories (k_list_active) and every kernel of the step runs over that many slots;
* the latency-sized backward kernel (k_bwd_team with a 1-wave/SIMD register budget).

A batch solved with compaction must equal the same batch solved with TOG_NO_COMPACT=1 bit for bit
(X, U and every per-trajectory statistic), and the first trajectories must equal the oracle."""
import os

import numpy as np
import pytest

TOL_SOLVE = 1e-6


def _solve(tog, B, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: v for k, v in env.items() if v is not None})
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
    try:
        prob, opts = tog.Problems.config_quadrotor(B=B)
        gpu = prob.copy()
        solver = tog.solve_b(gpu, opts)
        return prob, opts, gpu, solver.handle.get(tog.abi.FIELD_STATS)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.gpu
def test_compacted_tail_equals_full_launches(tog, gpu, oracle):
    B = 96
    prob, opts, a, Sa = _solve(tog, B, {"TOG_NO_COMPACT": None})
    _, _, b, Sb = _solve(tog, B, {"TOG_NO_COMPACT": "1"})
    assert np.array_equal(a._X, b._X)
    assert np.array_equal(a._U, b._U)
    assert np.array_equal(Sa, Sb)
    # spread of iteration counts: the later steps really ran with few trajectories active
    it = Sa[:, tog.abi.STAT_TOTAL_STEPS]
    assert it.max() > 2 * np.median(it)
    for bi in (0, int(np.argmax(it))):
        ref = oracle.OracleSolver(prob, opts, b=bi)
        steps = ref.solve()
        assert steps == int(it[bi])
        X, U = ref.get("X"), ref.get("U")
        assert np.abs(a._X[bi] - X).max() / max(1.0, np.abs(X).max()) < TOL_SOLVE
        assert np.abs(a._U[bi] - U).max() / max(1.0, np.abs(U).max()) < TOL_SOLVE


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["team"])
def test_tail_backward_kernels_agree(tog, gpu, kind):
    """The tail backward kernels (k_bwd_quad, the default, four waves per trajectory; the one-wave
    k_bwd_team; TOG_BWD_TAIL) perform the same operations in the same order: a batch solved with each equals the
    other bit for bit (X, U, every per-trajectory statistic). B = 24 keeps every step in the tail
    mode, and the restarts of the config-3 solves exercise the faithful replays. (Round 4's two- and
    three-wave variants are retired.)"""
    B = 24
    _, _, a, Sa = _solve(tog, B, {"TOG_BWD_TAIL": None})
    _, _, b, Sb = _solve(tog, B, {"TOG_BWD_TAIL": kind})
    assert np.array_equal(a._X, b._X)
    assert np.array_equal(a._U, b._U)
    assert np.array_equal(Sa, Sb)
    assert Sa[:, tog.abi.STAT_BP_RESTARTS].max() >= 0


@pytest.mark.gpu
def test_expansion_kernels_agree(tog, gpu):
    """The stage knots' square-root expansion on 4-lane teams (k_expand_u, the default) performs
    k_expand_team's operations in its order: a config-3 batch solved with TOG_EXPAND_QUAD=0 (every knot
    on k_expand_team) equals the default bit for bit (X, U, every per-trajectory statistic)."""
    B = 64
    _, _, a, Sa = _solve(tog, B, {"TOG_EXPAND_QUAD": None})
    _, _, b, Sb = _solve(tog, B, {"TOG_EXPAND_QUAD": "0"})
    assert np.array_equal(a._X, b._X)
    assert np.array_equal(a._U, b._U)
    assert np.array_equal(Sa, Sb)
