"""tog_cost_expansion: cost_expansion!(prob, solver) as its own entry point
(ilqr_methods.jl:55-62 -> objective.jl:51-94, cost.jl:183-198; AL augmented_lagrangian_methods.jl:
186-276), against the oracle's oc_cost_expansion bit for bit, and the reference's std/sqrt
relation Q = UᵀU (test/sqrt_bp_tests.jl:38-44)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _split(q, n, m):
    Qx, Qu = q[..., :n], q[..., n:n + m]
    o = n + m
    Qxx = q[..., o:o + n * n].reshape(q.shape[:-1] + (n, n)).swapaxes(-1, -2)
    o += n * n
    Quu = q[..., o:o + m * m].reshape(q.shape[:-1] + (m, m)).swapaxes(-1, -2)
    o += m * m
    Qux = q[..., o:o + m * n].reshape(q.shape[:-1] + (n, m)).swapaxes(-1, -2)
    return Qx, Qu, Qxx, Quu, Qux


def _device_and_oracle(tog, oracle, prob, opts, sqrt, al):
    s = tog.AugmentedLagrangianSolver(prob, opts)
    h = s.handle
    h.rollout_open_loop()
    h.update_constraints()
    h.cost_expansion(sqrt=sqrt, al=al)
    Q = h.get(tog.abi.FIELD_Q)
    ref = []
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        o.rollout_open_loop()
        o.update_constraints()
        assert o.cost_expansion(sqrt, al) == 0
        ref.append(o.get("Q"))
    return Q, np.stack(ref)


@pytest.mark.parametrize("sqrt", [False, True])
@pytest.mark.parametrize("al", [False, True])
def test_cost_expansion_matches_oracle(tog, oracle, gpu, sqrt, al):
    prob, opts = tog.Problems.config_quadrotor(B=3)
    Q, R = _device_and_oracle(tog, oracle, prob, opts, sqrt, al)
    assert np.array_equal(Q, R)


def test_cost_expansion_infeasible_maze(tog, oracle, gpu):
    """69 constraint rows per knot, m = 17 (slack controls), sqrt + AL."""
    p = tog.Problems.quadrotor_maze()
    pinf = tog.infeasible_problem(p, 0.001)
    opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(square_root=True))
    s = tog.AugmentedLagrangianSolver(pinf, opts)
    h = s.handle
    h.slack_controls()
    h.update_constraints()
    h.cost_expansion(sqrt=True, al=True)
    o = oracle.OracleSolver(pinf, opts)
    o.slack_controls()
    o.update_constraints()
    assert o.cost_expansion(True, True) == 0
    assert np.array_equal(h.get(tog.abi.FIELD_Q)[0], o.get("Q"))


def test_sqrt_expansion_is_a_factor(tog, gpu):
    """sqrt_bp_tests.jl:38-44: the square-root expansion's factors reproduce the std expansion."""
    prob, opts = tog.Problems.config_quadrotor(B=2)
    n, m = 13, 4
    h = tog.AugmentedLagrangianSolver(prob, opts).handle
    h.rollout_open_loop()
    h.update_constraints()
    h.cost_expansion(sqrt=False, al=True)
    Qs = _split(h.get(tog.abi.FIELD_Q), n, m)
    h.cost_expansion(sqrt=True, al=True)
    Qr = _split(h.get(tog.abi.FIELD_Q), n, m)
    UtU = np.einsum("...ki,...kj->...ij", Qr[2], Qr[2])
    assert np.allclose(UtU, Qs[2], rtol=np.sqrt(np.finfo(float).eps), atol=1e-10)
    UtU = np.einsum("...ki,...kj->...ij", Qr[3][:, :-1], Qr[3][:, :-1])
    assert np.allclose(UtU, Qs[3][:, :-1], rtol=np.sqrt(np.finfo(float).eps), atol=1e-10)
    assert np.array_equal(Qr[0], Qs[0]) and np.array_equal(Qr[1], Qs[1])


def test_solve_al_entry_point(tog, gpu):
    """tog_solve_al(h) == tog_solve(h, AL, iterations*al_iterations + 1) == solve_b."""
    prob, opts = tog.Problems.config_quadrotor(B=3)
    p1 = prob.copy()
    tog.solve_b(p1, opts)
    s = tog.AugmentedLagrangianSolver(prob.copy(), opts)
    tog.abi.check(s.handle.lib, s.handle.lib.tog_solve_al(s.handle.h))
    assert np.array_equal(s.handle.get(tog.abi.FIELD_X), p1._X)
