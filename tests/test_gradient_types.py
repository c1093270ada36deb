"""gradient_type options of iLQRSolverOptions (src/solvers/ilqr/ilqr_solver.jl:20): :todorov (default),
:feedforward, :ℓ2 and :ℓinf (calculate_gradient, src/solvers/ilqr/ilqr_methods.jl:91-116).

:ℓ2 / :ℓinf take the norm of compute_gradient, vcat(Q[1].x, Q[1].u, ..., Q[N].x) of the plain cost
expansion at the accepted trajectory (the AL objective's inside AL solves). The CPU tests pin the
oracle's recorded gradient to that definition, recomputed from the oracle's own cost expansion; the GPU
tests hold the device solve to the oracle (iteration counts exact, X and U to the north-star bar).
Parity with the reference for :ℓ2 is to rounding only: Julia 1.1 hands these long vectors to BLAS.nrm2,
whose accumulation order and precision belong to the BLAS build.
"""
import numpy as np
import pytest

from test_gpu_parity import _solve_and_compare

STAT_GRADIENT = 2


def _expansion_vector(o, al):
    """vcat(Q[k].x, Q[k].u ..., Q[N].x) from the oracle's plain cost expansion at its current X, U."""
    n, m, N = o.n, o.m, o.N
    o.cost_expansion(sqrt=False, al=al)
    Q = o.get("Q")
    parts = []
    for k in range(N - 1):
        parts += [Q[k, :n], Q[k, n:n + m]]
    parts.append(Q[N - 1, :n])
    return np.concatenate(parts)


@pytest.mark.parametrize("gt", ["ℓ2", "ℓinf"])
def test_oracle_gradient_is_norm_of_expansion(tog, oracle, gt):
    """The oracle's recorded gradient after an iLQR solve equals the norm of the cost expansion's
    gradient entries at the final trajectory (ilqr_methods.jl:104-116)."""
    prob, _ = tog.Problems.config_cartpole(B=1)
    opts = tog.iLQRSolverOptions(gradient_type=gt, iterations=40)
    o = oracle.OracleSolver(prob, opts, b=0)
    steps = o.solve()
    assert steps > 0
    g = o.get("stats")[STAT_GRADIENT]
    v = _expansion_vector(o, al=False)
    if gt == "ℓinf":
        assert g == np.max(np.abs(v))
    else:
        assert abs(g - np.linalg.norm(v)) <= 1e-12 * max(1.0, np.linalg.norm(v))


def test_oracle_gradient_types_change_the_solve(tog, oracle):
    """The measure feeds evaluate_convergence (ilqr_methods.jl:139-162): a tolerance that only the
    ℓinf norm of the expansion meets ends the solve at a different iteration than :todorov."""
    prob, _ = tog.Problems.config_cartpole(B=1)
    counts = {}
    for gt in ("todorov", "ℓinf"):
        opts = tog.iLQRSolverOptions(gradient_type=gt, gradient_norm_tolerance=1e-2, cost_tolerance=1e-12,
                                     iterations=300)
        counts[gt] = oracle.OracleSolver(prob, opts, b=0).solve()
    assert counts["todorov"] != counts["ℓinf"]


def test_gradient_type_validation(tog):
    with pytest.raises(ValueError):
        tog.to_tog_options(tog.iLQRSolverOptions(gradient_type="l1"))
    assert tog.to_tog_options(tog.iLQRSolverOptions(gradient_type="ℓinf")).gradient_type == 3
    assert tog.to_tog_options(tog.iLQRSolverOptions(gradient_type="l2")).gradient_type == 2


@pytest.mark.gpu
@pytest.mark.parametrize("gt", ["feedforward", "ℓ2", "ℓinf"])
def test_gradient_type_cartpole_ilqr(tog, oracle, gpu, gt):
    """Config 2 shape (unconstrained iLQR): device == oracle under each gradient measure."""
    prob, _ = tog.Problems.config_cartpole(B=4)
    opts = tog.iLQRSolverOptions(gradient_type=gt, gradient_norm_tolerance=1e-3, iterations=150)
    _solve_and_compare(tog, oracle, prob, opts)


@pytest.mark.gpu
@pytest.mark.parametrize("gt", ["feedforward", "ℓ2", "ℓinf"])
def test_gradient_type_quadrotor_al(tog, oracle, gpu, gt):
    """Config 3 shape (AL-iLQR, square-root backward pass): the ℓ2 / ℓinf measures take the AL
    objective's plain expansion (constraint terms included)."""
    prob, opts = tog.Problems.config_quadrotor(B=3)
    opts.opts_uncon.gradient_type = gt
    opts.opts_uncon.gradient_norm_tolerance = 1e-2
    opts.gradient_norm_tolerance_intermediate = 1e-2
    _solve_and_compare(tog, oracle, prob, opts)
