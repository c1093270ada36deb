"""Step-level entry points the reference exports and its tests call directly
(src/TrajectoryOptimization.jl:82-95; test/sqrt_bp_tests.jl:27-37). Each forwards to one
C-ABI call on the solver's device handle."""
from __future__ import annotations

import numpy as np

from . import abi
from .solvers import AbstractSolver, AugmentedLagrangianSolver, iLQRSolver, iLQRSolverOptions


def _al(solver) -> bool:
    return isinstance(solver, AugmentedLagrangianSolver)


def rollout_b(prob, solver: AbstractSolver | None = None, alpha: float | None = None):
    """``rollout!(prob)`` (src/rollout.jl:25-31) when ``alpha`` is None, else
    ``rollout!(prob, solver, alpha)`` (src/rollout.jl:2-23), which writes solver.X̄/Ū and returns
    the per-trajectory success flags."""
    if solver is None:
        solver = iLQRSolver(prob, iLQRSolverOptions())
    h = solver.handle
    if alpha is None:
        h.upload_state(prob)
        h.rollout_open_loop()
        prob._X[...] = h.get(abi.FIELD_X)
        return None
    ok = h.rollout(alpha)
    return ok if prob.batched else bool(ok[0])


def jacobian_b(prob, solver: AbstractSolver):
    """``jacobian!(prob, solver)`` (src/solvers.jl:126): A_k, B_k for k = 1..N-1 at (X, U)."""
    solver.handle.upload_state(prob)
    solver.handle.jacobians()


def update_constraints_b(prob, solver: AbstractSolver):
    """``update_constraints!(C, constraints, X, U)`` + ``update_active_set!`` on the current X, U
    (constraint_sets.jl:221-260; the AL expansion reads them, test/sqrt_bp_tests.jl:62-63)."""
    solver.handle.update_constraints()


def cost_expansion_b(prob, solver: AbstractSolver):
    """``cost_expansion!(prob, solver)`` (ilqr_methods.jl:55-62): ``reset!(solver.Q)`` then the
    stage/terminal expansion of the objective at (X, U) — the square-root factors when
    ``opts.square_root`` (objective.jl:51-94), plus the AL terms of the stored constraint values
    and active set for an AL solver (augmented_lagrangian_methods.jl:186-276). Computed on the device
    (``tog_cost_expansion``) into ``solver.Q``. The backward-pass kernels compute the same expansion
    fused, so ``backwardpass_b`` does not need this call; it is the reference's step-level entry point
    (test/sqrt_bp_tests.jl:27-37)."""
    sq = bool(_opts_ilqr(solver).square_root)
    solver.handle.cost_expansion(sqrt=sq, al=_al(solver))
    return solver.Q


def backwardpass_b(prob, solver: AbstractSolver, square_root: bool | None = None, store_S: bool = True):
    """``backwardpass!(prob, solver)`` (backward_pass.jl:1-7): returns ΔV (2,) or (B, 2)."""
    sq = bool(square_root) if square_root is not None else bool(_opts_ilqr(solver).square_root)
    dV = solver.handle.backward_pass(sqrt=sq, al=_al(solver), store_S=store_S)
    return dV if prob.batched else dV[0]


def forwardpass_b(prob, solver: AbstractSolver, dV, J_prev):
    """``forwardpass!(prob, solver, ΔV, J_prev)`` (forward_pass.jl:5-85): returns J."""
    J = solver.handle.forward_pass(J_prev, al=_al(solver))
    return J if prob.batched else float(J[0])


def cost(prob, solver: AbstractSolver | None = None):
    """``cost(prob)`` (src/problem.jl:240) — the AL cost when ``solver`` is an AL solver."""
    if solver is None:
        solver = iLQRSolver(prob, iLQRSolverOptions())
    solver.handle.upload_state(prob)
    J = solver.handle.cost(al=_al(solver))
    return J if prob.batched else float(J[0])


def _opts_ilqr(solver):
    o = solver.opts
    while not isinstance(o, iLQRSolverOptions):
        o = getattr(o, "opts_uncon", None) or getattr(o, "opts_al")
    return o
