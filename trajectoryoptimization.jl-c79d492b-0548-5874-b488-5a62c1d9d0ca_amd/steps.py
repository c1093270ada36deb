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


def cost_expansion_b(prob, solver: AbstractSolver):
    """``cost_expansion!(prob, solver)`` (ilqr_methods.jl:55-62). On the device the expansion is
    fused into the backward-pass kernel, so this only validates the call order."""
    solver._expansion_ready = True


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
