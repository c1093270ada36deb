"""Solver plugin interface mirror (src/solvers.jl:7-126, docs/src/solvers.md:25-47).

``iLQRSolverOptions`` / ``AugmentedLagrangianSolverOptions`` / ``ALTROSolverOptions`` mirror the
reference's ``@with_kw`` option structs (same field names and defaults);
``iLQRSolver`` / ``AugmentedLagrangianSolver`` / ``ALTROSolver`` are ``AbstractSolver``s whose
buffers live on the GPU behind the C ABI (include/tog.h); ``solve_b(prob, opts)`` is the
reference's ``solve!`` and ``solve(prob, opts)`` its copying variant (src/solvers.jl:91-123).

Errors follow the reference: invalid arguments raise ``ValueError`` (ArgumentError),
``Cost increased during Forward Pass`` raises ``RuntimeError`` when a trajectory reports it
(forward_pass.jl:80-82), and a ``PosDefException`` of the square-root backward pass's
``lowrankdowndate!`` (backward_pass.jl:186-192) raises ``PosDefException`` (a
``numpy.linalg.LinAlgError``); a batch raises after every trajectory has finished (the failed ones
stop where the reference's exception would, flagged ``TRAJ_SQRT_PD_FAIL | TRAJ_BP_ABORTED``). The
``@warn``s become per-trajectory status flags in ``solver.stats``.
"""
from __future__ import annotations

import copy as _copy
from dataclasses import dataclass, field

import numpy as np

from . import abi
import ctypes as C

from .device import BatchHandle, al_traj_stats, ilqr_traj_stats, stats_dict


class PosDefException(np.linalg.LinAlgError):
    """LinearAlgebra.PosDefException: a trajectory's square-root backward pass hit a downdate that is
    not positive definite (chol_minus, backward_pass.jl:186-192). ``trajectories`` lists them."""

    def __init__(self, trajectories):
        self.trajectories = list(trajectories)
        super().__init__(f"PosDefException in chol_minus (lowrankdowndate!) for trajectories {self.trajectories}")


def _raise_trajectory_errors(flags):
    """The reference's exceptions, after the batch: cost increase (forward_pass.jl:80-82) and the
    downdate's PosDefException."""
    flags = np.asarray(flags)
    if np.any(flags & abi.TRAJ_SQRT_PD_FAIL):
        raise PosDefException(np.nonzero(flags & abi.TRAJ_SQRT_PD_FAIL)[0].tolist())
    if np.any(flags & abi.TRAJ_COST_INCREASED):
        raise RuntimeError("Error: Cost increased during Forward Pass")


# ----------------------------------------------------------------------------- options

# gradient_type symbols (ilqr_solver.jl:20) -> tog_options.gradient_type; the ASCII spellings are accepted too
GRADIENT_TYPES = {"todorov": 0, "feedforward": 1, "ℓ2": 2, "l2": 2, "ℓinf": 3, "linf": 3}


@dataclass
class iLQRSolverOptions:
    """src/solvers/ilqr/ilqr_solver.jl:7-81 (defaults identical)."""

    verbose: bool = False
    live_plotting: str = "off"
    cost_tolerance: float = 1.0e-4
    gradient_type: str = "todorov"
    gradient_norm_tolerance: float = 1.0e-5
    iterations: int = 300
    dJ_counter_limit: int = 10
    square_root: bool = False
    line_search_lower_bound: float = 1.0e-8
    line_search_upper_bound: float = 10.0
    iterations_linesearch: int = 20
    bp_reg_initial: float = 0.0
    bp_reg_increase_factor: float = 1.6
    bp_reg_max: float = 1.0e8
    bp_reg_min: float = 1.0e-8
    bp_reg_type: str = "control"
    bp_reg_fp: float = 10.0
    bp_sqrt_inv_type: str = "pseudo"
    bp_reg_sqrt_initial: float = 1.0e-6
    bp_reg_sqrt_increase_factor: float = 10.0
    max_cost_value: float = 1.0e8
    max_state_value: float = 1.0e8
    max_control_value: float = 1.0e8

    def copy(self):
        return _copy.deepcopy(self)


@dataclass
class AugmentedLagrangianSolverOptions:
    """src/solvers/augmented_lagrangian/augmented_lagrangian_solver.jl:8-66."""

    verbose: bool = False
    opts_uncon: iLQRSolverOptions = field(default_factory=iLQRSolverOptions)
    cost_tolerance: float = 1.0e-4
    cost_tolerance_intermediate: float = 1.0e-3
    gradient_norm_tolerance: float = 1.0e-5
    gradient_norm_tolerance_intermediate: float = 1.0e-5
    constraint_tolerance: float = 1.0e-3
    constraint_tolerance_intermediate: float = 1.0e-3
    iterations: int = 30
    dual_min: float = -1.0e8
    dual_max: float = 1.0e8
    penalty_max: float = 1.0e8
    penalty_initial: float = 1.0
    penalty_scaling: float = 10.0
    penalty_scaling_no: float = 1.0
    constraint_decrease_ratio: float = 0.25
    outer_loop_update_type: str = "default"
    active_constraint_tolerance: float = 0.0
    kickout_max_penalty: bool = False

    def copy(self):
        return _copy.deepcopy(self)


@dataclass
class ProjectedNewtonSolverOptions:
    """``ProjectedNewtonSolverOptions`` (src/solvers/direct/direct_solvers.jl:14-30). Only
    ``solve_type = "feasible"`` (the default) is built."""

    verbose: bool = True
    n_steps: int = 1
    solve_type: str = "feasible"
    active_set_tolerance: float = 1.0e-3
    feasibility_tolerance: float = 1.0e-6

    def copy(self):
        return _copy.deepcopy(self)


def to_tog_pn_options(opts: ProjectedNewtonSolverOptions) -> abi.tog_pn_options:
    if opts.solve_type not in ("feasible", "optimal"):
        raise ValueError("solve_type must be :feasible or :optimal")
    o = abi.tog_pn_options()
    o.n_steps = int(opts.n_steps)
    o.solve_type = 1 if opts.solve_type == "optimal" else 0
    o.active_set_tolerance = float(opts.active_set_tolerance)
    o.feasibility_tolerance = float(opts.feasibility_tolerance)
    return o


@dataclass
class ALTROSolverOptions:
    """src/solvers/altro/altro_solver.jl:6-65. With a NaN initial state trajectory ALTRO is the AL
    solve; with a given X it is the infeasible-start solve (altro_methods.jl:98-124, infeasible.jl).
    ``projected_newton`` adds phase 2, the projected Newton feasible projection
    (altro_methods.jl:5-39). A problem with tf = 0 is solved as minimum_time_problem
    (src/solvers/altro/minimum_time.jl, R_minimum_time / dt_max / dt_min)."""

    verbose: bool = False
    opts_al: AugmentedLagrangianSolverOptions = field(default_factory=AugmentedLagrangianSolverOptions)
    constraint_tolerance_infeasible: float = 1.0e-5
    R_inf: float = 1.0
    dynamically_feasible_projection: bool = True
    resolve_feasible_problem: bool = True
    penalty_initial_infeasible: float = 1.0
    penalty_scaling_infeasible: float = 10.0
    R_minimum_time: float = 1.0
    dt_max: float = 1.0
    dt_min: float = 1.0e-3
    penalty_initial_minimum_time_inequality: float = 1.0
    penalty_initial_minimum_time_equality: float = 1.0
    penalty_scaling_minimum_time_inequality: float = 1.0
    penalty_scaling_minimum_time_equality: float = 1.0
    projected_newton: bool = False
    opts_pn: ProjectedNewtonSolverOptions = field(default_factory=ProjectedNewtonSolverOptions)
    projected_newton_tolerance: float = 1.0e-3

    def copy(self):
        return _copy.deepcopy(self)


def to_tog_options(opts) -> abi.tog_options:
    """Flatten reference option structs into the C ABI's POD ``tog_options``."""
    o = abi.default_options()
    if isinstance(opts, ALTROSolverOptions):
        opts = opts.opts_al
    if isinstance(opts, AugmentedLagrangianSolverOptions):
        al, il = opts, opts.opts_uncon
    else:
        al, il = AugmentedLagrangianSolverOptions(), opts
    o.cost_tolerance = il.cost_tolerance
    o.gradient_norm_tolerance = il.gradient_norm_tolerance
    o.iterations = int(il.iterations)
    o.dJ_counter_limit = int(il.dJ_counter_limit)
    o.square_root = int(bool(il.square_root))
    if il.bp_reg_type not in ("control", "state"):
        raise ValueError("bp_reg_type must be :control or :state")
    o.bp_reg_type = 0 if il.bp_reg_type == "control" else 1
    # calculate_gradient (ilqr_methods.jl:91-102): :todorov, :feedforward, :ℓ2, :ℓinf
    if il.gradient_type not in GRADIENT_TYPES:
        raise ValueError(f"gradient_type must be one of {sorted(GRADIENT_TYPES)}")
    o.gradient_type = GRADIENT_TYPES[il.gradient_type]
    o.iterations_linesearch = int(il.iterations_linesearch)
    o.line_search_lower_bound = il.line_search_lower_bound
    o.line_search_upper_bound = il.line_search_upper_bound
    o.bp_reg_increase_factor = il.bp_reg_increase_factor
    o.bp_reg_max = il.bp_reg_max
    o.bp_reg_min = il.bp_reg_min
    o.bp_reg_fp = il.bp_reg_fp
    o.max_cost_value = il.max_cost_value
    o.max_state_value = il.max_state_value
    o.max_control_value = il.max_control_value
    o.al_cost_tolerance = al.cost_tolerance
    o.al_cost_tolerance_intermediate = al.cost_tolerance_intermediate
    o.al_gradient_norm_tolerance = al.gradient_norm_tolerance
    o.al_gradient_norm_tolerance_intermediate = al.gradient_norm_tolerance_intermediate
    o.constraint_tolerance = al.constraint_tolerance
    o.dual_min = al.dual_min
    o.dual_max = al.dual_max
    o.penalty_max = al.penalty_max
    o.penalty_initial = al.penalty_initial
    o.penalty_scaling = al.penalty_scaling
    o.al_iterations = int(al.iterations)
    o.kickout_max_penalty = int(bool(al.kickout_max_penalty))
    return o


def solver_name(opts) -> str:
    """src/solvers.jl:35-41."""
    if isinstance(opts, iLQRSolverOptions):
        return "iLQR"
    if isinstance(opts, ALTROSolverOptions):
        return "ALTRO"
    if isinstance(opts, AugmentedLagrangianSolverOptions):
        return "AL-" + solver_name(opts.opts_uncon)
    return solver_name(opts.opts)


# ----------------------------------------------------------------------------- solvers

@dataclass
class Expansion:
    """``Expansion{T}`` (src/cost.jl:5-33): x, u, xx, uu, ux, batched over (B, N)."""

    x: np.ndarray
    u: np.ndarray
    xx: np.ndarray
    uu: np.ndarray
    ux: np.ndarray

    @classmethod
    def from_flat(cls, q, n, m):
        """Split TOG_FIELD_Q's per-knot record [x; u; xx; uu; ux] (matrices column-major)."""
        lead = q.shape[:-1]
        o = n + m
        xx = q[..., o:o + n * n].reshape(lead + (n, n)).swapaxes(-1, -2)
        o += n * n
        uu = q[..., o:o + m * m].reshape(lead + (m, m)).swapaxes(-1, -2)
        o += m * m
        ux = q[..., o:o + m * n].reshape(lead + (n, m)).swapaxes(-1, -2)
        return cls(q[..., :n].copy(), q[..., n:n + m].copy(), np.ascontiguousarray(xx), np.ascontiguousarray(uu),
                   np.ascontiguousarray(ux))

class AbstractSolver:
    """``AbstractSolver{T}`` (src/solvers.jl:7). Holds ``opts``, ``stats`` and the device handle."""

    mode = abi.MODE_ILQR

    def __init__(self, prob, opts, device: int = 0, stream=None, devices=None):
        self.opts = opts
        self.stats: dict = {}
        self.history = None
        self.handle = BatchHandle(prob, to_tog_options(opts), device=device, stream=stream, devices=devices)
        self.n, self.m, self.N = prob.model.n, prob.model.m, prob.N

    def size(self):
        return self.n, self.m, self.N

    def reset_b(self):
        self.stats = {}
        self.history = None

    def traj_stats(self, b: int) -> dict:
        """Trajectory b's ``solver.stats`` as the reference builds it, with its per-iteration vectors:
        iLQR :iterations, :cost, :dJ, :gradient, :dJ_zero_counter (ilqr_methods.jl:77-89); AL
        :iterations, :iterations_total, :iterations_inner, :cost, :c_max, :penalty_max and stats_uncon
        (augmented_lagrangian_methods.jl:79-97). ``solver.stats`` itself is the batch summary (final
        values, one entry per trajectory). Needs the histories the solve recorded (solve_b's `history`)."""
        if self.history is None:
            raise RuntimeError("no iteration histories: solve with history enabled (solve_b(..., history=True))")
        inner, outer, cnt = self.history
        n_in, n_out = int(cnt[b, 0]), int(cnt[b, 1])
        if self.mode == abi.MODE_AL:
            return al_traj_stats(inner[b], n_in, outer[b], n_out)
        zc = self.stats["dJ_zero_counter"][b] if "dJ_zero_counter" in self.stats else None
        d = ilqr_traj_stats(inner[b], min(n_in, inner.shape[1]), zc)
        d["truncated"] = bool(n_in > inner.shape[1])
        return d

    # ---- device views (copies to host), reference field names
    @property
    def K(self):
        return self.handle.get(abi.FIELD_K)

    @property
    def d(self):
        return self.handle.get(abi.FIELD_D)

    @property
    def Xbar(self):
        return self.handle.get(abi.FIELD_XBAR)

    @property
    def Ubar(self):
        return self.handle.get(abi.FIELD_UBAR)

    @property
    def rho(self):
        return self.handle.get(abi.FIELD_RHO)

    @property
    def Q(self):
        """``solver.Q``: the cost-to-go expansion of the last ``cost_expansion!`` (ilqr_solver.jl:
        130-131), per knot ``Expansion(x, u, xx, uu, ux)`` as batched arrays (B, N, ...). The
        terminal knot's u-parts are zero. With ``square_root`` xx and uu hold upper factors."""
        return Expansion.from_flat(self.handle.get(abi.FIELD_Q), self.n, self.m)


class iLQRSolver(AbstractSolver):
    """``iLQRSolver`` (ilqr_solver.jl:93-144)."""

    mode = abi.MODE_ILQR


class AugmentedLagrangianSolver(AbstractSolver):
    """``AugmentedLagrangianSolver`` (augmented_lagrangian_solver.jl:101-140)."""

    mode = abi.MODE_AL

    @property
    def lam(self):
        return self.handle.get(abi.FIELD_LAMBDA)

    @property
    def mu(self):
        return self.handle.get(abi.FIELD_MU)

    @property
    def C(self):
        return self.handle.get(abi.FIELD_C)


class ALTROSolver(AugmentedLagrangianSolver):
    """``ALTROSolver`` (altro_solver.jl:70-94). After ``solve_b(prob, ALTROSolverOptions)``: ``stats`` holds
    the reference's :time, :time_al, :time_pn (seconds, altro_methods.jl:44-48) next to the AL phase's
    batch summary; ``solver_al`` is the AL phase's solver (its device buffers: K, d, λ, μ, ... of the
    infeasible / minimum-time problem when the start was one; ``solver_al.traj_stats(b)`` its per-iteration
    statistics); ``solver_pn`` the projected Newton phase (``solver_pn.traj_stats(b)``: :iterations,
    :cost, :c_max per newton step). The solver's own device views are solver_al's."""


def history_capacity(opts, B: int, budget_bytes: float = 256e6) -> int:
    """Inner records per trajectory solve_b keeps by default: a whole solve's worth (an AL solve records at
    most al_iterations x (iterations + 1)), capped so that the batch's histories stay within `budget_bytes`
    of HBM (24 B a record; a longer history is counted, not stored)."""
    o = to_tog_options(opts)
    full = (o.iterations + 1) * (o.al_iterations if isinstance(opts, (AugmentedLagrangianSolverOptions,
                                                                       ALTROSolverOptions)) else 1) + 1
    return int(max(1, min(full, budget_bytes // (24 * max(1, B)))))


class ProjectedNewtonSolver(AbstractSolver):
    """``ProjectedNewtonSolver`` (direct_solvers.jl:43-113): the feasible projection of ALTRO's
    phase 2 on the device (tog_solve_pn). ``V`` starts from the problem's X, U
    (``PrimalDual(prob)``, primals.jl:158-193). ``stats`` holds per-trajectory ``c_max``, ``cost``,
    ``iterations`` (newton steps), the final projection ``viol`` and work counters."""

    mode = abi.MODE_AL

    def __init__(self, prob, opts: ProjectedNewtonSolverOptions | None = None, **kw):
        opts = ProjectedNewtonSolverOptions() if opts is None else opts
        super().__init__(prob, iLQRSolverOptions(), **kw)
        self.opts = opts
        self.handle.upload_state(prob)


def _pn_stats(out, flags):
    return {"c_max": out[:, abi.PN_C_MAX].copy(), "cost": out[:, abi.PN_J].copy(),
            "viol": out[:, abi.PN_VIOL].copy(), "iterations": out[:, abi.PN_STEPS].astype(int),
            "projections": out[:, abi.PN_PROJECTIONS].astype(int),
            "linesearches": out[:, abi.PN_LINESEARCHES].astype(int),
            "refinements": out[:, abi.PN_REFINEMENTS].astype(int), "flags": flags}


class _PNStatsView(ProjectedNewtonSolver):
    """ALTROSolver.solver_pn after an ALTRO solve: the projected Newton statistics on the AL phase's buffers."""

    def traj_stats(self, b: int) -> dict:
        """solver_pn.stats of trajectory b (projected_newton.jl:23-29): :iterations and the :cost, :c_max
        vectors, one entry per newton step."""
        hist, rec = self.pn_history
        k = int(rec[b])
        return {"iterations": k, "cost": hist[b, :k, 0].copy(), "c_max": hist[b, :k, 1].copy()}


def _solve_pn(prob, solver: ProjectedNewtonSolver):
    """``solve!(prob, ::ProjectedNewtonSolver)`` (projected_newton.jl:6-20). The reference raises
    (a MethodError in ``_projection_linesearch!``, projected_newton.jl:273-277) when a line search's
    first trial does not reduce the violation; that trajectory is flagged TRAJ_PN_ERROR and a
    ``RuntimeError`` is raised after the batch."""
    h = solver.handle
    out = h.solve_pn(to_tog_pn_options(solver.opts))
    h.download_state(prob)
    flags = h.status()
    solver.stats = _pn_stats(out, flags)
    solver.pn_history = h.pn_history(solver.opts.n_steps)
    _raise_pn_errors(flags, solver)
    return solver


class ProjectedNewtonError(RuntimeError):
    """The reference's exception in ``_projection_linesearch!`` (``count += a``, a MethodError, when the first
    trial does not reduce the violation; projected_newton.jl:273-277), raised after the batch.
    ``trajectories`` lists the flagged ones (TRAJ_PN_ERROR; they keep their last accepted iterate) and
    ``solver`` is the finished solve (its statistics and the other trajectories' results stand)."""

    def __init__(self, msg, trajectories, solver):
        super().__init__(msg)
        self.trajectories = list(trajectories)
        self.solver = solver


def _raise_pn_errors(flags, solver):
    flags = np.asarray(flags)
    if np.any(flags & abi.TRAJ_PN_BLOCK):
        raise ProjectedNewtonError("projected Newton: a block of n + active rows exceeded the device's 64 rows "
                                   "(TOG_TRAJ_PN_BLOCK)", np.flatnonzero(flags & abi.TRAJ_PN_BLOCK), solver)
    if np.any(flags & abi.TRAJ_PN_ERROR):
        bad = np.flatnonzero(flags & abi.TRAJ_PN_ERROR)
        raise ProjectedNewtonError("projected Newton: line search did not reduce the violation for trajectories "
                                   f"{bad.tolist()} (the reference's _projection_linesearch! raises here)", bad, solver)


def AbstractSolverFor(prob, opts, **kw):
    """``AbstractSolver(prob, opts)`` dispatch on the options type (src/solvers.jl:60-62)."""
    if isinstance(opts, iLQRSolverOptions):
        return iLQRSolver(prob, opts, **kw)
    if isinstance(opts, ALTROSolverOptions):
        _altro_pn_tolerances(opts)
        return ALTROSolver(prob, opts, **kw)
    if isinstance(opts, ProjectedNewtonSolverOptions):
        return ProjectedNewtonSolver(prob, opts, **kw)
    if isinstance(opts, AugmentedLagrangianSolverOptions):
        return AugmentedLagrangianSolver(prob, opts, **kw)
    raise ValueError("Can't create an Abstract Solver without knowing the type of the Solver Options")


def _altro_pn_tolerances(opts):
    """altro_methods.jl:5-13: with projected Newton the AL phase stops at projected_newton_tolerance
    (or runs to kickout at max penalty when that is negative). Mutates opts.opts_al, as the
    reference does."""
    if opts.projected_newton:
        if opts.projected_newton_tolerance >= 0:
            opts.opts_al.constraint_tolerance = opts.projected_newton_tolerance
        else:
            opts.opts_al.constraint_tolerance = 0.0
            opts.opts_al.kickout_max_penalty = True


def _altro_infeasible(prob) -> bool:
    """``!all(isnan, prob.X[1])`` (altro_methods.jl:101): the whole batch must agree."""
    given = ~np.isnan(prob._X[:, 0, :]).all(axis=1)
    if given.any() and not given.all():
        raise ValueError("infeasible start: X must be given for every trajectory of the batch or for none")
    return bool(given.all())


def to_tog_altro_options(opts: ALTROSolverOptions) -> abi.tog_altro_options:
    """ALTROSolverOptions -> the C ABI's ``tog_altro_options`` (its live fields)."""
    a = abi.tog_altro_options()
    a.opts_al = to_tog_options(opts.opts_al)
    a.R_inf = float(opts.R_inf)
    a.R_minimum_time = float(opts.R_minimum_time)
    a.dt_max = float(opts.dt_max)
    a.dt_min = float(opts.dt_min)
    a.projected_newton_tolerance = float(opts.projected_newton_tolerance)
    a.dynamically_feasible_projection = int(bool(opts.dynamically_feasible_projection))
    a.resolve_feasible_problem = int(bool(opts.resolve_feasible_problem))
    a.projected_newton = int(bool(opts.projected_newton))
    a.opts_pn = to_tog_pn_options(opts.opts_pn) if opts.projected_newton else abi.tog_pn_options(1, 0, 1e-3, 1e-6)
    return a


def _solve_altro(prob, opts: ALTROSolverOptions, device: int, max_steps=None, history=None):
    """``solve!(prob, ::ALTROSolverOptions)`` (altro_methods.jl:2-124) through ``tog_solve_altro_ex``: the C
    ABI runs altro_problem (an initial state trajectory -> infeasible_problem, infeasible.jl:2-33; tf = 0 ->
    minimum_time_problem, minimum_time.jl:2-34), the AL solve, projected Newton, process_results! and the
    feasible resolve (csrc/tog_altro.cpp), so the Julia binding and C callers reach the same flow.

    Returns the ``ALTROSolver`` as the reference does (altro_methods.jl:52): ``stats`` (:time, :time_al,
    :time_pn and the AL phase's batch summary), ``solver_al`` (the AL phase's solver on its live device
    buffers, with per-iteration ``traj_stats``), ``solver_pn`` (projected Newton), plus ``stats_feasible``
    (the resolve of an infeasible start, which the reference does not keep). A minimum-time solve's time
    steps go to ``prob.h`` (the reference stores [u; u; h] in prob.U) and ``total_time(prob)`` reads them."""
    lib = abi.load_library()
    infeasible = _altro_infeasible(prob)
    desc = prob.build_desc(tf_min=prob.tf == 0.0)
    a = to_tog_altro_options(opts)
    if max_steps is not None:
        a.max_steps = int(max_steps)
    B, N, n, m = prob.B, prob.N, prob.model.n, prob.model.m
    hcap = 0 if history is False else (int(history) if history not in (None, True) else history_capacity(opts, B))
    x0 = np.ascontiguousarray(prob.x0, dtype=np.float64)
    X = np.ascontiguousarray(prob._X, dtype=np.float64) if infeasible else np.full((B, N, n), np.nan)
    U = np.ascontiguousarray(prob._U, dtype=np.float64)
    h = np.zeros((B, N - 1))
    St = np.zeros((B, abi.NSTATS))
    St_res = np.zeros((B, abi.NSTATS))
    pn = np.zeros((B, abi.PN_NSTATS))
    ocap = a.opts_al.al_iterations + 1
    Hin = np.zeros((B, max(hcap, 1), 3))
    Hout = np.zeros((B, ocap, 4))
    Hcnt = np.zeros((B, 2))
    npn = max(int(a.opts_pn.n_steps), 0) if opts.projected_newton else 0
    Hpn = np.full((B, max(npn, 1), 2), np.nan)
    r = abi.tog_altro_result()
    r.inner_capacity = hcap
    r.keep_handle = 1
    r.stats, r.stats_resolve, r.stats_pn = abi.as_dp(St), abi.as_dp(St_res), abi.as_dp(pn)
    r.hist_inner, r.hist_outer, r.hist_count = abi.as_dp(Hin), abi.as_dp(Hout), abi.as_dp(Hcnt)
    r.hist_pn = abi.as_dp(Hpn) if npn else C.cast(None, C.POINTER(C.c_double))
    abi.check(lib, lib.tog_solve_altro_ex(C.byref(desc.desc), C.byref(a), int(device), abi.as_dp(x0), abi.as_dp(X),
                                          abi.as_dp(U), abi.as_dp(h), C.byref(r)))
    prob._X[...] = X
    prob._U[...] = U
    handle = BatchHandle.adopt(lib, r.handle, a.opts_al)
    handle.hcap = hcap

    def view(cls, o):  # a solver object on the AL phase's handle
        sv = cls.__new__(cls)
        sv.opts, sv.handle, sv.history = o, handle, None
        sv.n, sv.m, sv.N = handle.n, handle.m, handle.N
        return sv

    hist = (Hin[:, :hcap], Hout, Hcnt.astype(np.int64)) if hcap else None
    solver = view(ALTROSolver, opts)
    al = view(AugmentedLagrangianSolver, opts.opts_al)
    al.stats, al.history = stats_dict(St), hist
    solver.solver_al = al
    solver.stats = dict(stats_dict(St))
    solver.stats.update({"time": r.time, "time_al": r.time_al, "time_pn": r.time_pn})
    solver.history = hist
    pnv = view(_PNStatsView, opts.opts_pn)
    pnv.stats = _pn_stats(pn, solver.stats["flags"]) if opts.projected_newton else {}
    pnv.pn_history = (Hpn[:, :npn], pn[:, abi.PN_STEPS].astype(np.int32)) if npn else (np.zeros((B, 0, 2)), np.zeros(B, np.int32))
    solver.solver_pn = pnv
    if prob.tf == 0.0:
        prob.h = h
    if infeasible and opts.resolve_feasible_problem:
        solver.stats_feasible = stats_dict(St_res)
    flags = solver.stats["flags"] | (solver.stats_feasible["flags"] if hasattr(solver, "stats_feasible") else 0)
    _raise_trajectory_errors(flags)
    if opts.projected_newton:
        solver.stats_pn = pnv.stats
        _raise_pn_errors(solver.stats["flags"], solver)
    return solver


def solve_b(prob, solver_or_opts, *, max_steps: int | None = None, device: int = 0, history=None):
    """``solve!(prob, opts)`` / ``solve!(prob, solver)`` (src/solvers.jl:91-94). Mutates
    ``prob.X``/``prob.U`` in place and returns the solver.

    ``history``: record the per-iteration statistics (``solver.traj_stats(b)``): None = on with
    ``history_capacity`` records per trajectory, False = off, an int = that capacity."""
    if isinstance(solver_or_opts, ProjectedNewtonSolver):
        solver_or_opts.handle.upload_state(prob)
        return _solve_pn(prob, solver_or_opts)
    if isinstance(solver_or_opts, AbstractSolver):
        solver = solver_or_opts
        solver.handle.upload_state(prob)
    else:
        opts = solver_or_opts
        if isinstance(opts, ProjectedNewtonSolverOptions):
            return _solve_pn(prob, ProjectedNewtonSolver(prob, opts, device=device))
        if isinstance(opts, ALTROSolverOptions):
            _altro_pn_tolerances(opts)  # (mutates opts.opts_al, as the reference does)
            return _solve_altro(prob, opts, device, max_steps=max_steps, history=history)
        if isinstance(opts, AugmentedLagrangianSolverOptions) and not prob.is_constrained():
            # solve!(prob, ::AugmentedLagrangianSolverOptions) on an unconstrained problem
            # falls back to the unconstrained solver (augmented_lagrangian_methods.jl:33-36)
            opts = opts.opts_uncon
        solver = AbstractSolverFor(prob, opts, device=device)
    mode = solver.mode
    h = solver.handle
    hcap = 0 if history is False else (int(history) if history not in (None, True) else
                                       history_capacity(solver.opts, h.B))
    if hcap != h.hcap:
        h.enable_history(hcap)
    h.solve(mode, max_steps=max_steps if max_steps is not None else _default_max_steps(solver))
    h.download_state(prob)
    solver.stats = h.stats_dict()
    solver.history = h.history()
    _raise_trajectory_errors(solver.stats["flags"])
    return solver


def _default_max_steps(solver):
    """tog_solve_budget: the iteration budget times the line-search rounds an iteration may spread
    over in pending mode, so every trajectory reaches its own iteration limit (MAX_ITERS)."""
    return solver.handle.solve_budget(solver.mode)


def solve(prob, solver_or_opts, **kw):
    """``solve(prob, opts)`` (src/solvers.jl:104-123): returns ``(prob_copy, solver)``."""
    p0 = prob.copy()
    s = solve_b(p0, solver_or_opts, **kw)
    return p0, s
