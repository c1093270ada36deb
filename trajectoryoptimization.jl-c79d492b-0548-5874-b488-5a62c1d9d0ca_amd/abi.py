"""ctypes mirror of ``include/tog.h`` (the C ABI of the HIP hot path) and the loader of
``libtog.so``.

No torch types cross this boundary: plain fp64 column-major buffers, int32/int64 sizes,
int status codes. The library is built in-tree (``csrc/``) by ``__graft_entry__.build()``;
loading fails loudly when it is missing -- there is no CPU fallback in the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "csrc" / "libtog.so"

TOG_ABI_VERSION = 4

# models (include/tog.h tog_model_id)
MODEL_DOUBLE_INTEGRATOR, MODEL_CARTPOLE, MODEL_QUADROTOR, MODEL_CAR, MODEL_PENDULUM, MODEL_KUKA = range(6)
MODEL_NM = {0: (2, 1), 1: (4, 1), 2: (13, 4), 3: (3, 2), 4: (2, 1), 5: (14, 7)}
MODEL_USER = 100  # Model(f!, n, m) from a plugin (tog_model_load)
# status codes (include/tog.h tog_status_code)
OK, ERR_ARG, ERR_DEVICE, ERR_NOMEM, ERR_UNSUPPORTED = 0, -1, -2, -3, -4

RK3, RK4, MIDPOINT, RK3_IMPLICIT, MIDPOINT_IMPLICIT = 0, 1, 2, 3, 4
CON_BOUND, CON_GOAL, CON_CIRCLES, CON_SPHERES, CON_INFEASIBLE, CON_USER, CON_MIN_TIME_EQ = range(7)
PROB_INFEASIBLE = 1  # tog_problem_flag
PROB_MIN_TIME = 2
PROB_TF_MIN = 4  # tf = 0: tog_solve_altro solves minimum_time_problem
MODE_ILQR, MODE_AL = 0, 1

(FIELD_X, FIELD_U, FIELD_XBAR, FIELD_UBAR, FIELD_K, FIELD_D, FIELD_A, FIELD_B, FIELD_S, FIELD_SX,
 FIELD_DV, FIELD_LAMBDA, FIELD_MU, FIELD_C, FIELD_X0, FIELD_STATS, FIELD_RHO, FIELD_Q) = range(18)
# iteration histories (tog_history_enable): (3,cap,B) inner records, (4,al_iterations+1,B) outer, (2,B) counts
FIELD_HIST_INNER, FIELD_HIST_OUTER, FIELD_HIST_COUNT = 18, 19, 20

(STAT_J, STAT_DJ, STAT_GRADIENT, STAT_ITERATIONS, STAT_ZERO_COUNT, STAT_ALPHA, STAT_Z, STAT_C_MAX,
 STAT_AL_ITER, STAT_TOTAL_STEPS, STAT_LS_TRIALS, STAT_BP_RESTARTS, STAT_FLAGS, STAT_PENALTY_MAX) = range(14)
NSTATS = 14

TRAJ_ACTIVE = 1 << 0
TRAJ_CONVERGED = 1 << 1
TRAJ_MAX_ITERS = 1 << 2
TRAJ_COST_INCREASED = 1 << 3
TRAJ_COST_BLOWUP = 1 << 4
TRAJ_MAX_REG = 1 << 5
TRAJ_SQRT_PD_FAIL = 1 << 6
TRAJ_AL_CONVERGED = 1 << 7
TRAJ_AL_MAX_ITERS = 1 << 8
TRAJ_SINGULAR = 1 << 9
TRAJ_BP_ABORTED = 1 << 10
TRAJ_PN_ERROR = 1 << 11
TRAJ_PN_BLOCK = 1 << 12  # a projected Newton block outgrew the device's 64 rows (TOG_TRAJ_PN_BLOCK)

# projected Newton statistics row (tog_pn_stat)
PN_VIOL, PN_C_MAX, PN_J, PN_PROJECTIONS, PN_LINESEARCHES, PN_REFINEMENTS, PN_STEPS = range(7)
PN_NSTATS = 7
BP_MAX_RESTARTS = 1000  # TOG_BP_MAX_RESTARTS

BP_STORE_S = 1

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class tog_constraint(C.Structure):
    _fields_ = [("type", C.c_int32), ("count", C.c_int32), ("data", _dp)]


class tog_constraint_set(C.Structure):
    _fields_ = [("n_con", C.c_int32), ("con", C.POINTER(tog_constraint))]


class tog_problem_desc(C.Structure):
    _fields_ = [
        ("model", C.c_int32), ("integrator", C.c_int32), ("n", C.c_int32), ("m", C.c_int32),
        ("N", C.c_int32), ("flags", C.c_int32), ("batch", C.c_int64), ("dt", C.c_double),
        ("Q", _dp), ("R", _dp), ("H", _dp), ("q", _dp), ("r", _dp), ("c", C.c_double),
        ("Qf", _dp), ("qf", _dp), ("cf", C.c_double),
        ("n_sets", C.c_int32), ("reserved1", C.c_int32),
        ("sets", C.POINTER(tog_constraint_set)), ("knot_set", _ip),
        ("user_model", C.c_void_p), ("R_min_time", C.c_double), ("stage_costs", _dp),
    ]


class tog_options(C.Structure):
    _fields_ = [
        ("cost_tolerance", C.c_double), ("gradient_norm_tolerance", C.c_double),
        ("iterations", C.c_int32), ("dJ_counter_limit", C.c_int32), ("square_root", C.c_int32),
        ("bp_reg_type", C.c_int32), ("gradient_type", C.c_int32), ("iterations_linesearch", C.c_int32),
        ("line_search_lower_bound", C.c_double), ("line_search_upper_bound", C.c_double),
        ("bp_reg_increase_factor", C.c_double), ("bp_reg_max", C.c_double), ("bp_reg_min", C.c_double),
        ("bp_reg_fp", C.c_double), ("max_cost_value", C.c_double), ("max_state_value", C.c_double),
        ("max_control_value", C.c_double),
        ("al_cost_tolerance", C.c_double), ("al_cost_tolerance_intermediate", C.c_double),
        ("al_gradient_norm_tolerance", C.c_double), ("al_gradient_norm_tolerance_intermediate", C.c_double),
        ("constraint_tolerance", C.c_double), ("dual_min", C.c_double), ("dual_max", C.c_double),
        ("penalty_max", C.c_double), ("penalty_initial", C.c_double), ("penalty_scaling", C.c_double),
        ("al_iterations", C.c_int32), ("kickout_max_penalty", C.c_int32),
    ]


class tog_pn_options(C.Structure):
    """ProjectedNewtonSolverOptions (src/solvers/direct/direct_solvers.jl:14-30)."""
    _fields_ = [("n_steps", C.c_int32), ("solve_type", C.c_int32), ("active_set_tolerance", C.c_double),
                ("feasibility_tolerance", C.c_double)]


class tog_altro_options(C.Structure):
    """ALTROSolverOptions (src/solvers/altro/altro_solver.jl:6-65), the live fields."""
    _fields_ = [("opts_al", tog_options), ("R_inf", C.c_double), ("R_minimum_time", C.c_double),
                ("dt_max", C.c_double), ("dt_min", C.c_double), ("projected_newton_tolerance", C.c_double),
                ("dynamically_feasible_projection", C.c_int32), ("resolve_feasible_problem", C.c_int32),
                ("projected_newton", C.c_int32), ("max_steps", C.c_int32), ("opts_pn", tog_pn_options)]


class tog_altro_result(C.Structure):
    """What solve!(prob, ALTROSolverOptions) returns (include/tog.h tog_altro_result)."""
    _fields_ = [("inner_capacity", C.c_int32), ("keep_handle", C.c_int32),
                ("stats", _dp), ("stats_resolve", _dp), ("stats_pn", _dp),
                ("hist_inner", _dp), ("hist_outer", _dp), ("hist_count", _dp), ("hist_pn", _dp),
                ("time", C.c_double), ("time_al", C.c_double), ("time_pn", C.c_double),
                ("handle", C.c_void_p)]


def default_options() -> tog_options:
    """Reference defaults (ilqr_solver.jl:7-81, augmented_lagrangian_solver.jl:8-66)."""
    o = tog_options()
    o.cost_tolerance = 1e-4
    o.gradient_norm_tolerance = 1e-5
    o.iterations = 300
    o.dJ_counter_limit = 10
    o.square_root = 0
    o.bp_reg_type = 0
    o.gradient_type = 0
    o.iterations_linesearch = 20
    o.line_search_lower_bound = 1e-8
    o.line_search_upper_bound = 10.0
    o.bp_reg_increase_factor = 1.6
    o.bp_reg_max = 1e8
    o.bp_reg_min = 1e-8
    o.bp_reg_fp = 10.0
    o.max_cost_value = 1e8
    o.max_state_value = 1e8
    o.max_control_value = 1e8
    o.al_cost_tolerance = 1e-4
    o.al_cost_tolerance_intermediate = 1e-3
    o.al_gradient_norm_tolerance = 1e-5
    o.al_gradient_norm_tolerance_intermediate = 1e-5
    o.constraint_tolerance = 1e-3
    o.dual_min = -1e8
    o.dual_max = 1e8
    o.penalty_max = 1e8
    o.penalty_initial = 1.0
    o.penalty_scaling = 10.0
    o.al_iterations = 30
    o.kickout_max_penalty = 0
    return o


def as_dp(a: np.ndarray):
    if not (a.dtype == np.float64 and (a.flags["F_CONTIGUOUS"] or a.flags["C_CONTIGUOUS"])):
        raise TypeError(f"C ABI buffers must be contiguous float64 arrays, got {a.dtype} "
                        f"(C={a.flags['C_CONTIGUOUS']}, F={a.flags['F_CONTIGUOUS']})")
    return a.ctypes.data_as(_dp)


class DescBuilder:
    """Builds a ``tog_problem_desc`` and keeps every backing numpy array alive.

    ``sets`` is a list of ordered constraint sets; each set is a list of
    ``(type, count, data ndarray)``; ``knot_set`` has N entries (-1 = none).
    """

    def __init__(self, model, integrator, n, m, N, dt, Q, R, H, q, r, c, Qf, qf, cf, sets, knot_set,
                 batch=1, flags=0, user_model=None, R_min_time=0.0, stage_costs=None):
        """``stage_costs``: None, or the per-stage-knot table (N-1, nc) of a time-varying objective, each
        row [Q; R; H; q; r; c] with the matrices column-major (tog_problem_desc.stage_costs)."""
        self._keep = []

        def arr(x, shape):
            a = np.asfortranarray(np.asarray(x, dtype=np.float64).reshape(shape, order="F"))
            self._keep.append(a)
            return a

        d = tog_problem_desc()
        d.model, d.integrator, d.n, d.m, d.N = int(model), int(integrator), int(n), int(m), int(N)
        d.batch = int(batch)
        d.flags = int(flags)
        d.dt = float(dt)
        d.Q = as_dp(arr(Q, (n, n)))
        d.R = as_dp(arr(R, (m, m)))
        d.H = as_dp(arr(H, (m, n)))
        d.q = as_dp(arr(q, (n,)))
        d.r = as_dp(arr(r, (m,)))
        d.c = float(c)
        d.Qf = as_dp(arr(Qf, (n, n)))
        d.qf = as_dp(arr(qf, (n,)))
        d.cf = float(cf)
        cs_arr = (tog_constraint_set * max(1, len(sets)))()
        for i, s in enumerate(sets):
            carr = (tog_constraint * max(1, len(s)))()
            for j, (t, cnt, data) in enumerate(s):
                da = np.ascontiguousarray(np.asarray(data, dtype=np.float64).ravel())
                self._keep.append(da)
                carr[j].type = int(t)
                carr[j].count = int(cnt)
                carr[j].data = da.ctypes.data_as(_dp)
            self._keep.append(carr)
            cs_arr[i].n_con = len(s)
            cs_arr[i].con = carr
        self._keep.append(cs_arr)
        d.n_sets = len(sets)
        d.sets = cs_arr
        ks = np.ascontiguousarray(np.asarray(knot_set, dtype=np.int32))
        assert ks.shape == (N,)
        self._keep.append(ks)
        d.knot_set = ks.ctypes.data_as(_ip)
        d.user_model = user_model
        d.R_min_time = float(R_min_time)
        if stage_costs is not None:
            sc = np.ascontiguousarray(np.asarray(stage_costs, dtype=np.float64))
            if sc.shape != (N - 1, n * n + m * m + m * n + n + m + 1):
                raise ValueError("stage_costs must be (N-1, n*n + m*m + m*n + n + m + 1)")
            self._keep.append(sc)
            d.stage_costs = sc.ctypes.data_as(_dp)
        self.desc = d


def header_hash() -> str:
    """sha1 of the text of libtog's headers (csrc/Makefile HDRS, same files, same order), first 15
    hex digits: the TOG_HEADER_HASH libtog was built with. Plugins generated at run time are compiled
    with it and cached under it, so a header change rebuilds them, and the fingerprint check in
    tog_model_load / tog_generic_cost_load refuses a stale one."""
    import hashlib
    import re

    csrc = PKG_DIR / "csrc"
    mk = (csrc / "Makefile").read_text()
    hdrs = re.search(r"^HDRS = (.*)$", mk, re.M).group(1).split()
    h = hashlib.sha1()
    for f in hdrs:
        h.update((csrc / f).read_bytes())
    return h.hexdigest()[:15]


_LIB = None


def load_library(path: os.PathLike | None = None):
    """Load libtog.so (HIP). Raises if it has not been built -- no fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    if path is None and os.environ.get("TOG_LIBRARY"):  # A/B builds (e.g. tools/ab_build.sh)
        path = os.environ["TOG_LIBRARY"]
    p = pathlib.Path(path) if path else LIB_PATH
    if not p.exists():
        raise RuntimeError(f"libtog.so not found at {p}: run __graft_entry__.build() (hipcc, gfx950)")
    lib = C.CDLL(str(p))
    vp = C.c_void_p
    lib.tog_version.restype = C.c_int32
    lib.tog_device_count.restype = C.c_int32
    lib.tog_default_options.argtypes = [C.POINTER(tog_options)]
    lib.tog_create.argtypes = [C.POINTER(tog_problem_desc), C.POINTER(tog_options), C.c_int32, C.POINTER(vp)]
    lib.tog_create_multi.argtypes = [C.POINTER(tog_problem_desc), C.POINTER(tog_options), _ip, C.c_int32,
                                     C.POINTER(vp)]
    lib.tog_destroy.argtypes = [vp]
    lib.tog_set_stream.argtypes = [vp, vp]
    lib.tog_synchronize.argtypes = [vp]
    lib.tog_set_state.argtypes = [vp, _dp, _dp, _dp]
    lib.tog_set.argtypes = [vp, C.c_int32, _dp]
    lib.tog_get.argtypes = [vp, C.c_int32, _dp]
    lib.tog_get_device_ptr.argtypes = [vp, C.c_int32, C.POINTER(vp)]
    lib.tog_dims.argtypes = [vp, C.POINTER(C.c_int64)]
    lib.tog_rollout_open_loop.argtypes = [vp]
    lib.tog_jacobians.argtypes = [vp]
    lib.tog_update_constraints.argtypes = [vp]
    lib.tog_cost.argtypes = [vp, C.c_int32, _dp]
    lib.tog_backward_pass.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, _dp]
    lib.tog_forward_pass.argtypes = [vp, C.c_int32, _dp, _dp]
    lib.tog_rollout.argtypes = [vp, C.c_double, _ip]
    lib.tog_solve_init.argtypes = [vp, C.c_int32]
    lib.tog_solve_step.argtypes = [vp, C.c_int32]
    lib.tog_batch_stats.argtypes = [vp, _dp]
    lib.tog_batch_stats_device.argtypes = [vp, vp]
    lib.tog_total_steps.argtypes = [vp, C.POINTER(C.c_int64)]
    lib.tog_solve.argtypes = [vp, C.c_int32, C.c_int32]
    lib.tog_solve_budget.argtypes = [vp, C.c_int32]
    lib.tog_status.argtypes = [vp, _ip]
    lib.tog_profile.argtypes = [vp, C.c_int32]
    lib.tog_profile_read.argtypes = [vp, _dp, C.POINTER(C.c_int64)]
    lib.tog_last_error.restype = C.c_char_p
    lib.tog_dynamics_bias.argtypes = [C.c_int32, _dp, _dp]
    lib.tog_slack_controls.argtypes = [vp]
    lib.tog_cost_expansion.argtypes = [vp, C.c_int32, C.c_int32]
    lib.tog_solve_ilqr.argtypes = [vp]
    lib.tog_solve_al.argtypes = [vp]
    lib.tog_default_pn_options.argtypes = [C.POINTER(tog_pn_options)]
    lib.tog_solve_pn.argtypes = [vp, C.POINTER(tog_pn_options), _dp]
    lib.tog_default_altro_options.argtypes = [C.POINTER(tog_altro_options)]
    lib.tog_solve_altro.argtypes = [C.POINTER(tog_problem_desc), C.POINTER(tog_altro_options), C.c_int32, _dp, _dp,
                                    _dp, _dp, _dp, _dp, _dp]
    lib.tog_solve_altro_ex.argtypes = [C.POINTER(tog_problem_desc), C.POINTER(tog_altro_options), C.c_int32, _dp,
                                       _dp, _dp, _dp, C.POINTER(tog_altro_result)]
    lib.tog_history_enable.argtypes = [vp, C.c_int32]
    lib.tog_batch_stats_begin.argtypes = [vp]
    lib.tog_batch_stats_end.argtypes = [vp, _dp]
    lib.tog_get_pn_history.argtypes = [vp, _dp, _ip]
    lib.tog_model_load.argtypes = [C.c_char_p, C.POINTER(vp)]
    lib.tog_model_dims.argtypes = [vp, _ip, _ip]
    lib.tog_model_free.argtypes = [vp]
    lib.tog_generic_cost_load.argtypes = [C.c_char_p, C.POINTER(vp)]
    lib.tog_generic_cost_dims.argtypes = [vp, _ip, _ip]
    lib.tog_generic_cost_expand.argtypes = [vp, C.c_int32, C.c_int32, _dp, _dp, C.c_int64] + [_dp] * 6
    lib.tog_generic_cost_expand_device.argtypes = [vp, C.c_int32, vp, vp, C.c_int64] + [vp] * 6 + [vp]
    lib.tog_generic_cost_free.argtypes = [vp]
    for name in ("tog_create", "tog_create_multi", "tog_destroy", "tog_set_stream", "tog_synchronize", "tog_set_state",
                 "tog_set", "tog_get", "tog_get_device_ptr", "tog_dims", "tog_rollout_open_loop",
                 "tog_jacobians", "tog_update_constraints", "tog_cost", "tog_backward_pass",
                 "tog_forward_pass", "tog_rollout", "tog_solve_init", "tog_solve_step", "tog_batch_stats",
                 "tog_batch_stats_device", "tog_total_steps", "tog_solve", "tog_solve_budget", "tog_status",
                 "tog_profile", "tog_profile_read", "tog_dynamics_bias", "tog_slack_controls", "tog_cost_expansion",
                 "tog_solve_ilqr", "tog_solve_al", "tog_solve_pn", "tog_model_load", "tog_model_dims",
                 "tog_model_free", "tog_generic_cost_load", "tog_generic_cost_dims", "tog_generic_cost_expand", "tog_generic_cost_expand_device",
                 "tog_generic_cost_free", "tog_solve_altro", "tog_solve_altro_ex", "tog_history_enable",
                 "tog_get_pn_history", "tog_batch_stats_begin", "tog_batch_stats_end"):
        getattr(lib, name).restype = C.c_int32
    if lib.tog_version() != TOG_ABI_VERSION:
        raise RuntimeError("libtog ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


EXPORTED_SYMBOLS = (
    "tog_version", "tog_device_count", "tog_default_options", "tog_create", "tog_create_multi", "tog_destroy",
    "tog_set_stream",
    "tog_synchronize", "tog_set_state", "tog_set", "tog_get", "tog_get_device_ptr", "tog_dims",
    "tog_rollout_open_loop", "tog_jacobians", "tog_update_constraints", "tog_cost", "tog_backward_pass",
    "tog_forward_pass", "tog_rollout", "tog_solve_init", "tog_solve_step", "tog_batch_stats",
    "tog_batch_stats_device", "tog_total_steps", "tog_solve", "tog_solve_budget", "tog_status", "tog_profile",
    "tog_profile_read", "tog_last_error", "tog_dynamics_bias", "tog_slack_controls", "tog_cost_expansion", "tog_solve_ilqr",
    "tog_solve_al", "tog_default_pn_options", "tog_solve_pn", "tog_model_load", "tog_model_dims", "tog_model_free",
    "tog_generic_cost_load", "tog_generic_cost_dims", "tog_generic_cost_expand", "tog_generic_cost_expand_device", "tog_generic_cost_free",
    "tog_default_altro_options", "tog_solve_altro", "tog_solve_altro_ex", "tog_history_enable", "tog_get_pn_history",
    "tog_batch_stats_begin", "tog_batch_stats_end",
)
KERNEL_JACOBIAN, KERNEL_BACKWARD, KERNEL_FORWARD, KERNEL_EXPANSION = 0, 1, 2, 3
NKERNELS = 4


def check(lib, rc):
    if rc != 0:
        msg = lib.tog_last_error()
        raise RuntimeError(f"libtog error {rc}: {msg.decode() if msg else ''}")
    return rc
