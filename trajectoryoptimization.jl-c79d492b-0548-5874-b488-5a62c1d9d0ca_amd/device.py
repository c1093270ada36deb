"""``BatchHandle``: one ``tog_handle`` (include/tog.h) = one problem x B trajectories resident in
HBM on one GPU. Thin ctypes plumbing; all compute happens in libtog.so (HIP, gfx950).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class BatchHandle:
    def __init__(self, prob, opts: abi.tog_options, device: int = 0, stream=None, devices=None):
        """``devices``: a list of HIP device ids for one handle over several GPUs
        (tog_create_multi: the batch is split into contiguous slices, one per entry)."""
        self.lib = abi.load_library()
        self.hcap = 0
        self.desc_builder = prob.build_desc()
        self.opts = opts
        h = C.c_void_p()
        if devices is not None:
            devs = np.ascontiguousarray(np.asarray(devices, dtype=np.int32))
            abi.check(self.lib, self.lib.tog_create_multi(C.byref(self.desc_builder.desc), C.byref(opts),
                                                          devs.ctypes.data_as(C.POINTER(C.c_int32)), len(devs),
                                                          C.byref(h)))
        else:
            abi.check(self.lib, self.lib.tog_create(C.byref(self.desc_builder.desc), C.byref(opts), int(device),
                                                    C.byref(h)))
        self.h = h
        dims = (C.c_int64 * 6)()
        abi.check(self.lib, self.lib.tog_dims(self.h, dims))
        self.n, self.m, self.N, self.B, self.pmax, _ = [int(v) for v in dims]
        if stream is not None:
            abi.check(self.lib, self.lib.tog_set_stream(self.h, C.c_void_p(int(stream))))
        self.upload_state(prob)

    @classmethod
    def adopt(cls, lib, handle: int, opts: abi.tog_options):
        """Wrap a ``tog_handle`` created inside libtog (tog_solve_altro_ex's keep_handle): this object
        owns it from now on and destroys it."""
        self = cls.__new__(cls)
        self.lib, self.opts, self.desc_builder, self.hcap = lib, opts, None, 0
        self.h = C.c_void_p(handle)
        dims = (C.c_int64 * 6)()
        abi.check(self.lib, self.lib.tog_dims(self.h, dims))
        self.n, self.m, self.N, self.B, self.pmax, _ = [int(v) for v in dims]
        return self

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and self.h:
                self.lib.tog_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # ------------------------------------------------------------------ shapes per field
    def shape(self, field):
        n, m, N, B, P = self.n, self.m, self.N, self.B, max(self.pmax, 1)
        return {
            abi.FIELD_X: (B, N, n), abi.FIELD_U: (B, N - 1, m), abi.FIELD_XBAR: (B, N, n),
            abi.FIELD_UBAR: (B, N - 1, m), abi.FIELD_K: (B, N - 1, n, m), abi.FIELD_D: (B, N - 1, m),
            abi.FIELD_A: (B, N - 1, n, n), abi.FIELD_B: (B, N - 1, m, n), abi.FIELD_S: (B, N, n, n),
            abi.FIELD_SX: (B, N, n), abi.FIELD_DV: (B, 2), abi.FIELD_LAMBDA: (B, N, P),
            abi.FIELD_MU: (B, N, P), abi.FIELD_C: (B, N, P), abi.FIELD_X0: (B, n),
            abi.FIELD_STATS: (B, abi.NSTATS), abi.FIELD_RHO: (B, 2),
            abi.FIELD_Q: (B, N, n + m + n * n + m * m + m * n),
        }[field]

    def get(self, field, raw=False):
        """Copy a field to the host. Matrices come back as (…, rows, cols) (the raw buffer is
        column-major per block, i.e. the transpose in numpy C order)."""
        out = np.empty(self.shape(field), dtype=np.float64)
        abi.check(self.lib, self.lib.tog_get(self.h, field, abi.as_dp(out)))
        if raw:
            return out
        if field in (abi.FIELD_K, abi.FIELD_A, abi.FIELD_B, abi.FIELD_S):
            return np.ascontiguousarray(np.swapaxes(out, -1, -2))
        return out

    def set(self, field, value):
        v = np.asarray(value, dtype=np.float64)
        if field in (abi.FIELD_K, abi.FIELD_A, abi.FIELD_B, abi.FIELD_S):
            v = np.swapaxes(v, -1, -2)
        v = np.ascontiguousarray(v.reshape(self.shape(field)))
        abi.check(self.lib, self.lib.tog_set(self.h, field, abi.as_dp(v)))

    def device_ptr(self, field) -> int:
        p = C.c_void_p()
        abi.check(self.lib, self.lib.tog_get_device_ptr(self.h, field, C.byref(p)))
        return int(p.value or 0)

    # ------------------------------------------------------------------ state
    def upload_state(self, prob):
        x0 = np.ascontiguousarray(prob.x0, dtype=np.float64)
        U = np.ascontiguousarray(prob._U, dtype=np.float64)
        X = np.ascontiguousarray(prob._X, dtype=np.float64)
        Xp = abi.as_dp(X) if np.isfinite(X).all() else C.cast(None, C.POINTER(C.c_double))
        if not np.isfinite(X).all() and not np.isnan(X).all():
            # a partially finite X0: upload as given (rollout!(prob) will trigger on the NaNs)
            Xp = abi.as_dp(X)
        abi.check(self.lib, self.lib.tog_set_state(self.h, abi.as_dp(x0), abi.as_dp(U), Xp))

    def download_state(self, prob):
        prob._X[...] = self.get(abi.FIELD_X)
        prob._U[...] = self.get(abi.FIELD_U)

    # ------------------------------------------------------------------ step level
    def rollout_open_loop(self):
        abi.check(self.lib, self.lib.tog_rollout_open_loop(self.h))

    def slack_controls(self):
        """``slack_controls(prob)`` into U[m+1:m+n] (infeasible handles, infeasible.jl:63-80)."""
        abi.check(self.lib, self.lib.tog_slack_controls(self.h))

    def cost_expansion(self, sqrt=False, al=False):
        """``cost_expansion!`` into FIELD_Q (ilqr_methods.jl:55-62)."""
        abi.check(self.lib, self.lib.tog_cost_expansion(self.h, int(sqrt), int(al)))

    def jacobians(self):
        abi.check(self.lib, self.lib.tog_jacobians(self.h))

    def update_constraints(self):
        abi.check(self.lib, self.lib.tog_update_constraints(self.h))

    def cost(self, al=False):
        J = np.empty(self.B)
        abi.check(self.lib, self.lib.tog_cost(self.h, int(al), abi.as_dp(J)))
        return J

    def backward_pass(self, sqrt=False, al=False, store_S=False):
        dV = np.empty((self.B, 2))
        abi.check(self.lib, self.lib.tog_backward_pass(self.h, int(sqrt), int(al),
                                                       abi.BP_STORE_S if store_S else 0, abi.as_dp(dV)))
        return dV

    def forward_pass(self, J_prev, al=False):
        Jp = np.ascontiguousarray(np.broadcast_to(np.asarray(J_prev, dtype=np.float64), (self.B,)))
        J = np.empty(self.B)
        abi.check(self.lib, self.lib.tog_forward_pass(self.h, int(al), abi.as_dp(Jp), abi.as_dp(J)))
        return J

    def rollout(self, alpha=1.0):
        ok = np.empty(self.B, dtype=np.int32)
        abi.check(self.lib, self.lib.tog_rollout(self.h, float(alpha), ok.ctypes.data_as(C.POINTER(C.c_int32))))
        return ok.astype(bool)

    # ------------------------------------------------------------------ solve level
    def solve_init(self, mode):
        abi.check(self.lib, self.lib.tog_solve_init(self.h, int(mode)))

    def solve_step(self, nsteps=1):
        abi.check(self.lib, self.lib.tog_solve_step(self.h, int(nsteps)))

    def solve_budget(self, mode):
        """tog_solve_budget: default batch-step budget of a solve to completion."""
        rc = self.lib.tog_solve_budget(self.h, int(mode))
        if rc <= 0:
            abi.check(self.lib, rc)
        return int(rc)

    def solve(self, mode, max_steps=None):
        """tog_solve; max_steps None/0: the tog_solve_budget default"""
        abi.check(self.lib, self.lib.tog_solve(self.h, int(mode), int(max_steps or 0)))

    def solve_pn(self, pn_opts: abi.tog_pn_options):
        """tog_solve_pn: returns the (B, PN_NSTATS) statistics rows."""
        out = np.zeros((self.B, abi.PN_NSTATS))
        abi.check(self.lib, self.lib.tog_solve_pn(self.h, C.byref(pn_opts), abi.as_dp(out)))
        return out

    def batch_stats(self):
        out = np.empty(3)
        abi.check(self.lib, self.lib.tog_batch_stats(self.h, abi.as_dp(out)))
        return out

    def batch_stats_begin(self):
        """tog_batch_stats_begin: enqueue the stopping check (no host wait)."""
        abi.check(self.lib, self.lib.tog_batch_stats_begin(self.h))

    def batch_stats_end(self):
        """tog_batch_stats_end: wait for the enqueued check only; [n_active, Σ J, max c_max]."""
        out = np.empty(3)
        abi.check(self.lib, self.lib.tog_batch_stats_end(self.h, abi.as_dp(out)))
        return out

    def total_steps(self):
        v = C.c_int64()
        abi.check(self.lib, self.lib.tog_total_steps(self.h, C.byref(v)))
        return int(v.value)

    def profile(self, enable: bool):
        abi.check(self.lib, self.lib.tog_profile(self.h, int(bool(enable))))

    def profile_read(self):
        ms = np.zeros(abi.NKERNELS)
        cnt = (C.c_int64 * abi.NKERNELS)()
        abi.check(self.lib, self.lib.tog_profile_read(self.h, abi.as_dp(ms), cnt))
        return ms, np.array(list(cnt), dtype=np.int64)

    def synchronize(self):
        abi.check(self.lib, self.lib.tog_synchronize(self.h))

    def status(self):
        f = np.empty(self.B, dtype=np.int32)
        abi.check(self.lib, self.lib.tog_status(self.h, f.ctypes.data_as(C.POINTER(C.c_int32))))
        return f

    def stats_dict(self):
        return stats_dict(self.get(abi.FIELD_STATS))

    # ------------------------------------------------------------------ iteration histories
    def enable_history(self, capacity: int):
        """tog_history_enable: keep `capacity` inner records per trajectory (0: off)."""
        abi.check(self.lib, self.lib.tog_history_enable(self.h, int(capacity)))
        self.hcap = int(capacity)

    def history(self):
        """(inner (B, cap, 3) [cost, dJ, gradient], outer (B, al_iterations + 1, 4) [iterations_inner, cost,
        c_max, penalty_max], counts (B, 2) records written [inner, outer]) of the solve since
        tog_solve_init; None when recording is off."""
        if not self.hcap:
            return None
        inner = np.empty((self.B, self.hcap, 3))
        abi.check(self.lib, self.lib.tog_get(self.h, abi.FIELD_HIST_INNER, abi.as_dp(inner)))
        ocap = self.opts.al_iterations + 1
        outer = np.empty((self.B, ocap, 4))
        abi.check(self.lib, self.lib.tog_get(self.h, abi.FIELD_HIST_OUTER, abi.as_dp(outer)))
        cnt = np.empty((self.B, 2))
        abi.check(self.lib, self.lib.tog_get(self.h, abi.FIELD_HIST_COUNT, abi.as_dp(cnt)))
        return inner, outer, cnt.astype(np.int64)

    def pn_history(self, n_steps: int):
        """solver_pn.stats [:cost, :c_max] per newton step (B, n_steps, 2) and records per trajectory (B,)."""
        out = np.empty((self.B, max(int(n_steps), 0), 2))
        rec = np.zeros(self.B, dtype=np.int32)
        abi.check(self.lib, self.lib.tog_get_pn_history(self.h, abi.as_dp(out), rec.ctypes.data_as(C.POINTER(C.c_int32))))
        return out, rec


def stats_dict(S):
    """solver.stats from the (B, TOG_NSTATS) statistics rows (TOG_FIELD_STATS)."""
    return {
        "cost": S[:, abi.STAT_J], "dJ": S[:, abi.STAT_DJ], "gradient": S[:, abi.STAT_GRADIENT],
        "iterations": S[:, abi.STAT_ITERATIONS].astype(np.int64),
        "dJ_zero_counter": S[:, abi.STAT_ZERO_COUNT].astype(np.int64),
        "alpha": S[:, abi.STAT_ALPHA], "c_max": S[:, abi.STAT_C_MAX],
        "iterations_outer": S[:, abi.STAT_AL_ITER].astype(np.int64),
        "iterations_total": S[:, abi.STAT_TOTAL_STEPS].astype(np.int64),
        "penalty_max": S[:, abi.STAT_PENALTY_MAX],
        "flags": S[:, abi.STAT_FLAGS].astype(np.int64),
    }


def ilqr_traj_stats(inner, n_rec, zero_counter=None):
    """One inner solve's ``solver.stats`` as iLQRSolver's record_iteration! builds it (ilqr_methods.jl:77-89):
    :iterations, and the :cost, :dJ, :gradient vectors; `inner` holds its records."""
    d = {"iterations": int(n_rec), "cost": inner[:n_rec, 0].copy(), "dJ": inner[:n_rec, 1].copy(),
         "gradient": inner[:n_rec, 2].copy()}
    if zero_counter is None:  # dJ == 0 counts consecutive records (the counter's value after the last one)
        z = 0
        for v in d["dJ"]:
            z = z + 1 if v == 0.0 else 0
        zero_counter = z
    d["dJ_zero_counter"] = int(zero_counter)
    return d


def al_traj_stats(inner, n_in, outer, n_out):
    """AugmentedLagrangianSolver.stats of one trajectory (augmented_lagrangian_methods.jl:79-97):
    :iterations, :iterations_total, the :iterations_inner, :cost, :c_max, :penalty_max vectors, and
    stats_uncon (the inner solver's stats at every outer record; the first is the reset solver's). The
    inner records are split by :iterations_inner; records past the history's capacity are absent, so a
    truncated history leaves the later inner solves short."""
    it_in = outer[:n_out, 0].astype(np.int64)
    d = {"iterations": int(n_out), "iterations_total": int(it_in.sum()), "iterations_inner": it_in,
         "cost": outer[:n_out, 1].copy(), "c_max": outer[:n_out, 2].copy(), "penalty_max": outer[:n_out, 3].copy()}
    inner = inner[:min(int(n_in), inner.shape[0])]
    uncon, o = [], 0
    for k in it_in:
        sl = inner[o:o + int(k)]
        uncon.append(ilqr_traj_stats(sl, len(sl)))
        o += int(k)
    d["stats_uncon"] = uncon
    d["truncated"] = bool(n_in > inner.shape[0])
    return d

