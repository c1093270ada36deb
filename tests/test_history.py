"""Iteration histories: the reference's solver.stats vectors behind the C ABI.

iLQR record_iteration! (src/solvers/ilqr/ilqr_methods.jl:77-89) pushes [:cost, :dJ, :gradient] once per
inner record; AL record_iteration! (src/solvers/augmented_lagrangian/augmented_lagrangian_methods.jl:79-97)
pushes [:iterations_inner, :cost, :c_max, :penalty_max] per outer record; projected Newton's
(src/solvers/direct/projected_newton.jl:23-29) [:cost, :c_max] per newton step. The device records them as
the solve runs (tog_history_enable, TOG_FIELD_HIST_*); the oracle (oracle/tog_oracle.c record_iteration /
record_outer) records the same values in the same order, so device and oracle histories are compared bit
for bit (projected Newton's to the PN tolerance of tests/test_projected_newton.py).
"""
import numpy as np
import pytest

from test_projected_newton import car_al_opts, car_batch

TOL_PN = 1e-13


def _oracle_hist(oracle, prob, opts, b):
    o = oracle.OracleSolver(prob, opts, b=b)
    o.solve()
    return o, o.history()


def _check_al(tog, solver, oracle, prob, opts, b):
    st = solver.traj_stats(b)
    o, (hin, hout, _) = _oracle_hist(oracle, prob, opts, b)
    assert not st["truncated"]
    assert st["iterations"] == len(hout), (b, st["iterations"], len(hout))
    assert np.array_equal(st["iterations_inner"], hout[:, 0].astype(np.int64)), b
    for key, col in (("cost", 1), ("c_max", 2), ("penalty_max", 3)):
        assert np.array_equal(st[key], hout[:, col], equal_nan=True), (b, key, st[key], hout[:, col])
    # the inner solves, concatenated in order
    inner = np.concatenate([np.stack([u["cost"], u["dJ"], u["gradient"]], axis=1) for u in st["stats_uncon"]])
    assert inner.shape == hin[:len(inner)].shape
    assert np.array_equal(inner, hin[:len(inner)], equal_nan=True), b
    assert st["stats_uncon"][0]["iterations"] == 0  # the reset inner solver's stats at the initial record
    # the summary row agrees with the vectors: every completed inner solve records its step!s + 1
    assert st["iterations_total"] == int(solver.stats["iterations_total"][b]) + st["iterations"] - 1
    assert st["c_max"][-1] == solver.stats["c_max"][b]
    return st


# ----------------------------------------------------------------------------- CPU: host logic


def test_traj_stats_split(tog):
    """al_traj_stats splits the inner records by :iterations_inner into stats_uncon (ilqr_traj_stats)."""
    inner = np.array([[10.0, np.inf, 0.5], [9.0, 1.0, 0.4], [9.0, 0.0, 0.3], [8.0, np.inf, 0.2], [7.0, 1.0, 0.1]])
    outer = np.array([[0, 11.0, 0.5, 1.0], [3, 9.0, 0.1, 10.0], [2, 7.0, 1e-4, 100.0]])
    d = tog.device.al_traj_stats(inner, 5, outer, 3)
    assert d["iterations"] == 3 and d["iterations_total"] == 5
    assert [u["iterations"] for u in d["stats_uncon"]] == [0, 3, 2]
    assert np.array_equal(d["stats_uncon"][1]["cost"], [10.0, 9.0, 9.0])
    assert d["stats_uncon"][1]["dJ_zero_counter"] == 1 and d["stats_uncon"][2]["dJ_zero_counter"] == 0
    assert np.array_equal(d["c_max"], [0.5, 0.1, 1e-4]) and not d["truncated"]
    assert tog.device.al_traj_stats(inner[:2], 5, outer, 3)["truncated"]


def test_history_capacity(tog):
    """A whole AL solve fits (al_iterations x (iterations + 1) + 1) for small batches; large batches are
    capped at the HBM budget."""
    al = tog.AugmentedLagrangianSolverOptions()
    assert tog.solvers.history_capacity(al, 4) == 30 * 301 + 1
    assert tog.solvers.history_capacity(tog.iLQRSolverOptions(), 4) == 302
    assert tog.solvers.history_capacity(al, 8192) == int(256e6 // (24 * 8192))


def test_oracle_history_records(tog, oracle):
    """The oracle's histories have the reference's shape: one inner record per stats[:iterations], the
    first of each inner solve with dJ = Inf, outer records = AL stats[:iterations]."""
    prob, opts = tog.Problems.config_quadrotor(B=1)
    opts.iterations = 3
    o, (hin, hout, hpn) = _oracle_hist(oracle, prob, opts, 0)
    assert len(hout) == int(o.get("stats")[tog.abi.STAT_AL_ITER]) + 1
    assert hout[0, 0] == 0 and hout[0, 3] == opts.penalty_initial
    assert int(hout[:, 0].sum()) <= len(hin)
    starts = np.cumsum(np.concatenate([[0], hout[1:, 0]]))[:-1].astype(int)
    assert np.all(np.isinf(hin[starts, 1]))
    assert len(hpn) == 0


def test_altro_max_steps_reaches_the_abi(tog):
    """solve_b(..., max_steps) with ALTROSolverOptions fills tog_altro_options.max_steps."""
    opts = tog.ALTROSolverOptions()
    a = tog.solvers.to_tog_altro_options(opts)
    assert a.max_steps == 0


# ----------------------------------------------------------------------------- GPU: device vs oracle


@pytest.mark.gpu
def test_history_config3_equals_oracle(tog, oracle, gpu):
    """Config 3 (AL, square-root BP), B = 4: every inner and outer record of each trajectory equals the
    oracle's bit for bit."""
    prob, opts = tog.Problems.config_quadrotor(B=4)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    assert solver.history is not None
    for b in range(prob.B):
        _check_al(tog, solver, oracle, prob, opts, b)


@pytest.mark.gpu
def test_history_ilqr_cartpole_equals_oracle(tog, oracle, gpu):
    """Unconstrained iLQR (config 2): the inner records (cost, dJ, gradient), the first (J0, Inf, ·)."""
    prob, opts = tog.Problems.config_cartpole(B=3)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        st = solver.traj_stats(b)
        o, (hin, hout, _) = _oracle_hist(oracle, prob, opts, b)
        assert st["iterations"] == len(hin) == int(solver.stats["iterations"][b])
        got = np.stack([st["cost"], st["dJ"], st["gradient"]], axis=1)
        assert np.array_equal(got, hin, equal_nan=True), b
        assert np.isinf(st["dJ"][0]) and len(hout) == 0


@pytest.mark.gpu
def test_history_altro_maze_equals_oracle(tog, oracle, gpu):
    """The maze ALTRO case (infeasible start): solver_al.traj_stats is the infeasible problem's AL solve
    record for record, as the oracle's restatement of the same flow records it; stats carry :time,
    :time_al, :time_pn; the AL phase's handle stays live (solver.K, solver.lam)."""
    B = 2
    p0 = tog.Problems.quadrotor_maze()
    N = p0.N
    guesses = [tog.problems._maze_guess(N, 5.0, p0.x0[0], p0.xf, tog.problems._MAZE_WAYPOINTS + 0.5 *
                                        np.random.default_rng(5000 + b).standard_normal((3, 5))) for b in range(B)]
    prob = tog.Problem(p0.model, p0.obj, np.repeat(p0._U, B, axis=0), constraints=p0.constraints,
                       x0=np.repeat(p0.x0, B, axis=0), xf=p0.xf, N=N, dt=p0.dt)
    prob._X[...] = np.stack(guesses)
    opts = tog.Problems.maze_altro_options()
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    assert solver.stats["time"] >= solver.stats["time_al"] > 0 and solver.stats["time_pn"] == 0.0
    assert solver.K.shape == (B, N - 1, 4 + 13, 13)  # the infeasible problem's gains (m + n controls)
    assert solver.lam.shape[0] == B
    for b in range(B):
        _, _, si, _ = oracle.solve_altro_infeasible(prob, opts, b)
        hin, hout, _ = si.history()
        st = solver.solver_al.traj_stats(b)
        assert st["iterations"] == len(hout)
        for key, col in (("iterations_inner", 0), ("cost", 1), ("c_max", 2), ("penalty_max", 3)):
            assert np.array_equal(np.asarray(st[key], dtype=float), hout[:, col], equal_nan=True), (b, key)
        inner = np.concatenate([np.stack([u["cost"], u["dJ"], u["gradient"]], axis=1) for u in st["stats_uncon"]])
        assert np.array_equal(inner, hin[:len(inner)], equal_nan=True), b


@pytest.mark.gpu
def test_history_pn_equals_oracle(tog, oracle, gpu):
    """ALTRO with projected Newton (car, 3 starts, 6 newton steps): solver_pn.traj_stats(b) :cost and
    :c_max per newton step against the oracle's, and the AL phase's records bit for bit."""
    prob = car_batch(tog, 3, seed=11)
    al = car_al_opts(tog, tol=1e-3)
    opts = tog.ALTROSolverOptions(opts_al=al, projected_newton=True, projected_newton_tolerance=1e-2)
    opts.opts_pn.feasibility_tolerance = 1e-10
    opts.opts_pn.active_set_tolerance = 1e-4
    opts.opts_pn.n_steps = 6
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    assert solver.stats["time_pn"] > 0.0
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts.opts_al, b=b)
        o.solve()
        o.solve_pn(opts.opts_pn)
        hin, hout, hpn = o.history()
        pn = solver.solver_pn.traj_stats(b)
        assert pn["iterations"] == len(hpn) == solver.stats_pn["iterations"][b]
        assert np.allclose(pn["cost"], hpn[:, 0], rtol=TOL_PN, atol=0)
        assert np.allclose(pn["c_max"], hpn[:, 1], rtol=0, atol=TOL_PN)
        st = solver.solver_al.traj_stats(b)
        assert np.array_equal(st["c_max"], hout[:, 2]) and np.array_equal(st["cost"], hout[:, 1])


@pytest.mark.gpu
def test_history_off_by_default_on_handles(tog, gpu):
    """A handle records nothing until tog_history_enable (the bench's solves pay no history stores);
    reading a history field then fails loudly."""
    prob, opts = tog.Problems.config_quadrotor(B=2)
    s = tog.AbstractSolverFor(prob, opts)
    assert s.handle.history() is None
    with pytest.raises(RuntimeError):
        out = np.empty((2, 1, 3))
        tog.abi.check(s.handle.lib, s.handle.lib.tog_get(s.handle.h, tog.abi.FIELD_HIST_INNER, tog.abi.as_dp(out)))


@pytest.mark.gpu
def test_history_reenable_reuses_buffers(tog, gpu):
    """tog_history_enable on one long-lived handle with shrinking and growing capacities (advisor round 5: each
    change used to allocate new buffers and keep the old ones until tog_destroy): a smaller capacity reuses the
    allocation, a larger one replaces it, off (0) and on again works, and every solve's records equal those of
    a fresh handle with the same capacity."""
    prob, opts = tog.Problems.config_quadrotor(B=2)
    solver = tog.AbstractSolverFor(prob, opts)
    for cap in (4000, 30, 0, 2500, 6000):
        gp = prob.copy()
        s = tog.solve_b(gp, solver, history=cap if cap else False)
        if cap == 0:
            assert s.history is None
            continue
        fresh = tog.solve_b(prob.copy(), tog.AbstractSolverFor(prob, opts), history=cap)
        for a, b_ in zip(s.history, fresh.history):
            assert a.shape == b_.shape, cap
            if a.ndim == 3 and a.shape[-1] == 3:  # inner records: compare the written ones
                cnt = s.history[2][:, 0]
                for b in range(prob.B):
                    # (record 0's gradient is calculate_gradient at the start with the solver's current d: the
                    # previous solve's on a reused solver, as in the reference; zero on the fresh one)
                    k = min(int(cnt[b]), cap)
                    assert np.array_equal(a[b, 0, :2], b_[b, 0, :2]), (cap, b)
                    assert np.array_equal(a[b, 1:k], b_[b, 1:k], equal_nan=True), (cap, b)
            elif a.ndim == 3:  # outer records: the written ones (unwritten slots hold whatever memory held)
                cnt = s.history[2][:, 1]
                for b in range(prob.B):
                    k = min(int(cnt[b]), a.shape[1])
                    assert np.array_equal(a[b, :k], b_[b, :k], equal_nan=True), (cap, b)
            else:
                assert np.array_equal(a, b_), cap
