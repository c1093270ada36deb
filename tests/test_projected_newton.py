"""ALTRO phase 2, the projected Newton feasible projection:
src/solvers/direct/projected_newton.jl:6-303 with ProjectedNewtonSolverOptions
(direct_solvers.jl:14-30), driven from ALTRO by altro_methods.jl:5-39.

CPU tests pin the oracle (oracle/tog_oracle_pn.c) on the reference's own assertions
(test/projected_newton_test.jl:111-120: after the projection ``max_violation < feasibility_tolerance``;
test/altro_tests.jl:40-46,65: the 1e-10 polish after an AL phase stopped at 1e-2). The ``gpu`` tests
hold libtog.so (k_pn_begin / k_pn_project / k_pn_finish, tog_pn.hpp, through the C ABI) bit for bit
to the oracle from the same AL iterate: X, U and every statistic.
"""
import numpy as np
import pytest

TOL_STEP = 1e-13


def rel(a, b):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    scale = max(1.0, float(np.max(np.abs(b)))) if b.size else 1.0
    return float(np.max(np.abs(a - b))) / scale if b.size else 0.0


def car_al_opts(tog, tol=1e-3):
    """test/projected_newton_test.jl:29-35 (AL phase before the projection)."""
    return tog.AugmentedLagrangianSolverOptions(opts_uncon=tog.iLQRSolverOptions(), constraint_tolerance=tol,
                                                constraint_tolerance_intermediate=1e-1)


def car_batch(tog, B, seed=3):
    """Problems.car_obstacles with B perturbed copies of the reference's U0 = ones."""
    rng = np.random.default_rng(seed)
    U0 = np.ones((B, 50, 2)) + 0.05 * rng.standard_normal((B, 50, 2))
    U0[0] = 1.0
    return tog.Problems.car_obstacles(U0=U0, B=B)


def oracle_al_state(tog, oracle, prob, opts):
    """AL-solve every trajectory on the oracle; returns a copy of prob holding the AL iterates."""
    p = prob.copy()
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts, b=b)
        o.solve()
        p._X[b] = o.get("X")
        p._U[b] = o.get("U")
    return p


# ----------------------------------------------------------------------------- CPU: host + oracle


def test_pn_options_defaults(tog):
    """ProjectedNewtonSolverOptions defaults (direct_solvers.jl:14-30) on both sides of the ABI."""
    o = tog.ProjectedNewtonSolverOptions()
    assert (o.n_steps, o.solve_type, o.active_set_tolerance, o.feasibility_tolerance) == (1, "feasible", 1e-3, 1e-6)
    c = tog.to_tog_pn_options(o)
    assert (c.n_steps, c.solve_type, c.active_set_tolerance, c.feasibility_tolerance) == (1, 0, 1e-3, 1e-6)
    lib = tog.abi.load_library()
    d = tog.abi.tog_pn_options()
    lib.tog_default_pn_options(d)
    assert (d.n_steps, d.solve_type, d.active_set_tolerance, d.feasibility_tolerance) == (1, 0, 1e-3, 1e-6)
    assert tog.to_tog_pn_options(tog.ProjectedNewtonSolverOptions(solve_type="optimal")).solve_type == 1
    with pytest.raises(ValueError):
        tog.to_tog_pn_options(tog.ProjectedNewtonSolverOptions(solve_type="fast"))


def test_altro_pn_tolerances(tog):
    """altro_methods.jl:5-13: projected_newton moves the AL phase's constraint tolerance."""
    opts = tog.ALTROSolverOptions(projected_newton=True, projected_newton_tolerance=1e-2)
    tog.solvers._altro_pn_tolerances(opts)
    assert opts.opts_al.constraint_tolerance == 1e-2 and not opts.opts_al.kickout_max_penalty
    opts = tog.ALTROSolverOptions(projected_newton=True, projected_newton_tolerance=-1.0)
    tog.solvers._altro_pn_tolerances(opts)
    assert opts.opts_al.constraint_tolerance == 0.0 and opts.opts_al.kickout_max_penalty
    opts = tog.ALTROSolverOptions(projected_newton=False)
    tol0 = opts.opts_al.constraint_tolerance
    tog.solvers._altro_pn_tolerances(opts)
    assert opts.opts_al.constraint_tolerance == tol0


def test_iros_maze_options(tog):
    """The IROS 2019 quadrotor maze demo's options (examples/IROS_2019/quadrotor_maze.jl:8-34), and
    altro_methods.jl:5-13's AL tolerance once projected Newton is on."""
    opts = tog.Problems.quadrotor_maze_iros_options()
    assert opts.projected_newton and not opts.resolve_feasible_problem and opts.R_inf == 1e-8
    assert opts.opts_pn.feasibility_tolerance == 1e-8 and opts.opts_pn.solve_type == "feasible"
    assert opts.opts_pn.n_steps == 1 and opts.opts_pn.active_set_tolerance == 1e-3
    al = opts.opts_al
    assert (al.iterations, al.cost_tolerance, al.cost_tolerance_intermediate, al.penalty_scaling,
            al.penalty_initial, al.opts_uncon.iterations) == (40, 1e-5, 1e-4, 10.0, 1.0, 300)
    tog.solvers._altro_pn_tolerances(opts)
    assert opts.opts_al.constraint_tolerance == 1e-4


@pytest.mark.parametrize("ft,at", [(1e-6, 1e-3), (1e-10, 1e-3), (1e-10, 1e-4)])
def test_oracle_projection_reaches_tolerance(tog, oracle, ft, at):
    """test/projected_newton_test.jl:111-120: after the projection every constraint is satisfied to
    the feasibility tolerance (``max_violation(solver) < feasibility_tolerance``), and the AL iterate it
    starts from is not (1e-3 AL tolerance)."""
    prob = tog.Problems.car_obstacles()
    o = oracle.OracleSolver(prob, car_al_opts(tog))
    o.solve()
    c0 = o.max_violation()
    assert 1e-7 < c0 < 1e-3
    J0 = o.cost()
    out = o.solve_pn(tog.ProjectedNewtonSolverOptions(feasibility_tolerance=ft, active_set_tolerance=at, n_steps=3))
    assert out[tog.abi.PN_C_MAX] < ft
    assert out[tog.abi.PN_C_MAX] == o.max_violation()
    assert out[tog.abi.PN_VIOL] < ft
    assert out[tog.abi.PN_STEPS] >= 1 and out[tog.abi.PN_PROJECTIONS] >= 1
    assert out[tog.abi.PN_LINESEARCHES] >= out[tog.abi.PN_PROJECTIONS]
    # a feasibility projection: the cost moves by a small amount only
    assert abs(out[tog.abi.PN_J] - J0) < 1e-2 * abs(J0)


def test_oracle_projection_noop_when_feasible(tog, oracle):
    """projection_solve!'s while loop (projected_newton.jl:198-210) does not run when viol <= eps;
    solve! still records one iteration."""
    prob = tog.Problems.car_obstacles()
    o = oracle.OracleSolver(prob, car_al_opts(tog))
    o.solve()
    o.solve_pn(tog.ProjectedNewtonSolverOptions(feasibility_tolerance=1e-10))
    X, U = o.get("X"), o.get("U")
    out = o.solve_pn(tog.ProjectedNewtonSolverOptions(feasibility_tolerance=1e-2))
    assert out[tog.abi.PN_PROJECTIONS] == 0 and out[tog.abi.PN_STEPS] == 1
    assert np.array_equal(o.get("X"), X) and np.array_equal(o.get("U"), U)


def _optimal_vs_feasible(tog, oracle, ft=1e-10, n_steps=1, prob=None):
    prob = prob if prob is not None else tog.Problems.car_obstacles()
    res = {}
    for st in ("feasible", "optimal"):
        o = oracle.OracleSolver(prob, car_al_opts(tog))
        o.solve()
        out = o.solve_pn(tog.ProjectedNewtonSolverOptions(feasibility_tolerance=ft, n_steps=n_steps, solve_type=st))
        res[st] = (o, out, int(o.get("stats")[tog.abi.STAT_FLAGS]))
    return res


def test_oracle_optimal_newton_step(tog, oracle):
    """solve_type :optimal (newton_step!, projected_newton.jl:501-547: the projection, multiplier_projection!,
    solveKKT_Shur with stats[:S], line_search with projection! at each trial) on the reference's projected
    Newton problem: test/projected_newton_test.jl:161-170's assertions for a newton step -- the result is
    feasible to 1e-10 and costs less than the start -- and it costs less than the :feasible projection of the
    same AL iterate (the KKT step moves along the constraint manifold towards the optimum)."""
    r = _optimal_vs_feasible(tog, oracle)
    (of, outf, ff), (oo, outo, fo) = r["feasible"], r["optimal"]
    assert not fo & tog.abi.TRAJ_PN_ERROR and not ff & tog.abi.TRAJ_PN_ERROR
    assert outo[tog.abi.PN_C_MAX] < 1e-10 and outo[tog.abi.PN_C_MAX] == oo.max_violation()
    assert outo[tog.abi.PN_J] < outf[tog.abi.PN_J]
    assert outo[tog.abi.PN_J] == oo.cost()
    assert outo[tog.abi.PN_STEPS] == 1 and outo[tog.abi.PN_PROJECTIONS] >= 1


def test_oracle_optimal_steps_restart_from_solver_v(tog, oracle):
    """solve! copies each newton step's V_ into prob but never into solver.V (projected_newton.jl:8-17), so a
    second :optimal step restarts from the projected solver.V: with a tolerance the first step cannot meet
    (feasibility_tolerance = 0 never breaks), three steps return what one step returns, or flag the stale
    stats[:S] (a step that did not project uses the previous factor)."""
    one = _optimal_vs_feasible(tog, oracle, ft=0.0, n_steps=1)["optimal"]
    three = _optimal_vs_feasible(tog, oracle, ft=0.0, n_steps=3)["optimal"]
    if not three[2] & tog.abi.TRAJ_PN_ERROR:
        assert np.array_equal(one[0].get("X"), three[0].get("X"))
        assert np.array_equal(one[0].get("U"), three[0].get("U"))


def test_oracle_optimal_on_min_time(tog, oracle):
    """solve_type :optimal on a minimum-time problem (round 6): the minimum-time problem's H (MinTimeCost's
    hessian! diagonal) and g (its gradient!) move with V, so they are re-formed wherever newton_step! and
    line_search call cost_expansion! (projected_newton.jl:463-547). The step reaches the feasibility tolerance
    and costs no more than the :feasible projection of the same AL iterate, or is flagged as the reference
    would raise."""
    import test_minimum_time as T
    make, opts, xf, U0, dt, dt_mt, _ = T.pendulum_case(tog)
    p = make(U0, dt_mt, tf="min")
    pmt = tog.minimum_time_problem(p, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    al = opts.opts_al
    al.constraint_tolerance = 1e-3
    res = {}
    for st in ("feasible", "optimal"):
        o = oracle.OracleSolver(pmt, al)
        o.solve()
        out = o.solve_pn(tog.ProjectedNewtonSolverOptions(feasibility_tolerance=1e-8, n_steps=2, solve_type=st))
        res[st] = (o, out, int(o.get("stats")[tog.abi.STAT_FLAGS]))
    (of, outf, ff), (oo, outo, fo) = res["feasible"], res["optimal"]
    assert np.isfinite(oo.get("X")).all() and np.isfinite(oo.get("U")).all()
    if not fo & tog.abi.TRAJ_PN_ERROR:
        assert outo[tog.abi.PN_C_MAX] <= 1e-8
        assert outo[tog.abi.PN_J] <= outf[tog.abi.PN_J] * (1 + 1e-9)


def test_car_batch_problem(tog, oracle):
    """The batched car problem the GPU tests use: B trajectories, the AL iterates are finite."""
    prob = car_batch(tog, 2)
    assert prob.B == 2 and prob._U.shape == (2, 50, 2)
    st = oracle_al_state(tog, oracle, prob, car_al_opts(tog))
    assert np.isfinite(st._X).all() and np.isfinite(st._U).all()


# ----------------------------------------------------------------------------- GPU: device vs oracle


def _pn_compare(tog, oracle, prob, al_opts, pn_opts):
    """Device projected Newton from the oracle's AL iterates vs the oracle from the same state."""
    start = oracle_al_state(tog, oracle, prob, al_opts)
    gp = start.copy()
    solver = tog.ProjectedNewtonSolver(gp, pn_opts)
    tog.solve_b(gp, solver)
    st = solver.stats
    for b in range(prob.B):
        o = oracle.OracleSolver(start, al_opts, b=b)  # X given: PrimalDual(prob) from the AL iterate
        out = o.solve_pn(pn_opts)
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        for key, idx in (("projections", tog.abi.PN_PROJECTIONS), ("linesearches", tog.abi.PN_LINESEARCHES),
                         ("refinements", tog.abi.PN_REFINEMENTS), ("iterations", tog.abi.PN_STEPS)):
            assert st[key][b] == out[idx], (b, key, st[key][b], out[idx])
        assert abs(st["c_max"][b] - out[tog.abi.PN_C_MAX]) <= 1e-13 * max(1.0, abs(out[tog.abi.PN_C_MAX]))
        assert rel(st["cost"][b], out[tog.abi.PN_J]) < TOL_STEP
        assert rel(st["viol"][b], out[tog.abi.PN_VIOL]) < TOL_STEP
    return gp, st


@pytest.mark.gpu
@pytest.mark.parametrize("ft,at", [(1e-6, 1e-3), (1e-10, 1e-4)])
def test_gpu_pn_car_parity(tog, oracle, gpu, ft, at):
    """Device vs oracle on the reference's projected Newton problem, 4 perturbed starts."""
    prob = car_batch(tog, 4)
    pn = tog.ProjectedNewtonSolverOptions(feasibility_tolerance=ft, active_set_tolerance=at, n_steps=3)
    gp, st = _pn_compare(tog, oracle, prob, car_al_opts(tog), pn)
    ok = (st["flags"] & tog.abi.TRAJ_PN_ERROR) == 0
    assert np.all(st["c_max"][ok] < ft)


@pytest.mark.gpu
def test_gpu_altro_projected_newton(tog, oracle, gpu):
    """ALTRO with projected_newton (test/altro_tests.jl:40-46,65): AL to 1e-2, then the polish to
    1e-10 on the same device buffers; the oracle runs the same two phases."""
    prob = car_batch(tog, 3, seed=11)
    al = car_al_opts(tog, tol=1e-3)
    opts = tog.ALTROSolverOptions(opts_al=al, projected_newton=True, projected_newton_tolerance=1e-2)
    opts.opts_pn.feasibility_tolerance = 1e-10
    opts.opts_pn.active_set_tolerance = 1e-4
    # one newton step (the default) leaves rows that were outside the 1e-4 active set violated by
    # up to ~1e-2 (the step moves them); later steps re-evaluate the active set and finish the polish
    opts.opts_pn.n_steps = 6
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    assert opts.opts_al.constraint_tolerance == 1e-2
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts.opts_al, b=b)
        o.solve()
        out = o.solve_pn(opts.opts_pn)
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        assert solver.stats_pn["iterations"][b] == out[tog.abi.PN_STEPS]
        assert abs(solver.stats_pn["c_max"][b] - out[tog.abi.PN_C_MAX]) <= 1e-13
        if not solver.stats_pn["flags"][b] & tog.abi.TRAJ_PN_ERROR:
            assert solver.stats_pn["c_max"][b] < 1e-10


@pytest.mark.gpu
def test_gpu_pn_quad_maze(tog, oracle, gpu):
    """Config 4 constraint set (n + pmax = 32 rows per block, the largest the wave kernels take)
    at a short horizon: device vs oracle from the oracle's AL iterates."""
    prob, opts = tog.Problems.config_quad_maze(B=2, N=41)
    pn = tog.ProjectedNewtonSolverOptions(feasibility_tolerance=1e-8, n_steps=2)
    _pn_compare(tog, oracle, prob, opts, pn)


@pytest.mark.gpu
@pytest.mark.parametrize("ft,at,n_steps", [(1e-10, 1e-3, 1), (1e-6, 1e-3, 1), (1e-8, 1e-5, 3), (1e-8, 0.0, 1)])
def test_gpu_pn_optimal_parity(tog, oracle, gpu, ft, at, n_steps):
    """solve_type :optimal on the device (k_pn_kkt, k_pn_ls_begin / k_pn_ls_proj / k_pn_ls_end, tog_pn.hpp)
    against the oracle from the same AL iterates, 4 perturbed car starts: X, U and every statistic to 1e-13.
    The small active-set tolerances make the full KKT step violate rows outside the active set, so the line
    search's projection! grows the active set past the free variables and rejects trials (the reject path)."""
    prob = car_batch(tog, 4)
    pn = tog.ProjectedNewtonSolverOptions(feasibility_tolerance=ft, active_set_tolerance=at, n_steps=n_steps,
                                          solve_type="optimal")
    gp, st = _pn_compare(tog, oracle, prob, car_al_opts(tog), pn)
    assert np.all(np.isfinite(gp._X)) and np.all(np.isfinite(gp._U))


@pytest.mark.gpu
def test_gpu_altro_pn_optimal(tog, oracle, gpu):
    """ALTRO with opts_pn.solve_type = :optimal end to end (altro_methods.jl:31-39): the AL phase to 1e-2 and
    the KKT polish on the device against the oracle's two phases."""
    prob = car_batch(tog, 3, seed=11)
    opts = tog.ALTROSolverOptions(opts_al=car_al_opts(tog, tol=1e-3), projected_newton=True,
                                  projected_newton_tolerance=1e-2)
    opts.opts_pn.feasibility_tolerance = 1e-8
    opts.opts_pn.solve_type = "optimal"
    gp = prob.copy()
    solver = tog.solve_b(gp, opts)
    for b in range(prob.B):
        o = oracle.OracleSolver(prob, opts.opts_al, b=b)
        o.solve()
        out = o.solve_pn(opts.opts_pn)
        assert rel(gp._X[b], o.get("X")) < TOL_STEP and rel(gp._U[b], o.get("U")) < TOL_STEP, b
        assert solver.stats_pn["iterations"][b] == out[tog.abi.PN_STEPS]
        assert abs(solver.stats_pn["c_max"][b] - out[tog.abi.PN_C_MAX]) <= 1e-13


def _oracle_iros(args):
    oracle, prob, opts, b = args
    X, U, si, _ = oracle.solve_altro_infeasible(prob, opts, b)
    _, hout, hpn = si.history()
    return X, U, len(hout), hpn, int(si.get("stats")[oracle._pkg.abi.STAT_FLAGS])


@pytest.mark.gpu
def test_gpu_iros_quadrotor_maze_altro_pn(tog, oracle, gpu):
    """The reference's IROS 2019 demo, solve(Problems.quadrotor_maze, opts_altro) with projected Newton
    (examples/IROS_2019/quadrotor_maze.jl:23-48): the infeasible-start AL phase (n = 13, m = 4 + 13, 69 rows a
    knot) to 1e-4, then the feasible projection on the infeasible problem (blocks of n + active rows, up to
    n + m = 30 variables a knot) to 1e-8. Trajectory 0 starts from the reference's own guess
    (problems/quadrotor_maze.jl:104-113), 1-3 from jittered way-points. Device == oracle within the north star's
    1e-6 (relative, fp64), equal AL outer iterations, newton steps and flags. Starts 1 and 2 hit the reference's
    own exception in _projection_linesearch! (projected_newton.jl:273-277) on both sides; the reference's start
    ends feasible to 1e-8, as the notebook's 9.63e-9 (examples/quadrotor/Quadrotor Maze.ipynb, cell 3)."""
    from concurrent.futures import ThreadPoolExecutor
    B = 4
    prob = tog.Problems.quadrotor_maze_batch(B)
    prob._X[0] = tog.Problems.quadrotor_maze_batch(1, jitter=0.0)._X[0]
    opts = tog.Problems.quadrotor_maze_iros_options()
    gp = prob.copy()
    try:
        solver = tog.solve_b(gp, opts)
        raised = []
    except tog.ProjectedNewtonError as e:  # the reference raises for such a start; the batch's results stand
        solver, raised = e.solver, e.trajectories
    assert solver.stats["time_pn"] > 0.0
    o_opts = tog.Problems.quadrotor_maze_iros_options()
    tog.solvers._altro_pn_tolerances(o_opts)
    with ThreadPoolExecutor(B) as ex:  # the oracle's C calls release the GIL
        refs = list(ex.map(_oracle_iros, [(oracle, prob, o_opts, b) for b in range(B)]))
    print(f"\nIROS maze ALTRO+PN on the device: {B} starts in {solver.stats['time']:.2f} s "
          f"(AL {solver.stats['time_al']:.2f} s, PN {solver.stats['time_pn']:.3f} s); "
          f"the reference publishes 85.8 s for one start (context only)")
    flags = solver.stats_pn["flags"]
    err_o = []
    for b, (X, U, n_out, hpn, fo) in enumerate(refs):
        assert rel(gp._X[b], X) < 1e-6 and rel(gp._U[b], U) < 1e-6, b
        assert solver.solver_al.traj_stats(b)["iterations"] == n_out, b
        assert solver.stats_pn["iterations"][b] == len(hpn), b
        assert bool(flags[b] & tog.abi.TRAJ_PN_ERROR) == bool(fo & tog.abi.TRAJ_PN_ERROR), b
        if fo & tog.abi.TRAJ_PN_ERROR:
            err_o.append(b)
        c = solver.stats_pn["c_max"][b]
        assert abs(c - hpn[-1, 1]) <= 1e-9 * max(1.0, hpn[-1, 1]), (b, c, hpn[-1, 1])
        print(f"  start {b}: AL outer {n_out}, c_max after PN {c:.3e} (oracle {hpn[-1, 1]:.3e})"
              + (" [the reference's _projection_linesearch! exception]" if fo & tog.abi.TRAJ_PN_ERROR else ""))
    assert list(raised) == err_o
    assert solver.stats_pn["c_max"][0] <= 1e-8 and not flags[0] & tog.abi.TRAJ_PN_ERROR
    assert not np.any(flags & tog.abi.TRAJ_PN_BLOCK)
