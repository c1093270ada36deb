"""The oracle and tog_altro.cpp's descriptor transforms under AddressSanitizer + UBSan.

tests/c/asan_oracle (tests/c/Makefile: gcc/g++ -fsanitize=address,undefined -fno-sanitize-recover=all)
links oracle/tog_oracle.c (with its projected Newton and cost units) and csrc/tog_altro_desc.hpp (the
infeasible_desc / min_time_desc transforms tog_solve_altro runs). Each case writes one problem as a blob
(the tog_problem_desc arrays, every constraint's data in a buffer of exactly its own length, the options and
trajectory 0's state), the sanitized driver solves it — directly, or after the C++ infeasible / minimum-time
transform — and its X, U, statistics and histories must equal liboracle.so's for the same problem (through
the Python transforms for the ALTRO kinds) bit for bit. A sanitizer report fails the driver (non-zero exit).
CPU only; the build takes ≈40 s once.
"""
import ctypes as C
import pathlib
import struct
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CDIR = ROOT / "tests" / "c"
BIN = CDIR / "asan_oracle"


@pytest.fixture(scope="module")
def driver():
    r = subprocess.run(["make", "-s", "asan_oracle"], cwd=CDIR, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return BIN


def _con_len(t, count, n, m, abi):
    """doubles of one constraint's data (tog_altro_desc.hpp con_len)."""
    return {abi.CON_BOUND: 2 * n + 2 * m, abi.CON_GOAL: count if count > 0 else n, abi.CON_CIRCLES: 3 * count,
            abi.CON_SPHERES: 4 * count, abi.CON_USER: 3}.get(t, 0)


def write_blob(path, tog, prob, opts_c, mode, kind=0, altro=None, pn=None):
    abi = tog.abi
    db = prob.build_desc()
    d = db.desc
    n, m, N = d.n, d.m, d.N
    out = bytearray()
    i32 = lambda *v: out.extend(struct.pack(f"<{len(v)}i", *v))  # noqa: E731
    f64 = lambda *v: out.extend(struct.pack(f"<{len(v)}d", *v))  # noqa: E731

    def arr(p, k):
        if k:
            out.extend(np.ctypeslib.as_array(p, shape=(k,)).astype("<f8").tobytes())

    def raw(s):
        i32(C.sizeof(s))
        out.extend(bytes(s))

    i32(0x544F4742, kind, d.model, d.integrator, n, m, N, d.flags)
    f64(d.dt, d.c, d.cf, d.R_min_time)
    for p, k in ((d.Q, n * n), (d.R, m * m), (d.H, m * n), (d.q, n), (d.r, m), (d.Qf, n * n), (d.qf, n)):
        arr(p, k)
    if d.stage_costs:
        i32(1)
        arr(d.stage_costs, (N - 1) * (n * n + m * m + m * n + n + m + 1))
    else:
        i32(0)
    i32(d.n_sets)
    for s in range(d.n_sets):
        st = d.sets[s]
        i32(st.n_con)
        for c in range(st.n_con):
            con = st.con[c]
            L = _con_len(con.type, con.count, n, m, abi) if con.data else 0
            i32(con.type, con.count, L)
            arr(con.data, L)
    for k in range(N):
        i32(d.knot_set[k])
    i32(mode)
    raw(opts_c)
    raw(altro if altro is not None else abi.tog_altro_options())
    i32(1 if pn is not None else 0)
    raw(pn if pn is not None else abi.tog_pn_options())
    f64(*prob.x0[0])
    f64(*np.ascontiguousarray(prob._U[0]).ravel())
    X = prob._X[0]
    if np.isfinite(X).all():
        i32(1)
        f64(*np.ascontiguousarray(X).ravel())
    else:
        i32(0)
    pathlib.Path(path).write_bytes(bytes(out))


def run_driver(driver, blob, out):
    r = subprocess.run([str(driver), str(blob), str(out)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-6000:])
    buf = pathlib.Path(out).read_bytes()
    steps, n, m, N = struct.unpack_from("<4i", buf, 0)
    at = 16
    take = lambda k: np.frombuffer(buf, "<f8", k, at)  # noqa: E731
    X = take(N * n).reshape(N, n)
    at += 8 * N * n
    U = take((N - 1) * m).reshape(N - 1, m)
    at += 8 * (N - 1) * m
    stats = take(14)
    at += 8 * 14
    hist = []
    for w in (3, 4, 2):
        (k,) = struct.unpack_from("<i", buf, at)
        at += 4
        hist.append(take(k * w).reshape(k, w))
        at += 8 * k * w
    return steps, X, U, stats, hist


def check_equal(res, o, steps):
    s, X, U, stats, hist = res
    assert s == steps
    assert np.array_equal(X, o.get("X")) and np.array_equal(U, o.get("U"))
    assert np.array_equal(stats, o.get("stats"), equal_nan=True)
    for a, b in zip(hist, o.history()):
        assert np.array_equal(a, b, equal_nan=True)


def _limit(opts, outer=None, inner=None):
    al = getattr(opts, "opts_al", opts)
    if outer is not None and hasattr(al, "opts_uncon"):
        al.iterations = outer
    il = getattr(al, "opts_uncon", al)
    if inner is not None:
        il.iterations = inner
    return opts


def _cases(tog):
    from test_time_varying import cartpole_varying

    out = {}
    p, o = tog.Problems.config_quadrotor(B=1)
    out["config3_al_sqrt"] = (p, o)
    p, o = cartpole_varying(tog, B=1, cross=0.2)
    out["cartpole_varying_dense"] = (p, _limit(o, inner=60))
    p, o = tog.Problems.config_quad_maze(B=1, N=101)
    out["quad_maze_circles_spheres"] = (p, _limit(o, outer=4, inner=40))
    p, o = tog.Problems.config_kuka(B=1)
    out["kuka_al"] = (p, _limit(o, outer=3, inner=20))
    return out


CASES = ["config3_al_sqrt", "cartpole_varying_dense", "quad_maze_circles_spheres", "kuka_al"]


@pytest.mark.parametrize("case", CASES)
def test_asan_oracle_solve(tog, oracle, driver, tmp_path, case):
    """Plain solves (iLQR / AL, std / sqrt, bounds, goal, circles, spheres, a time-varying objective, the
    Kuka RBD model) under the sanitizers equal liboracle.so."""
    prob, opts = _cases(tog)[case]
    o = oracle.OracleSolver(prob, opts)
    write_blob(tmp_path / "p.bin", tog, prob, o.opts, o.mode)
    res = run_driver(driver, tmp_path / "p.bin", tmp_path / "o.bin")
    check_equal(res, o, o.solve())


def test_asan_oracle_projected_newton(tog, oracle, driver, tmp_path):
    """AL then projected Newton (oracle/tog_oracle_pn.c) on the car with obstacles."""
    from test_projected_newton import car_al_opts, car_batch

    prob = car_batch(tog, 1, seed=11)
    al = car_al_opts(tog, tol=1e-3)
    pn = tog.ProjectedNewtonSolverOptions()
    pn.feasibility_tolerance, pn.active_set_tolerance, pn.n_steps = 1e-10, 1e-4, 4
    o = oracle.OracleSolver(prob, al)
    write_blob(tmp_path / "p.bin", tog, prob, o.opts, o.mode, pn=tog.to_tog_pn_options(pn))
    res = run_driver(driver, tmp_path / "p.bin", tmp_path / "o.bin")
    steps = o.solve()
    o.solve_pn(pn)
    check_equal(res, o, steps)


@pytest.mark.parametrize("varying", [False, True])
def test_asan_infeasible_desc(tog, oracle, driver, tmp_path, varying):
    """tog_altro.cpp's infeasible_desc (sanitized) ≡ infeasible_problem: the AL phase of an infeasible-start
    solve of the quadrotor from a line guess, bit for bit."""
    from test_infeasible import quad_line_batch

    prob = quad_line_batch(tog, B=1, N=31, seed=11)
    if varying:
        from test_time_varying import ramp_objective, with_objective

        st, term = prob.obj.stage, prob.obj.terminal
        prob = with_objective(tog, prob, ramp_objective(tog, st.Q, st.R, term.Q, prob.xf, prob.N))
    opts = _limit(tog.ALTROSolverOptions(), outer=4, inner=30)
    ao = tog.solvers.to_tog_altro_options(opts)
    write_blob(tmp_path / "p.bin", tog, prob, ao.opts_al, tog.abi.MODE_AL, kind=1, altro=ao)
    res = run_driver(driver, tmp_path / "p.bin", tmp_path / "o.bin")
    si = oracle.OracleSolver(tog.infeasible_problem(prob, opts.R_inf), opts)
    si.slack_controls()
    check_equal(res, si, si.solve())


@pytest.mark.parametrize("varying", [False, True])
def test_asan_min_time_desc(tog, oracle, driver, tmp_path, varying):
    """tog_altro.cpp's min_time_desc (sanitized) ≡ minimum_time_problem on test/minimum_time_tests.jl's
    pendulum (ramped per-knot weights with ``varying``)."""
    from test_minimum_time import pendulum_case
    from test_time_varying import _pendulum_mt

    make, opts, *_ = (_pendulum_mt if varying else pendulum_case)(tog)
    opts = _limit(opts, outer=6)
    p = make(np.ones((30, 1)), 0.075, tf="min")
    ao = tog.solvers.to_tog_altro_options(opts)
    write_blob(tmp_path / "p.bin", tog, p, ao.opts_al, tog.abi.MODE_AL, kind=2, altro=ao)
    res = run_driver(driver, tmp_path / "p.bin", tmp_path / "o.bin")
    pmt = tog.minimum_time_problem(p, opts.R_minimum_time, opts.dt_max, opts.dt_min)
    s = oracle.OracleSolver(pmt, opts.opts_al)
    check_equal(res, s, s.solve())
