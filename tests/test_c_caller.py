"""A plain C caller of the ABI (tests/c/test_capi_config3.c): it fills tog_problem_desc for BASELINE
config 3 exactly as integration/julia/libtog.jl's tog_desc marshals the reference Problem (the Julia
binding itself cannot run here: no Julia in the image), solves through tog_create -> tog_set_state ->
tog_solve -> tog_get, and must equal the Python (ctypes) path bit for bit: same descriptor, same
device code, so X, U and every per-trajectory statistic agree exactly."""
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
BIN = ROOT / "tests" / "c" / "test_capi_config3"
BIN_ALTRO = ROOT / "tests" / "c" / "test_capi_altro"


def test_c_caller_links_the_library(tog):
    """The C program links libtog.so and sees the same ABI version (no device needed)."""
    assert BIN.exists(), "tests/c/test_capi_config3 not built: __graft_entry__.build() builds it"
    r = subprocess.run([str(BIN), "--version"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip()) == tog.abi.TOG_ABI_VERSION


@pytest.mark.gpu
def test_c_caller_equals_python_path(tog, gpu, tmp_path):
    B = 16
    prob, opts = tog.Problems.config_quadrotor(B=B)
    n, m, N = 13, 4, 101
    # prob.x0 (B, n) and prob.U (B, N-1, m) row-major are the ABI's column-major (n, B), (m, N-1, B)
    U0 = np.ascontiguousarray(prob.U)
    with open(tmp_path / "in.bin", "wb") as f:
        f.write(np.int64(B).tobytes())
        f.write(np.ascontiguousarray(prob.x0).tobytes())
        f.write(U0.tobytes())
    r = subprocess.run([str(BIN), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = np.fromfile(tmp_path / "out.bin", dtype=np.float64)
    X_c = out[:B * N * n].reshape(B, N, n)
    U_c = out[B * N * n:B * N * n + B * (N - 1) * m].reshape(B, N - 1, m)
    St_c = out[B * N * n + B * (N - 1) * m:].reshape(B, tog.abi.NSTATS)
    gpu = prob.copy()
    solver = tog.solve_b(gpu, opts)
    St_py = solver.handle.get(tog.abi.FIELD_STATS)
    assert np.array_equal(X_c, gpu._X), np.max(np.abs(X_c - gpu._X))
    assert np.array_equal(U_c, gpu._U), np.max(np.abs(U_c - gpu._U))
    assert np.array_equal(St_c, St_py)


@pytest.mark.gpu
def test_c_caller_altro_equals_python_path(tog, gpu, tmp_path):
    """tog_solve_altro from C (tests/c/test_capi_altro.c: the quadrotor_maze ALTRO case of
    test/infeasible_tests.jl:57-76 as libtog.jl marshals it, an infeasible start from a state guess) equals
    solve_b(prob, ALTROSolverOptions) from Python bit for bit, on B = 4 jittered way-point guesses."""
    assert BIN_ALTRO.exists(), "tests/c/test_capi_altro not built: __graft_entry__.build() builds it"
    B = 4
    p0 = tog.Problems.quadrotor_maze()
    n, m, N = 13, 4, p0.N
    guesses = [tog.problems._maze_guess(N, 5.0, p0.x0[0], p0.xf, tog.problems._MAZE_WAYPOINTS + 0.5 *
                                        np.random.default_rng(5000 + b).standard_normal((3, 5))) for b in range(B)]
    prob = tog.Problem(p0.model, p0.obj, np.repeat(p0._U, B, axis=0), constraints=p0.constraints,
                       x0=np.repeat(p0.x0, B, axis=0), xf=p0.xf, N=N, dt=p0.dt)
    prob._X[...] = np.stack(guesses)
    with open(tmp_path / "in.bin", "wb") as f:
        f.write(np.int64(B).tobytes())
        f.write(np.ascontiguousarray(prob.x0).tobytes())
        f.write(np.ascontiguousarray(prob._U).tobytes())
        f.write(np.ascontiguousarray(prob._X).tobytes())
    r = subprocess.run([str(BIN_ALTRO), str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    out = np.fromfile(tmp_path / "out.bin", dtype=np.float64)
    X_c = out[:B * N * n].reshape(B, N, n)
    U_c = out[B * N * n:B * N * n + B * (N - 1) * m].reshape(B, N - 1, m)
    o = B * N * n + B * (N - 1) * m
    St_c = out[o:o + B * tog.abi.NSTATS].reshape(B, tog.abi.NSTATS)
    o += B * tog.abi.NSTATS
    opts = tog.Problems.maze_altro_options()
    ocap = opts.opts_al.iterations + 1
    cap = opts.opts_al.iterations * (opts.opts_al.opts_uncon.iterations + 1) + 1
    cnt_c = out[o:o + 2 * B].reshape(B, 2).astype(np.int64)
    o += 2 * B
    Hout_c = out[o:o + 4 * ocap * B].reshape(B, ocap, 4)
    o += 4 * ocap * B
    Hin_c = out[o:].reshape(B, cap, 3)
    gp = prob.copy()
    solver = tog.solve_b(gp, opts, history=cap)
    assert np.array_equal(X_c, gp._X), np.max(np.abs(X_c - gp._X))
    assert np.array_equal(U_c, gp._U), np.max(np.abs(U_c - gp._U))
    assert np.array_equal(St_c[:, tog.abi.STAT_TOTAL_STEPS], solver.stats["iterations_total"])
    assert np.array_equal(St_c[:, tog.abi.STAT_FLAGS].astype(np.int64), solver.stats["flags"])
    # the C caller reads the same solver_al.stats histories
    Hin, Hout, cnt = solver.solver_al.history
    assert np.array_equal(cnt_c, cnt)
    for b in range(B):
        assert np.array_equal(Hin_c[b, :cnt[b, 0]], Hin[b, :cnt[b, 0]], equal_nan=True)
        assert np.array_equal(Hout_c[b, :cnt[b, 1]], Hout[b, :cnt[b, 1]], equal_nan=True)
        st = solver.solver_al.traj_stats(b)
        assert st["iterations_total"] == int(St_c[b, tog.abi.STAT_TOTAL_STEPS]) + st["iterations"] - 1
