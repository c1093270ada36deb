"""CPU-side checks of the drop-in boundary: libtog.so loads and exports every function that
include/tog.h declares, option defaults mirror the reference's, the host mirror builds the same
problem descriptor the kernels read, and the product path fails loudly without the HIP library or
a device (no CPU fallback). No compute calls are made here.
"""
import ctypes
import math
import pathlib
import re

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "tog.h"


def declared_functions():
    src = HEADER.read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tog_[a-z0-9_]+)\s*\(", src)))


def test_header_and_python_mirror_agree(tog):
    assert declared_functions() == sorted(tog.abi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(tog):
    lib = tog.abi.load_library()
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_version_and_device_count_without_gpu(tog):
    lib = tog.abi.load_library()
    assert lib.tog_version() == tog.abi.TOG_ABI_VERSION
    assert lib.tog_device_count() >= 0  # 0 in a GPU-less container, never a crash


def test_default_options_mirror_reference_defaults(tog):
    """tog_default_options == iLQRSolverOptions() + AugmentedLagrangianSolverOptions() defaults
    (ilqr_solver.jl:7-81, augmented_lagrangian_solver.jl:8-66)."""
    lib = tog.abi.load_library()
    o = tog.abi.tog_options()
    lib.tog_default_options(ctypes.byref(o))
    ref = tog.to_tog_options(tog.AugmentedLagrangianSolverOptions())
    for name, _ in tog.abi.tog_options._fields_:
        assert getattr(o, name) == getattr(ref, name), name
    assert o.cost_tolerance == 1e-4 and o.iterations == 300 and o.iterations_linesearch == 20
    assert o.bp_reg_increase_factor == 1.6 and o.bp_reg_min == 1e-8 and o.bp_reg_max == 1e8
    assert o.line_search_lower_bound == 1e-8 and o.line_search_upper_bound == 10.0


def test_create_without_device_fails_loudly(tog):
    """With no HIP device the boundary returns TOG_ERR_DEVICE with a message — never computes on
    the CPU."""
    lib = tog.abi.load_library()
    if lib.tog_device_count() > 0:
        pytest.skip("a device is visible")
    prob = tog.Problems.cartpole(constrained=False)
    desc = prob.build_desc()
    o = tog.to_tog_options(tog.iLQRSolverOptions())
    h = ctypes.c_void_p()
    rc = lib.tog_create(ctypes.byref(desc.desc), ctypes.byref(o), 0, ctypes.byref(h))
    assert rc == tog.abi.ERR_DEVICE
    assert lib.tog_last_error()
    with pytest.raises(RuntimeError):
        tog.iLQRSolver(prob, tog.iLQRSolverOptions())


def test_missing_library_raises(tog, tmp_path):
    with pytest.raises(RuntimeError, match="libtog.so not found"):
        tog.abi.load_library(tmp_path / "libtog.so")


# ------------------------------------------------------------------ problem descriptor

def test_desc_dimensions_and_costs(tog):
    prob = tog.Problems.quadrotor_test("goal+bounds")
    keep = prob.build_desc()  # owns the arrays the descriptor points at
    d = keep.desc
    assert (d.model, d.n, d.m, d.N, d.batch) == (tog.abi.MODEL_QUADROTOR, 13, 4, 101, 1)
    assert d.integrator == tog.abi.RK4 and d.dt == 0.05
    Q = np.ctypeslib.as_array(d.Q, shape=(13 * 13,)).reshape(13, 13, order="F")
    assert np.array_equal(Q, 1e-2 * np.eye(13))
    qf = np.ctypeslib.as_array(d.qf, shape=(13,))
    assert np.array_equal(qf, -1000.0 * prob.xf)  # LQRCostTerminal q = -Qf xf


def test_desc_constraint_sets(tog):
    """Stage knots share [bounds, goal] (goal is terminal-only), terminal gets the x parts."""
    prob = tog.Problems.quadrotor_test("goal+bounds")
    keep = prob.build_desc()  # owns the arrays the descriptor points at
    d = keep.desc
    knot_set = np.ctypeslib.as_array(d.knot_set, shape=(prob.N,))
    assert len(set(knot_set[:-1].tolist())) == 1
    assert d.n_sets >= 1


def test_problem_validation(tog):
    """problem.jl:169-219 / 308-314: inconsistent N, dt, tf are ArgumentErrors."""
    model = tog.rk3(tog.Dynamics.doubleintegrator)
    obj = tog.LQRObjective(np.eye(2), np.eye(1), np.eye(2), np.zeros(2), 11)
    with pytest.raises(ValueError):
        tog.Problem(model, obj, N=12, dt=0.1)
    with pytest.raises(ValueError):
        tog.Problem(model, obj, N=11, dt=0.1, tf=5.0)
    p = tog.Problem(model, obj, N=11, tf=1.0)
    assert p.dt == pytest.approx(0.1)
    assert np.isnan(p._X).all()  # X starts as NaN (problem.jl:232) -> initial rollout


def test_batched_problem_shapes(tog):
    prob, _ = tog.Problems.config_quadrotor(B=3)
    assert prob.x0.shape == (3, 13) and prob._U.shape == (3, 100, 4)
    assert not np.array_equal(prob._U[0], prob._U[1])  # per-trajectory seeds 2000+b
    prob2, _ = tog.Problems.config_quadrotor(B=3)
    assert np.array_equal(prob._U, prob2._U)  # deterministic


def test_unconstrained_al_uses_inner_options(tog):
    """solve!(prob, AugmentedLagrangianSolverOptions) on an unconstrained problem runs the inner
    iLQR options (solvers.jl dispatch)."""
    ilqr = tog.iLQRSolverOptions(cost_tolerance=3e-5)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr)
    o = tog.to_tog_options(al)
    assert o.cost_tolerance == 3e-5
    assert o.al_cost_tolerance == al.cost_tolerance and o.constraint_tolerance == al.constraint_tolerance


def test_math_kernels_match_libm(oracle):
    """include/tog_math.h sin/cos (fdlibm kernels shared by the oracle and the GPU) stay within
    2 ulp of libm over the angles the models see; next to the zeros (x ~ kπ) the two-constant
    reduction leaves an absolute error below 2^-80."""
    L = oracle.lib()
    L.oc_sin.restype = L.oc_cos.restype = ctypes.c_double
    L.oc_sin.argtypes = L.oc_cos.argtypes = [ctypes.c_double]
    x = np.concatenate([np.linspace(-50, 50, 40001), [0.0, 1e-300, -0.0, math.pi, -math.pi / 2, 1e5]])
    for f, ref in ((L.oc_sin, np.sin), (L.oc_cos, np.cos)):
        got = np.array([f(float(t)) for t in x])
        want = ref(x)
        ulp = np.spacing(np.maximum(np.abs(want), np.finfo(float).tiny))
        assert np.all(np.abs(got - want) <= 2 * ulp + 2.0 ** -80), f
