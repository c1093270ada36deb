"""GenericCost (src/cost.jl:239-347) as libtog cost plugins (csrc/tog_cost_plugin.hpp).

* ``plugins/cost_mycost.hip`` is the reference test's ``mycost`` (test/cost_tests.jl:98-108), its
  expansion by the second-order dual numbers of the plugin kernel (ForwardDiff's
  auto_expansion_function, src/cost.jl:289-322); ``plugins/cost_mycost_analytic.hip`` is the
  ``GenericCost(mycost, mycost, gradient, hess, n, m)`` form (test/cost_tests.jl:112-132).
* ``plugins/cost_soft_obstacle.hip`` is a non-quadratic cost (/, sqrt, sin) whose expansion the oracle
  restates operation for operation (oracle/tog_oracle_cost.c).
The reference KATs (E.x == gradient, E.xx == hess, E.ux == hess, stage_cost == mycost) hold exactly on
the oracle and on the device; device and oracle agree bit for bit on random points.
"""
import ctypes as C
import math
import pathlib

import numpy as np
import pytest

PLUG = pathlib.Path(__file__).resolve().parents[1] / "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd" / "csrc" / "plugins"


def _mycost(x, u=None):  # test/cost_tests.jl:100-107, same operation order as the plugin
    if u is None:
        return math.cos(x[0]) + x[1] * x[1]
    return (math.cos(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1])


def _ref_grad_hess(x, u, tog_cos, tog_sin):  # test/cost_tests.jl:114-131
    Q = np.diag([-tog_cos(x[0]), 2 * 0.1])
    R = np.array([[2 * 0.1]])
    H = np.zeros((1, 2))
    q = np.array([-tog_sin(x[0]), (2 * 0.1) * x[1]])
    r = (2 * 0.1) * np.asarray(u)
    return Q, R, H, q, r


def _oracle_trig(oracle):
    L = oracle.lib()
    L.oc_cos.restype = L.oc_sin.restype = C.c_double
    L.oc_cos.argtypes = L.oc_sin.argtypes = [C.c_double]
    return L.oc_cos, L.oc_sin


def test_oracle_reference_kats(oracle):
    """cost_tests.jl:134-142 on the oracle: the dual-number expansion equals the analytic gradient and
    Hessian exactly, for both GenericCost constructors."""
    cos_, sin_ = _oracle_trig(oracle)
    rng = np.random.default_rng(7)
    for _ in range(50):
        x, u = rng.random(2), rng.random(1)
        Q, R, H, q, r = _ref_grad_hess(x, u, cos_, sin_)
        for analytic in (False, True):
            J, Ex, Eu, Exx, Euu, Eux = oracle.generic_cost_expand(oracle.COST_MYCOST, x, u, analytic=analytic)
            assert np.array_equal(Ex[0], q) and np.array_equal(Eu[0], r)
            assert np.array_equal(Exx[0], Q) and np.array_equal(Euu[0], R) and np.array_equal(Eux[0], H)
            assert J[0] == (cos_(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1])
            Jt, Ext, _, Exxt, _, _ = oracle.generic_cost_expand(oracle.COST_MYCOST, x, None, analytic=analytic)
            assert np.array_equal(Ext[0], [-sin_(x[0]), 2 * x[1]])
            assert np.array_equal(Exxt[0], np.diag([-cos_(x[0]), 2.0]))
            assert Jt[0] == cos_(x[0]) + x[1] * x[1]
        assert abs(J[0] - _mycost(x, u)) < 1e-15  # the deterministic cos agrees with libm here


def test_oracle_soft_obstacle_derivatives(oracle):
    """The restated expansion of the non-quadratic cost is a true gradient / Hessian: symmetric and equal
    to central differences of ℓ (rtol 1e-6)."""
    rng = np.random.default_rng(11)
    X, U = rng.normal(size=(20, 4)), rng.normal(size=(20, 2))
    J, Ex, Eu, Exx, Euu, Eux = oracle.generic_cost_expand(oracle.COST_SOFT_OBSTACLE, X, U)
    h = 1e-5
    for p in range(X.shape[0]):
        z = np.concatenate([X[p], U[p]])
        f = lambda zz: oracle.generic_cost_expand(oracle.COST_SOFT_OBSTACLE, zz[:4], zz[4:])[0][0]
        g = lambda zz: np.concatenate([a[0] for a in
                                       oracle.generic_cost_expand(oracle.COST_SOFT_OBSTACLE, zz[:4], zz[4:])[1:3]])
        Hfull = np.block([[Exx[p], Eux[p].T], [Eux[p], Euu[p]]])
        assert np.array_equal(Hfull, Hfull.T) or np.allclose(Hfull, Hfull.T, rtol=1e-14, atol=1e-14)
        gn = np.array([(f(z + h * e) - f(z - h * e)) / (2 * h) for e in np.eye(6)])
        Hn = np.array([(g(z + h * e) - g(z - h * e)) / (2 * h) for e in np.eye(6)]).T
        assert np.allclose(np.concatenate([Ex[p], Eu[p]]), gn, rtol=1e-6, atol=1e-7)
        assert np.allclose(Hfull, Hn, rtol=1e-6, atol=1e-6)


def test_plugin_load_dims_and_errors(tog):
    lib = tog.abi.load_library()
    c = tog.GenericCost(PLUG / "cost_mycost.so")
    assert c.sizes() == (2, 1)
    assert tog.GenericCost(PLUG / "cost_soft_obstacle.so").sizes() == (4, 2)
    assert c.copy().ptr == c.ptr
    h = C.c_void_p()
    assert lib.tog_generic_cost_load(b"/nonexistent/cost.so", C.byref(h)) == tog.abi.ERR_ARG and not h.value
    # a model plugin is not a cost plugin
    assert lib.tog_generic_cost_load(str(PLUG / "user_pendulum.so").encode(), C.byref(h)) == tog.abi.ERR_ARG
    n, m = C.c_int32(), C.c_int32()
    assert lib.tog_generic_cost_dims(None, C.byref(n), C.byref(m)) == tog.abi.ERR_ARG
    # argument checks happen before any device work
    dp = C.POINTER(C.c_double)
    nul = C.cast(None, dp)
    assert lib.tog_generic_cost_expand(c.ptr, 0, 0, nul, nul, -1, nul, nul, nul, nul, nul, nul) == tog.abi.ERR_ARG
    assert lib.tog_generic_cost_expand(c.ptr, 0, 0, nul, nul, 4, nul, nul, nul, nul, nul, nul) == tog.abi.ERR_ARG
    assert lib.tog_generic_cost_expand(c.ptr, 0, 0, nul, nul, 0, nul, nul, nul, nul, nul, nul) == tog.abi.OK


@pytest.mark.gpu
def test_device_reference_kats(tog, oracle, gpu):
    """cost_tests.jl:108-145 through the Python API on the device."""
    cos_, sin_ = _oracle_trig(oracle)
    nl = tog.GenericCost(PLUG / "cost_mycost.so")
    nl2 = tog.GenericCost(PLUG / "cost_mycost_analytic.so")
    rng = np.random.default_rng(3)
    x, u = rng.random(2), rng.random(1)
    assert nl.stage_cost(x, u) == (cos_(x[0]) + u[0] * (0.1 * u[0])) + 0.1 * (x[1] * x[1])
    assert nl.stage_cost(x) == cos_(x[0]) + x[1] * x[1]
    Q, R, H, q, r = _ref_grad_hess(x, u, cos_, sin_)
    for cst in (nl, nl2):
        E = tog.Expansion(np.zeros(2), np.zeros(1), np.zeros((2, 2)), np.zeros((1, 1)), np.zeros((1, 2)))
        cst.cost_expansion(E, x, u)
        assert np.array_equal(E.x, q) and np.array_equal(E.xx, Q) and np.array_equal(E.ux, H)
        assert np.array_equal(E.u, r) and np.array_equal(E.uu, R)
        cst.cost_expansion(E, x)
        assert np.array_equal(E.x, [-sin_(x[0]), 2 * x[1]]) and np.array_equal(E.xx, np.diag([-cos_(x[0]), 2.0]))
    nl3 = nl.copy()
    assert nl3.stage_cost(x, u) == nl.stage_cost(x, u)


@pytest.mark.gpu
@pytest.mark.parametrize("name,cid,analytic", [("cost_mycost", 0, False), ("cost_mycost_analytic", 0, True),
                                                ("cost_soft_obstacle", 1, False)])
def test_device_equals_oracle(tog, oracle, gpu, name, cid, analytic):
    """Batched expansion on the device == oracle bit for bit (stage and terminal), ragged count."""
    c = tog.GenericCost(PLUG / f"{name}.so")
    n, m = c.sizes()
    rng = np.random.default_rng(100 + cid)
    cnt = 1237
    X, U = rng.normal(size=(cnt, n)) * 2.0, rng.normal(size=(cnt, m))
    for Uarg in (U, None):
        J, E = c.expand(X, Uarg)
        Jo, Exo, Euo, Exxo, Euuo, Euxo = oracle.generic_cost_expand(cid, X, Uarg, analytic=analytic)
        assert np.array_equal(J, Jo)
        assert np.array_equal(E.x, Exo) and np.array_equal(E.xx, Exxo)
        if Uarg is not None:
            assert np.array_equal(E.u, Euo) and np.array_equal(E.uu, Euuo) and np.array_equal(E.ux, Euxo)
    J, _ = c.expand(np.zeros((0, n)), np.zeros((0, m)))
    assert J.shape == (0,)


def _hip():
    """libamdhip64 through ctypes: the runtime libtog itself links (torch bundles its own)."""
    h = C.CDLL("/opt/rocm/lib/libamdhip64.so")
    vp = C.c_void_p
    h.hipMalloc.argtypes = [C.POINTER(vp), C.c_size_t]
    h.hipFree.argtypes = [vp]
    h.hipMemcpy.argtypes = [vp, vp, C.c_size_t, C.c_int]
    h.hipStreamCreate.argtypes = [C.POINTER(vp)]
    h.hipStreamSynchronize.argtypes = [vp]
    h.hipStreamDestroy.argtypes = [vp]
    return h


@pytest.mark.gpu
def test_device_pointer_entry_large_batch(tog, oracle, gpu):
    """tog_generic_cost_expand_device on device buffers and a non-default stream, 2^20 points: finite,
    symmetric Hessians, and a seeded sample equal to the oracle bit for bit."""
    c = tog.GenericCost(PLUG / "cost_soft_obstacle.so")
    lib = tog.abi.load_library()
    hip = _hip()
    n, m, cnt = 4, 2, 1 << 20
    rng = np.random.default_rng(5)
    X, U = rng.normal(size=(cnt, n)), rng.normal(size=(cnt, m))
    sizes = [cnt * n, cnt * m, cnt, cnt * n, cnt * m, cnt * n * n, cnt * m * m, cnt * n * m]
    ptrs = []
    try:
        for sz in sizes:
            p = C.c_void_p()
            assert hip.hipMalloc(C.byref(p), sz * 8) == 0
            ptrs.append(p)
        assert hip.hipMemcpy(ptrs[0], X.ctypes.data, X.nbytes, 1) == 0
        assert hip.hipMemcpy(ptrs[1], U.ctypes.data, U.nbytes, 1) == 0
        st = C.c_void_p()
        assert hip.hipStreamCreate(C.byref(st)) == 0
        assert lib.tog_generic_cost_expand_device(c.ptr, 0, ptrs[0], ptrs[1], cnt, *ptrs[2:], st) == 0
        assert hip.hipStreamSynchronize(st) == 0
        hip.hipStreamDestroy(st)
        outs = [np.empty(sz) for sz in sizes[2:]]
        for o, p in zip(outs, ptrs[2:]):
            assert hip.hipMemcpy(o.ctypes.data, p, o.nbytes, 2) == 0
    finally:
        for p in ptrs:
            hip.hipFree(p)
    J, Ex, Eu = outs[0], outs[1].reshape(cnt, n), outs[2].reshape(cnt, m)
    Exx = outs[3].reshape(cnt, n, n).swapaxes(1, 2)
    Euu = outs[4].reshape(cnt, m, m).swapaxes(1, 2)
    Eux = outs[5].reshape(cnt, n, m).swapaxes(1, 2)
    assert np.isfinite(J).all() and np.isfinite(Exx).all() and np.isfinite(Eux).all()
    assert np.allclose(Exx, Exx.swapaxes(1, 2), rtol=1e-12, atol=1e-12)
    idx = np.random.default_rng(0).choice(cnt, 512, replace=False)
    Jo, Exo, Euo, Exxo, Euuo, Euxo = oracle.generic_cost_expand(1, X[idx], U[idx])
    assert np.array_equal(J[idx], Jo) and np.array_equal(Ex[idx], Exo) and np.array_equal(Eu[idx], Euo)
    assert np.array_equal(Exx[idx], Exxo) and np.array_equal(Euu[idx], Euuo) and np.array_equal(Eux[idx], Euxo)


def test_generic_cost_source_generation(tog):
    """generic_cost() compiles a generated plugin once per source (hash-keyed in-tree cache)."""
    st = "return 0.5 * (x[0] * x[0] + u[0] * u[0]) + cos_(x[1]);"
    tm = "return x[0] * x[0] + x[1] * x[1];"
    c1 = tog.generic_cost(st, tm, 2, 1, name="Quadish")
    c2 = tog.generic_cost(st, tm, 2, 1, name="Quadish")
    assert c1.ptr == c2.ptr and c1.sizes() == (2, 1)
    assert pathlib.Path(c1.path).parent == PLUG and pathlib.Path(c1.path).name.startswith("gen_Quadish_")
    with pytest.raises(ValueError):
        tog.generic_cost("return undefined_symbol;", tm, 2, 1, name="Broken")
