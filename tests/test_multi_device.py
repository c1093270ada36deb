"""tog_create_multi: one handle over several devices, the batch split into
contiguous slices. On the one-GPU test box the slices share device 0 (devices may repeat), which
exercises the same fan-out, split and gather code; results must equal the single-device handle's
bit for bit, since every trajectory runs the same kernels on the same data."""
import ctypes as C

import numpy as np
import pytest


def test_create_multi_without_device_fails_loudly(tog):
    lib = tog.abi.load_library()
    if lib.tog_device_count() > 0:
        pytest.skip("a HIP device is visible")
    prob, opts = tog.Problems.config_quadrotor(B=4)
    desc = prob.build_desc()
    o = tog.to_tog_options(opts)
    devs = (C.c_int32 * 2)(0, 1)
    h = C.c_void_p()
    rc = lib.tog_create_multi(C.byref(desc.desc), C.byref(o), devs, 2, C.byref(h))
    assert rc == tog.abi.ERR_DEVICE and not h.value
    assert lib.tog_create_multi(C.byref(desc.desc), C.byref(o), devs, 0, C.byref(h)) == tog.abi.ERR_ARG


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_solve_equals_single(tog, gpu, devices):
    prob, opts = tog.Problems.config_quadrotor(B=7)
    p1, p2 = prob.copy(), prob.copy()
    s1 = tog.AugmentedLagrangianSolver(p1, opts)
    s2 = tog.AugmentedLagrangianSolver(p2, opts, devices=devices)
    assert s2.handle.B == 7
    for s, p in ((s1, p1), (s2, p2)):
        s.handle.solve(tog.abi.MODE_AL, max_steps=600)
        s.handle.download_state(p)
    assert np.array_equal(p1._X, p2._X) and np.array_equal(p1._U, p2._U)
    st1, st2 = s1.handle.stats_dict(), s2.handle.stats_dict()
    assert np.array_equal(st1["iterations_total"], st2["iterations_total"])
    assert np.array_equal(s1.handle.status(), s2.handle.status())
    b1, b2 = s1.handle.batch_stats(), s2.handle.batch_stats()
    assert b1[0] == b2[0] and b1[2] == b2[2] and abs(b1[1] - b2[1]) <= 1e-12 * max(1.0, abs(b1[1]))
    assert s1.handle.total_steps() == s2.handle.total_steps()
    for f in (tog.abi.FIELD_LAMBDA, tog.abi.FIELD_MU, tog.abi.FIELD_K, tog.abi.FIELD_A, tog.abi.FIELD_DV):
        assert np.array_equal(s1.handle.get(f), s2.handle.get(f)), f


@pytest.mark.gpu
def test_multi_step_level_equals_single(tog, gpu):
    prob, opts = tog.Problems.config_quadrotor(B=5)
    hs = [tog.AugmentedLagrangianSolver(prob.copy(), opts).handle,
          tog.AugmentedLagrangianSolver(prob.copy(), opts, devices=[0, 0]).handle]
    out = []
    for h in hs:
        h.rollout_open_loop()
        h.update_constraints()
        J = h.cost(al=True)
        h.jacobians()
        dV = h.backward_pass(sqrt=True, al=True)
        Jf = h.forward_pass(J, al=True)
        ok = h.rollout(0.5)
        out.append((J, dV, Jf, ok, h.get(tog.abi.FIELD_XBAR)))
    for a, b in zip(*out):
        assert np.array_equal(a, b)
    # unsupported per-device entry points on a multi-device handle
    vp = C.c_void_p()
    assert hs[1].lib.tog_get_device_ptr(hs[1].h, tog.abi.FIELD_X, C.byref(vp)) == tog.abi.ERR_UNSUPPORTED
    assert hs[1].lib.tog_set_stream(hs[1].h, None) == tog.abi.ERR_UNSUPPORTED
