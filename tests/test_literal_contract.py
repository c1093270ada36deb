"""How far the arithmetic contract moves results from the reference's literal arithmetic
(VERDICT r3 #2). The oracle is built twice: liboracle.so (the contract the HIP kernels reproduce bit
for bit) and liboracle_literal.so (-DTOG_ORACLE_LITERAL): LAPACK dgeqr2/dlarfg Householder QR with plain
sums, lowrankdowndate! with its sqrt and divisions (backward_pass.jl:186-192), substitution by division
(backward_pass.jl:141-142,148), ForwardDiff straight through the Kuka's RK3 step (src/model.jl:491-522).

Findings pinned here (profiles/r4_literal_vs_contract.txt holds the full report, tools/literal_report.py):
* step level the two agree to rounding times conditioning (config 3's first backward pass: K, d within
  4e-9 relative, ΔV 1e-15; the reference's own car fixture, sqrt_bp_tests.jl, far tighter);
* config 3's solves are chaotic: moving one input by one ulp (x0[1] + 1 ulp, contract build) changes the
  per-trajectory iteration counts as much as switching the arithmetic does, and the costs leave 1e-6
  agreement after a handful of iterations in both comparisons. So no implementation with different
  rounding (the reference on another BLAS included) reproduces config 3's per-trajectory iterates; what
  carries over is the batch behaviour (convergence, medians), asserted below, and the per-trajectory
  parity of well-conditioned solves (the notebook pins, in literal mode too)."""
import json
import pathlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))) / max(1.0, float(np.max(np.abs(b)))))


def _first_backward(oracle, prob, opts, b, literal, sqrt, al):
    o = oracle.OracleSolver(prob, opts, b=b, literal=literal)
    o.rollout_open_loop()
    if al:
        o.update_constraints()
    o.jacobians()
    assert o.cost_expansion(sqrt, al) == 0
    dV, _ = o.backward(sqrt)
    return dV, o.get("K"), o.get("d"), o.get("S")


def test_step_level_config3(tog, oracle):
    prob, opts = tog.Problems.config_quadrotor(B=8)
    worst = np.zeros(4)
    for b in range(prob.B):
        c = _first_backward(oracle, prob, opts, b, False, True, True)
        lt = _first_backward(oracle, prob, opts, b, True, True, True)
        worst = np.maximum(worst, [rel(x, y) for x, y in zip(c, lt)])
    assert worst[0] < 1e-13          # ΔV
    assert worst[1] < 1e-7 and worst[2] < 1e-7 and worst[3] < 1e-7  # K, d, S (cond(Quu) up to 1e8)


@pytest.mark.parametrize("constrained", [False, True])
def test_step_level_reference_car_fixture(tog, oracle, constrained):
    """test/sqrt_bp_tests.jl's car problem (rk4, N = 31, U = ones; unconstrained and AL): the
    well-conditioned fixture the reference pins std ≡ sqrt on; literal and contract sqrt passes agree
    within 1e-11 (2.3e-12 measured; the reference's own std ≡ sqrt tolerance is √eps)."""
    prob = tog.Problems.car_sqrt_bp(constrained=constrained)
    opts = tog.AugmentedLagrangianSolverOptions() if constrained else tog.iLQRSolverOptions()
    c = _first_backward(oracle, prob, opts, 0, False, True, constrained)
    lt = _first_backward(oracle, prob, opts, 0, True, True, constrained)
    for x, y in zip(c, lt):
        assert rel(x, y) < 1e-11


def test_kuka_jacobian_chain_vs_dual(tog, oracle):
    """The Kuka's stage-chain Jacobian (contract) against ForwardDiff through the RK3 step (literal)."""
    L = oracle.lib()
    import ctypes as C
    dp = C.POINTER(C.c_double)
    L.oc_discrete_jacobian_fd.argtypes = [C.c_int, C.c_int, dp, dp, dp, C.c_double]
    rng = np.random.default_rng(5)
    for _ in range(50):
        x = np.concatenate([rng.uniform(-1, 1, 7), rng.uniform(-0.5, 0.5, 7)])
        u = rng.uniform(-5, 5, 7)
        S = oracle.discrete_jacobian(5, 0, x, u, 0.1)
        F = np.empty((22, 14))
        L.oc_discrete_jacobian_fd(5, 0, F.ctypes.data_as(dp), x.ctypes.data_as(dp), u.ctypes.data_as(dp), 0.1)
        F = F.T
        assert np.abs(S[:, :21] - F[:, :21]).max() / np.abs(F[:, :21]).max() < 1e-12


def test_notebook_pins_in_literal_mode(tog, oracle):
    """The reference-held outputs hold for the literal build as well: the Kuka notebook's 23-iterate log
    (Kuka iiwa.ipynb cell 16, ForwardDiff through RK3 here) and the quadrotor notebook's final cost."""
    log = json.loads((ROOT / "tests" / "golden" / "kuka_notebook_log.json").read_text())
    prob, opts = tog.Problems.kuka(), tog.Problems.kuka_options()
    o = oracle.OracleSolver(prob, opts, b=0, literal=True)
    assert o.solve() == len(log["inner"]) == 23
    for row, ref in zip(o.trace(), log["inner"]):
        assert abs(row[0] - ref["cost"]) <= 1e-9 * ref["cost"] + 5e-9
        assert row[1] == ref["alpha"]
    from test_reference_kats import _notebook_quadrotor
    s = oracle.OracleSolver(_notebook_quadrotor(tog), tog.iLQRSolverOptions(), literal=True)
    s.solve()
    assert abs(s.get("stats")[tog.abi.STAT_J] - 18.17292526) / 18.17292526 < 5e-6


@pytest.mark.timeout(900)
def test_config3_batch_statistics_literal_vs_contract(tog, oracle):
    """32 seeded config-3 trajectories solved in both builds and, as the control, in the contract build
    with x0[1] moved by one ulp. Per trajectory the solves part ways after a few iterations in both
    comparisons (chaotic): the one-ulp control itself leaves 1e-6 cost agreement within a dozen
    iterations (median; 7.5 measured), the literal build a few iterations earlier (5: it injects a
    rounding difference at every step, the control only once). The batch agrees: every trajectory
    converges in both builds up to one, and the median iteration counts are within 15 %."""
    abi = tog.abi
    B = 32
    prob, opts = tog.Problems.config_quadrotor(B=B)
    p1 = prob.copy()
    p1.x0[:, 0] = np.nextafter(p1.x0[:, 0], np.inf)
    runs = [(prob, False), (prob, True), (p1, False)]

    def solve(a):
        r, b = a
        o = oracle.OracleSolver(runs[r][0], opts, b=b, literal=runs[r][1])
        steps = o.solve()
        return steps, int(o.get("stats")[abi.STAT_FLAGS]), o.trace()

    args = [(r, b) for r in range(3) for b in range(B)]
    with ThreadPoolExecutor(8) as ex:
        res = dict(zip(args, ex.map(solve, args)))

    def first_div(ta, tb):
        n = min(len(ta), len(tb))
        return next((i for i in range(n) if abs(ta[i][0] - tb[i][0]) > 1e-6 * abs(tb[i][0])), n)

    its = [np.array([res[(r, b)][0] for b in range(B)]) for r in range(3)]
    conv = [sum((res[(r, b)][1] & abi.TRAJ_AL_CONVERGED) != 0 for b in range(B)) for r in range(3)]
    assert conv[0] >= B - 1 and conv[1] >= B - 1
    assert abs(np.median(its[1]) - np.median(its[0])) <= 0.15 * np.median(its[0])
    div_lit = np.median([first_div(res[(0, b)][2], res[(1, b)][2]) for b in range(B)])
    div_ulp = np.median([first_div(res[(0, b)][2], res[(2, b)][2]) for b in range(B)])
    assert div_ulp <= 12, div_ulp       # per-trajectory iterates do not survive a one-ulp input change
    assert div_lit >= 3, div_lit        # the first iterations agree with the literal arithmetic to 1e-6
