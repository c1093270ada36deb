"""How far the arithmetic contract moves the solves from the reference's literal arithmetic.

Runs the CPU oracle in its two builds — liboracle.so (the contract the HIP kernels reproduce bit for
bit) and liboracle_literal.so (-DTOG_ORACLE_LITERAL: dgeqr2/dlarfg Householder QR, lowrankdowndate!
with sqrt and divisions, substitution by division, ForwardDiff through the Kuka's RK3 step) — on:
  1. the first backward pass of config 3 (step level: K, d, ΔV, S);
  2. config 3's eight full-batch picks (trajectories 0-3, the slowest one, three that end without AL
     convergence; tests/test_config3_full.py) solved to completion in both builds;
  3. a 64-trajectory batch in both builds and, as a control, the contract build with x0[1] moved by one
     ulp: per-trajectory iteration counts, the first iteration whose cost differs by more than 1e-6
     relative, batch medians and convergence.
  python tools/literal_report.py > profiles/r4_literal_vs_contract.txt
"""
import pathlib
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__  # noqa: E402

tog = __graft_entry__.load_package()
orc = __graft_entry__.load_oracle()
abi = tog.abi
PICKS = [0, 1, 2, 3, 1457, 236, 1023, 1174]


def first_div(ta, tb, rel=1e-6):
    n = min(len(ta), len(tb))
    return next((i for i in range(n) if abs(ta[i][0] - tb[i][0]) > rel * abs(tb[i][0])), None)


def solve(prob, opts, b, literal):
    o = orc.OracleSolver(prob, opts, b=b, literal=literal)
    steps = o.solve()
    st = o.get("stats")
    return steps, int(st[abi.STAT_FLAGS]), o.get("X"), o.get("U"), o.trace()


def step_level(B=8):
    prob, opts = tog.Problems.config_quadrotor(B=B)
    worst = {}
    for b in range(B):
        res = []
        for lit in (False, True):
            o = orc.OracleSolver(prob, opts, b=b, literal=lit)
            o.rollout_open_loop()
            o.update_constraints()
            o.jacobians()
            assert o.cost_expansion(True, True) == 0
            dV, _ = o.backward(True)
            res.append({"dV": dV, "K": o.get("K"), "d": o.get("d"), "S": o.get("S")})
        for k in res[0]:
            a, c = res[0][k], res[1][k]
            worst[k] = max(worst.get(k, 0.0), float(np.max(np.abs(a - c)) / max(1.0, np.max(np.abs(c)))))
    return worst


def main():
    print("# literal (reference arithmetic) vs contract (device arithmetic), CPU oracle, config 3 (AL-iLQR, sqrt BP)")
    w = step_level()
    print("step level, first backward pass, B = 8, max relative difference:",
          ", ".join(f"{k} {v:.2e}" for k, v in w.items()))
    prob, opts = tog.Problems.config_quadrotor(B=max(PICKS) + 1)
    with ThreadPoolExecutor(8) as ex:
        R = dict(zip([(b, l) for b in PICKS for l in (False, True)],
                     ex.map(lambda a: solve(prob, opts, *a), [(b, l) for b in PICKS for l in (False, True)])))
    print("\nfull-batch picks (solved to completion in both builds):")
    print("traj | iterations contract / literal | flags contract / literal | X, U rel. diff | first iter |ΔJ| > 1e-6 J")
    for b in PICKS:
        sc, fc, Xc, Uc, tc = R[(b, False)]
        sl, fl, Xl, Ul, tl = R[(b, True)]
        ex_ = np.abs(Xc - Xl).max() / max(1.0, np.abs(Xl).max())
        eu = np.abs(Uc - Ul).max() / max(1.0, np.abs(Ul).max())
        print(f"{b:5d} | {sc:5d} / {sl:5d} | {fc:4d} / {fl:4d} | {ex_:.1e}, {eu:.1e} | {first_div(tc, tl)}")
    B = 64
    prob, opts = tog.Problems.config_quadrotor(B=B)
    p1 = prob.copy()
    p1.x0[:, 0] = np.nextafter(p1.x0[:, 0], np.inf)
    runs = [(prob, False), (prob, True), (p1, False)]
    args = [(r, b) for r in range(3) for b in range(B)]
    with ThreadPoolExecutor(8) as ex:
        out = list(ex.map(lambda a: solve(runs[a[0]][0], opts, a[1], runs[a[0]][1]), args))
    res = {a: o for a, o in zip(args, out)}
    names = ["contract", "literal", "contract, x0[1] + 1 ulp"]
    print(f"\nbatch of {B} (seeded config-3 starts):")
    for r in range(3):
        its = np.array([res[(r, b)][0] for b in range(B)])
        conv = sum((res[(r, b)][1] & abi.TRAJ_AL_CONVERGED) != 0 for b in range(B))
        print(f"  {names[r]:26s} iterations mean {its.mean():7.1f} median {np.median(its):5.0f} max {its.max():5d};"
              f" AL-converged {conv}/{B}")
    for r in (1, 2):
        same = sum(res[(0, b)][0] == res[(r, b)][0] for b in range(B))
        fd = [first_div(res[(0, b)][4], res[(r, b)][4]) for b in range(B)]
        fdn = [f for f in fd if f is not None]
        print(f"  contract vs {names[r]}: same iteration count {same}/{B}; costs within 1e-6 throughout "
              f"{fd.count(None)}/{B}; first divergence median {np.median(fdn):.0f} (min {min(fdn)}, max {max(fdn)})")


if __name__ == "__main__":
    main()
