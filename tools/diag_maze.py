"""Diagnostic: step-level GPU vs oracle on the quadrotor_maze infeasible problem (69 rows/knot)."""
import sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as g
tog = g.load_package(); orc = g.load_oracle(); abi = tog.abi


def rel(a, b):
    a = np.asarray(a, float); b = np.asarray(b, float)
    return float(np.nanmax(np.abs(a - b))) / max(1.0, float(np.nanmax(np.abs(b))))


p = tog.Problems.quadrotor_maze()
pinf = tog.infeasible_problem(p, 0.001)
il = tog.iLQRSolverOptions(square_root=len(sys.argv) > 1 and sys.argv[1] == "sqrt")
opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=il)
s = tog.AugmentedLagrangianSolver(pinf, opts)
h = s.handle
h.slack_controls()
o = orc.OracleSolver(pinf, opts)
o.slack_controls()
print("U", rel(h.get(abi.FIELD_U)[0], o.get("U")))
h.update_constraints(); o.update_constraints()
Cg, Co = h.get(abi.FIELD_C)[0], o.get("C")
print("C", rel(Cg, Co), "pmax", h.pmax, o.pmax)
Jg = h.cost(al=True)[0]; Jo = o.cost(True)
print("J", Jg, Jo)
h.jacobians(); o.jacobians()
print("A", rel(h.get(abi.FIELD_A)[0], o.get("A")), "B", rel(h.get(abi.FIELD_B)[0], o.get("B")))
sq = il.square_root
dV = h.backward_pass(sqrt=sq, al=True)[0]
assert o.cost_expansion(sq, True) == 0
dVo, _ = o.backward(sq)
K, d = h.get(abi.FIELD_K)[0], h.get(abi.FIELD_D)[0]
Ko, do = o.get("K"), o.get("d")
print("dV", dV, dVo)
print("K", rel(K, Ko), "d", rel(d, do))
bad = [k for k in range(p.N - 1) if rel(K[k], Ko[k]) > 1e-12 or rel(d[k], do[k]) > 1e-12]
print("first bad knots", bad[-5:] if bad else None)
if bad:
    k = bad[-1]
    print("d gpu", d[k]); print("d orc", do[k])
# forward pass from the same K, d
h.rollout(1.0); ok = o.rollout(1.0)
print("rollout a=1 ok", ok, "Xbar", rel(h.get(abi.FIELD_XBAR)[0], o.get("Xbar")), "Ubar", rel(h.get(abi.FIELD_UBAR)[0], o.get("Ubar")))
Jb = orc.lib().oc_cost_bar(o.s, 1)
print("oracle J(alpha=1)", Jb)
Jf = h.forward_pass(Jo, al=True)[0]
Jof = o.forward(Jo, True)
S = h.get(abi.FIELD_STATS)[0]
print("forward J", Jf, Jof, "gpu alpha", S[abi.STAT_ALPHA], "trials", S[abi.STAT_LS_TRIALS], "oracle stats", o.get("stats")[[abi.STAT_ALPHA, abi.STAT_LS_TRIALS, abi.STAT_Z]])
# solve path: init + one step, compare the gains with the step-level ones
s2 = tog.AugmentedLagrangianSolver(pinf, opts)
h2 = s2.handle
h2.slack_controls()
print("U2", rel(h2.get(abi.FIELD_U)[0], o.get("U")))
h2.solve_init(abi.MODE_AL)
S = h2.get(abi.FIELD_STATS)[0]
print("init J", S[abi.STAT_J], "Jo", Jo, "C", rel(h2.get(abi.FIELD_C)[0], Co), "X", rel(h2.get(abi.FIELD_X)[0], pinf.X))
print("lam", np.abs(h2.get(abi.FIELD_LAMBDA)[0]).max(), "mu", h2.get(abi.FIELD_MU)[0].min(), h2.get(abi.FIELD_MU)[0].max())
h2.solve_step(1)
K2, d2 = h2.get(abi.FIELD_K)[0], h2.get(abi.FIELD_D)[0]
print("solve-step K", rel(K2, Ko), "d", rel(d2, do), "dV", h2.get(abi.FIELD_DV)[0])
S = h2.get(abi.FIELD_STATS)[0]
print("after step J", S[abi.STAT_J], "alpha", S[abi.STAT_ALPHA], "trials", S[abi.STAT_LS_TRIALS])
