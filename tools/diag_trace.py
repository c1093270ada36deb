"""Diagnostic: per-step trace of one trajectory, GPU vs oracle (J, alpha, rho, restarts, trials)."""
import sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as g
tog = g.load_package(); orc = g.load_oracle(); abi = tog.abi

def trace(prob, opts, b=0, nsteps=200, slack=False):
    o = orc.OracleSolver(prob, opts, b=b)
    if slack:
        o.slack_controls()
    steps = o.solve()
    tr = o.trace()
    p1 = prob.copy(); p1.x0 = prob.x0[b:b+1].copy(); p1._X = prob._X[b:b+1].copy(); p1._U = prob._U[b:b+1].copy(); p1.batched = True
    s = tog.AbstractSolverFor(p1, opts)
    h = s.handle
    mode = abi.MODE_AL if isinstance(opts, (tog.AugmentedLagrangianSolverOptions, tog.ALTROSolverOptions)) and prob.is_constrained() else abi.MODE_ILQR
    if slack:
        h.slack_controls()
    h.solve_init(mode)
    rows = []
    for i in range(min(nsteps, len(tr))):
        h.solve_step(1)
        S = h.get(abi.FIELD_STATS)[0]
        rho = h.get(abi.FIELD_RHO)[0]
        rows.append((S[abi.STAT_J], S[abi.STAT_ALPHA], rho[0], S[abi.STAT_BP_RESTARTS], S[abi.STAT_LS_TRIALS], S[abi.STAT_AL_ITER], S[abi.STAT_Z]))
    print(f"oracle steps={steps}")
    first_bad = None
    for i, (r, t) in enumerate(zip(rows, tr)):
        dJ = abs(r[0]-t[0])/max(1,abs(t[0]))
        flag = "" if dJ < 1e-9 and r[1]==t[1] and r[3]==t[3] and r[4]==t[4] else "  <--"
        if flag and first_bad is None: first_bad = i
        if i < 5 or flag or i % 10 == 0:
            print(f"{i:4d} GPU J={r[0]:.15e} a={r[1]:.4g} rho={r[2]:.3e} rs={int(r[3])} tr={int(r[4])} al={int(r[5])} z={r[6]:.6g} | ORC J={t[0]:.15e} a={t[1]:.4g} rho={t[2]:.3e} rs={int(t[3])} tr={int(t[4])} z={t[5]:.6g} dJ={dJ:.2e}{flag}")
        if first_bad is not None and i > first_bad + 8: break

which = sys.argv[1] if len(sys.argv) > 1 else "quad"
if which == "quad":
    prob, opts = tog.Problems.config_quadrotor(B=4)
    trace(prob, opts, b=0)
elif which == "obs":
    prob, opts = tog.Problems.config_quad_maze(B=2, N=101)
    trace(prob, opts, b=0)
elif which == "maze_inf":
    prob = tog.Problems.quadrotor_maze()
    il = tog.iLQRSolverOptions(iterations=300)
    al = tog.AugmentedLagrangianSolverOptions(opts_uncon=il, iterations=40, cost_tolerance=1e-5,
                                              cost_tolerance_intermediate=1e-4, constraint_tolerance=1e-3,
                                              penalty_scaling=10.0, penalty_initial=1.0)
    opts = tog.ALTROSolverOptions(resolve_feasible_problem=False, opts_al=al, R_inf=0.001)
    trace(tog.infeasible_problem(prob, opts.R_inf), opts, b=0, slack=True)
