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
        flag = "" if dJ < 1e-9 and r[1]==t[1] and r[4]==t[4] else "  <--"
        if flag and first_bad is None: first_bad = i
        if i < 5 or flag or i % 10 == 0 or 15 <= i <= 25:
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
elif which == "mt_kuka":
    sys.path.insert(0, str(ROOT / "tests"))
    from test_minimum_time import _mt_model_case
    prob, opts = _mt_model_case(tog, "kuka")
    # Jacobians at the initial rollout, device vs oracle
    o = orc.OracleSolver(prob, opts, b=0)
    o.rollout_open_loop(); o.jacobians()
    s = tog.AbstractSolverFor(prob.copy(), opts)
    h = s.handle
    h.rollout_open_loop(); h.jacobians()
    for f, nm in ((abi.FIELD_A, "A"), (abi.FIELD_B, "B"), (abi.FIELD_X, "X")):
        d = h.get(f)[0]
        r = o.get(nm)
        print(nm, "finite", np.isfinite(d).all(), "max|diff|", np.nanmax(np.abs(d - r)), "nan at", np.argwhere(~np.isfinite(d))[:3].tolist())
    trace(prob, opts, b=0)
elif which == "mt_kuka_ls":
    # the line search of step 20 (index 19) of the min-time Kuka case, trial by trial, device vs oracle,
    # from the same state (the device's after 19 steps, which equals the oracle's bit for bit)
    sys.path.insert(0, str(ROOT / "tests"))
    from test_minimum_time import _mt_model_case
    prob, opts = _mt_model_case(tog, "kuka")
    s = tog.AbstractSolverFor(prob.copy(), opts)
    h = s.handle
    h.solve_init(abi.MODE_AL)
    for i in range(19):
        h.solve_step(1)
    st = {f: h.get(f, raw=True) for f in (abi.FIELD_X, abi.FIELD_U, abi.FIELD_LAMBDA, abi.FIELD_MU, abi.FIELD_RHO)}
    S = h.get(abi.FIELD_STATS)[0]
    print("after 19 steps: J", S[abi.STAT_J], "iters", S[abi.STAT_ITERATIONS])
    o = orc.OracleSolver(prob, opts, b=0)
    for f, nm in ((abi.FIELD_X, "X"), (abi.FIELD_U, "U"), (abi.FIELD_LAMBDA, "lambda"), (abi.FIELD_MU, "mu"), (abi.FIELD_RHO, "rho")):
        o.set(nm, st[f][0])
    h2 = tog.AbstractSolverFor(prob.copy(), opts).handle
    for f in st:
        h2.set(f, st[f] if f not in (abi.FIELD_X, abi.FIELD_U) else st[f])
    h2.update_constraints(); o.update_constraints()
    print("J_al device", h2.cost(al=True)[0], "oracle", o.cost(True))
    h2.jacobians(); o.jacobians()
    print("A diff", np.nanmax(np.abs(h2.get(abi.FIELD_A)[0] - o.get("A"))), "B diff", np.nanmax(np.abs(h2.get(abi.FIELD_B)[0] - o.get("B"))))
    dV = h2.backward_pass(sqrt=False, al=True)[0]
    assert o.cost_expansion(False, True) == 0
    dVo, r = o.backward(False)
    print("dV", dV, dVo, "restarts", r, "K diff", np.nanmax(np.abs(h2.get(abi.FIELD_K)[0] - o.get("K"))),
          "d diff", np.nanmax(np.abs(h2.get(abi.FIELD_D)[0] - o.get("d"))))
    for j in range(12):
        a = 2.0 ** -j
        okd = h2.rollout(a)[0]
        oko = o.rollout(a)
        Jd = h2.cost(al=True)[0] if False else None
        Xd, Ud = h2.get(abi.FIELD_XBAR)[0], h2.get(abi.FIELD_UBAR)[0]
        Xo, Uo = o.get("Xbar"), o.get("Ubar")
        Jo = o.cost_bar(True)
        print(f"alpha {a:.4g}: ok dev {okd} orc {oko}; Xbar diff {np.nanmax(np.abs(Xd - Xo)):.3e} finite dev {np.isfinite(Xd).all()} orc {np.isfinite(Xo).all()};"
              f" max|x| dev {np.nanmax(np.abs(Xd)):.3e}; nan X at {np.argwhere(~np.isfinite(Xd))[:2].tolist()}; Ubar diff {np.nanmax(np.abs(Ud - Uo)):.3e}; J orc {Jo:.6e}")
elif which == "mt_kuka_trials":
    # the speculative trials of the failing step (index 19): device J / ok per trial vs the oracle's rollouts
    import ctypes as C
    sys.path.insert(0, str(ROOT / "tests"))
    from test_minimum_time import _mt_model_case
    prob, opts = _mt_model_case(tog, "kuka")
    s = tog.AbstractSolverFor(prob.copy(), opts)
    h = s.handle
    h.solve_init(abi.MODE_AL)
    for i in range(19):
        h.solve_step(1)
    st0 = {f: h.get(f, raw=True) for f in (abi.FIELD_X, abi.FIELD_U, abi.FIELD_LAMBDA, abi.FIELD_MU, abi.FIELD_RHO)}
    S0 = h.get(abi.FIELD_STATS)[0]
    h.solve_step(1)
    nc = C.c_int32()
    J = np.zeros(64); ok = np.zeros(64, dtype=np.int32)
    h.lib.tog__debug_ls(h.h, J.ctypes.data_as(C.POINTER(C.c_double)), ok.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(nc))
    S1 = h.get(abi.FIELD_STATS)[0]
    print("J_prev", S0[abi.STAT_J], "-> J", S1[abi.STAT_J], "alpha", S1[abi.STAT_ALPHA], "trials", S1[abi.STAT_LS_TRIALS], "nc", nc.value)
    o = orc.OracleSolver(prob, opts, b=0)
    for f, nm in ((abi.FIELD_X, "X"), (abi.FIELD_U, "U"), (abi.FIELD_LAMBDA, "lambda"), (abi.FIELD_MU, "mu"), (abi.FIELD_RHO, "rho")):
        o.set(nm, st0[f][0])
    o.update_constraints(); o.jacobians()
    assert o.cost_expansion(False, True) == 0
    o.backward(False)
    for j in range(nc.value):
        a = 2.0 ** -j
        oko = o.rollout(a)
        Jo = o.cost_bar(True) if oko else float("nan")
        print(f"trial {j:2d} alpha {a:.4g}: device ok {ok[j]} J {J[j]:.10e} | oracle ok {int(oko)} J {Jo:.10e}")
