"""MFMA A/B for the backward pass's dense products (north_star "MFMA only for the
quadrotor/Kuka-sized dense Q-block contractions").

The one-wave-per-trajectory backward kernel (k_backward, matrices in LDS) computes S·[A B], (S B)ᵀ(S A),
AᵀS A, … with the wave-level product wmm. Built with -DTOG_MFMA, wmm runs on the fp64 matrix cores
(v_mfma_f64_16x16x4_f64). This script, run on the GPU box once per build with TOG_BWD=lds, reports:
  * step level: max relative error of K, d, ΔV against the CPU oracle (Kuka, config 5 options, and the
    quadrotor, config 3 options; sqrt and std backward passes);
  * solve level: per trajectory, X/U within 1e-6 of the oracle and the same iteration count;
  * time: the backward kernel's average duration over a bench window (HIP events, tog_profile).

    TOG_BWD=lds TOG_LIBRARY=build_ab/mfma/libtog.so python tools/mfma_ab.py mfma
    TOG_BWD=lds python tools/mfma_ab.py lds-valu
    python tools/mfma_ab.py team-valu
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()
orc = __graft_entry__.load_oracle()
abi = pkg.abi


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b))))


def step_level(name, prob, opts, sqrt):
    il = pkg.iLQRSolverOptions(square_root=sqrt)
    al_opts = pkg.AugmentedLagrangianSolverOptions(opts_uncon=il)
    h = pkg.AbstractSolverFor(prob, al_opts).handle
    h.rollout_open_loop()
    h.update_constraints()
    h.jacobians()
    dV = h.backward_pass(sqrt=sqrt, al=True)
    K, d = h.get(abi.FIELD_K), h.get(abi.FIELD_D)
    err = 0.0
    for b in range(prob.B):
        o = orc.OracleSolver(prob, al_opts, b=b)
        o.rollout_open_loop()
        o.update_constraints()
        o.jacobians()
        o.cost_expansion(sqrt, True)
        dV_ref, _ = o.backward(sqrt)
        err = max(err, rel(K[b], o.get("K")), rel(d[b], o.get("d")), rel(dV[b], dV_ref))
    return {"case": name, "sqrt": sqrt, "max_rel_err": err}


def solve_level(name, prob, opts):
    ref = prob.copy()
    s = pkg.solve_b(prob, opts)
    ok = same_iters = 0
    worst = 0.0
    for b in range(prob.B):
        o = orc.OracleSolver(ref, opts, b=b)
        o.solve()
        e = max(rel(prob._X[b], o.get("X")), rel(prob._U[b], o.get("U")))
        worst = max(worst, e)
        ok += e < 1e-6
        same_iters += int(s.stats["iterations_total"][b]) == int(o.get("stats")[abi.STAT_TOTAL_STEPS])
    return {"case": name, "B": prob.B, "within_1e-6": ok, "same_iterations": same_iters, "max_rel_err": worst}


def bwd_time(name, cfg, B, steps=10):
    prob, opts = getattr(pkg.Problems, cfg)(B=B)
    h = pkg.AbstractSolverFor(prob, opts).handle
    h.solve_init(abi.MODE_AL)
    h.solve_step(2)
    h.synchronize()
    h.profile(True)
    h.solve_step(steps)
    h.synchronize()
    ms, launches = h.profile_read()
    h.profile(False)
    return {"case": name, "B": B, "backward_ms": float(ms[1] / max(1, launches[1]))}


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "run"
    out = {"label": label, "TOG_BWD": os.environ.get("TOG_BWD"), "TOG_LIBRARY": os.environ.get("TOG_LIBRARY"),
           "step": [], "solve": [], "time": []}
    pk, ok = pkg.Problems.config_kuka(B=3)
    pq, oq = pkg.Problems.config_quadrotor(B=3)
    for sq in (False, True):
        out["step"].append(step_level("kuka", pk, ok, sq))
        out["step"].append(step_level("quadrotor", pq, oq, sq))
    pk8, ok8 = pkg.Problems.config_kuka(B=8)
    out["solve"].append(solve_level("kuka", pk8, ok8))
    pq8, oq8 = pkg.Problems.config_quadrotor(B=8)
    out["solve"].append(solve_level("quadrotor", pq8, oq8))
    out["time"].append(bwd_time("kuka", "config_kuka", 4096))
    out["time"].append(bwd_time("quadrotor", "config_quadrotor", 8192))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
