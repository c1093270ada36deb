"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

There are no golden trajectories in the reference and no Julia to run it,
so the fixtures come from oracle/tog_oracle.c *after* it has passed the reference's own assertions
(tests/test_reference_kats.py: sqrt_bp_tests, constraint/cost/utils KATs, quadrotor/car/pendulum
convergence thresholds). They pin the oracle against regressions and give the GPU tests a fixed
contract. Inputs are stored alongside outputs, so every case is reproducible from the file alone.

    python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))

import __graft_entry__  # noqa: E402

tog = __graft_entry__.load_package()
oracle = __graft_entry__.load_oracle()

MODELS = [("doubleintegrator", "rk3"), ("pendulum", "rk4"), ("car", "rk3"), ("car", "rk4"), ("cartpole", "rk3"),
          ("quadrotor", "rk3"), ("quadrotor", "rk4")]


def jacobians():
    out = {}
    for name, integ in MODELS:
        model = getattr(tog.Dynamics, name)
        ig = tog.abi.RK4 if integ == "rk4" else tog.abi.RK3
        rng = np.random.default_rng(11)
        xs, us, Ss = [], [], []
        for _ in range(4):
            x = 0.5 * rng.standard_normal(model.n)
            if name == "quadrotor":
                x[3:7] += [1.0, 0, 0, 0]
            u = 0.5 * rng.standard_normal(model.m)
            xs.append(x)
            us.append(u)
            Ss.append(oracle.discrete_jacobian(model.model_id, ig, x, u, 0.05))
        out[f"{name}_{integ}_x"] = np.array(xs)
        out[f"{name}_{integ}_u"] = np.array(us)
        out[f"{name}_{integ}_S"] = np.array(Ss)
    np.savez_compressed(HERE / "jacobians.npz", **out)


def backward_passes():
    """test/sqrt_bp_tests.jl setups: one rollout + jacobians + expansion + backward pass."""
    out = {}
    for constrained in (False, True):
        for sq in (False, True):
            prob = tog.Problems.car_sqrt_bp(constrained=constrained)
            ilqr = tog.iLQRSolverOptions(square_root=sq)
            opts = tog.AugmentedLagrangianSolverOptions(opts_uncon=ilqr) if constrained else ilqr
            s = oracle.OracleSolver(prob, opts)
            s.rollout_open_loop()
            if constrained:
                s.update_constraints()
            s.jacobians()
            s.cost_expansion(sqrt=sq, al=constrained)
            dV, _ = s.backward(sqrt=sq)
            key = f"car_{'al' if constrained else 'uncon'}_{'sqrt' if sq else 'std'}"
            out[key + "_X"] = s.get("X")
            out[key + "_K"] = s.get("K")
            out[key + "_d"] = s.get("d")
            out[key + "_dV"] = dV
            out[key + "_S"] = s.get("S")
            out[key + "_Sx"] = s.get("Sx")
    np.savez_compressed(HERE / "backward.npz", **out)


def solves():
    """Full solves on seeded batched inputs (BASELINE configs 1-3 at small B, plus pendulum)."""
    out = {}
    cases = {
        "cartpole": tog.Problems.config_cartpole(B=2),
        "quadrotor": tog.Problems.config_quadrotor(B=2),
        "doubleintegrator": tog.Problems.config_doubleintegrator(),
        "pendulum": (tog.Problems.pendulum("rk3"),
                     tog.ALTROSolverOptions(opts_al=tog.AugmentedLagrangianSolverOptions(iterations=50))),
    }
    for name, (prob, opts) in cases.items():
        Xs, Us, Js, its = [], [], [], []
        for b in range(prob.B):
            s = oracle.OracleSolver(prob, opts, b)
            s.solve()
            st = s.get("stats")
            Xs.append(s.get("X"))
            Us.append(s.get("U"))
            Js.append(st[tog.abi.STAT_J])
            its.append(st[tog.abi.STAT_TOTAL_STEPS])
        out[name + "_x0"] = prob.x0
        out[name + "_U0"] = prob._U
        out[name + "_X"] = np.array(Xs)
        out[name + "_U"] = np.array(Us)
        out[name + "_J"] = np.array(Js)
        out[name + "_steps"] = np.array(its)
    np.savez_compressed(HERE / "solves.npz", **out)


def quad_maze_n201():
    """BASELINE config 4 at its own horizon (quad_obs, N=201, dt=0.025): the first 4 seeded starts
    of ``config_quad_maze`` (seeds 3000+b) solved by AL-iLQR. Two converge, two exhaust the AL
    iterations (c_max > 1), which pins the failure path too. Stats: J, c_max, total steps, flags."""
    prob, opts = tog.Problems.config_quad_maze(B=4, N=201)
    Xs, Us, st = [], [], []
    for b in range(prob.B):
        s = oracle.OracleSolver(prob, opts, b)
        s.solve()
        Xs.append(s.get("X"))
        Us.append(s.get("U"))
        st.append(s.get("stats"))
    np.savez_compressed(HERE / "quad_maze_n201.npz", x0=prob.x0, U0=prob._U, X=np.array(Xs), U=np.array(Us),
                        stats=np.array(st))


if __name__ == "__main__":
    if sys.argv[1:] == ["quad_maze"]:
        quad_maze_n201()
        sys.exit(0)
    jacobians()
    backward_passes()
    solves()
    quad_maze_n201()
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)
