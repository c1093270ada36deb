"""The reference's IROS 2019 quadrotor maze demo (examples/IROS_2019/quadrotor_maze.jl:23-48: ALTRO with projected
Newton from the maze way-point guess) as a batch on the device, timed.

    python tools/iros_maze.py [--batch B] [--jitter 0.5] [--out file.json]

Trajectory 0 starts from the reference's own guess (problems/quadrotor_maze.jl:104-113), the others from
way-points jittered by N(0, jitter^2). One solve_b of the whole batch (infeasible-start AL phase, projected
Newton on the infeasible problem, process_results!); wall time, phase times, and per-trajectory outcomes:
final max violation, AL outer iterations, the reference's _projection_linesearch! exception
(TRAJ_PN_ERROR). The reference publishes 85.8 s and 9.63e-9 for one solve (examples/quadrotor/Quadrotor
Maze.ipynb, cell 3) on a CPU: context, not a like-for-like baseline."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--jitter", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tog = __graft_entry__.load_package()
    B = a.batch
    prob = tog.Problems.quadrotor_maze_batch(B, jitter=a.jitter)
    prob._X[0] = tog.Problems.quadrotor_maze_batch(1, jitter=0.0)._X[0]
    # warm-up: one small solve (module loading, first-launch costs)
    w = tog.Problems.quadrotor_maze_batch(2, offset=10_000)
    try:
        tog.solve_b(w, tog.Problems.quadrotor_maze_iros_options(), history=False)
    except tog.ProjectedNewtonError:
        pass
    opts = tog.Problems.quadrotor_maze_iros_options()
    t0 = time.perf_counter()
    try:
        solver, raised = tog.solve_b(prob, opts, history=False), []
    except tog.ProjectedNewtonError as e:
        solver, raised = e.solver, list(e.trajectories)
    wall = time.perf_counter() - t0
    c_max = np.asarray(solver.stats_pn["c_max"], dtype=float)
    flags = np.asarray(solver.stats_pn["flags"])
    err = (flags & tog.abi.TRAJ_PN_ERROR) != 0
    iters = np.asarray(solver.stats["iterations_total"])
    line = {
        "what": "IROS 2019 quadrotor maze, ALTRO + projected Newton (examples/IROS_2019/quadrotor_maze.jl:23-48)",
        "batch": B, "jitter": a.jitter, "wall_s": round(wall, 4),
        "time_al_s": round(float(solver.stats["time_al"]), 4), "time_pn_s": round(float(solver.stats["time_pn"]), 4),
        "per_trajectory_ms": round(1e3 * wall / B, 4),
        "reference_start": {"c_max": float(c_max[0]), "pn_error": bool(err[0]), "al_iterations": int(iters[0])},
        "feasible_1e-8": int(np.count_nonzero((c_max <= 1e-8) & ~err)),
        "pn_error_reference_exception": int(np.count_nonzero(err)),
        "c_max_median": float(np.median(c_max)), "al_iterations_total": int(iters.sum()),
        "al_iterations_max": int(iters.max()),
        "reference_published": {"seconds": 85.8, "c_max": 9.63e-9, "note": "one solve on a CPU (notebook): context only"},
    }
    print(json.dumps(line))
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(line, indent=1) + "\n")


if __name__ == "__main__":
    main()
