"""Predict config 4's 8-GPU weak scaling on one GPU.

BASELINE.json configs[3] is 65,536 quad_obs starts over 8 GPUs: each rank solves its contiguous shard
(distributed.shard) and the only exchange is the 24-byte statistics all-gather every 4 steps,
so an 8-GPU job's wall time is the slowest shard's solve, and its rate Σ steps ÷ max shard wall. This runs
the 8 shards one after another on one GPU with bench.py's whole-solve leg (time_solve) and reports each
shard's wall time, iterations and slowest trajectory, and the predicted weak-scaling efficiency
(Σ steps ÷ (8 x max wall)) ÷ (shard 0's rate: the N = 1 bench line's workload). A prediction, not a
measured 8-GPU curve.

  python tools/shards_config4.py [--world 8] [--total 65536] > profiles/r5_shards_config4.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--total", type=int, default=65536)
    ap.add_argument("--N", type=int, default=201)
    args = ap.parse_args()
    pkg = __graft_entry__.load_package()
    abi = pkg.abi
    shards = []
    for r in range(args.world):
        offset, count = pkg.distributed.shard(args.total, r, args.world)
        prob, opts = pkg.Problems.config_quad_maze(B=count, offset=offset, N=args.N)
        t0 = time.perf_counter()
        solver = pkg.AbstractSolverFor(prob, opts)
        h = solver.handle
        setup = time.perf_counter() - t0
        leg = bench.time_solve(h, abi, abi.MODE_AL, prob, None, lambda: None, h.synchronize, 0, pkg)
        row = {"rank": r, "offset": offset, "count": count, "setup_s": round(setup, 2), "wall_s": leg["wall_s"],
               "steps": leg["steps"], "rate": leg["value"], "batch_steps": leg["batch_steps"],
               "traj_iterations_max": leg["traj_iterations"]["max"], "converged": leg["converged"],
               "tail_share": leg["tail_share"]}
        shards.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
        del solver, h
    steps = sum(s["steps"] for s in shards)
    wall = max(s["wall_s"] for s in shards)
    job_rate = steps / wall
    one = shards[0]["rate"]
    out = {
        "workload": "quad_obs maze N=%d, AL-iLQR (BASELINE.json configs[3]), %d starts as %d contiguous shards"
                    % (args.N, args.total, args.world),
        "method": "each shard solved alone on one MI355X with bench.py's whole-solve leg, one after another; "
                  "an %d-GPU job runs them concurrently, one per rank, with no data-path collective, so its "
                  "wall time is predicted as the slowest shard's" % args.world,
        "shards": shards,
        "sum_steps": steps,
        "max_wall_s": wall,
        "predicted_job_rate": round(job_rate, 2),
        "shard0_rate": one,
        "predicted_weak_scaling_efficiency": round(job_rate / (args.world * one), 4),
        "note": "prediction from single-GPU shard solves, not a measured multi-GPU curve (DESIGN.md §7)",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
