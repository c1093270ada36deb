"""Solve config 3's slowest trajectory alone and attribute its per-batch-step time.

    python tools/tail_solve.py [--offset 1457] [--chunk 4] [--stats-pass] > out.json

Trajectories are independent and the device arithmetic does not depend on the batch, so trajectory
`offset` of config 3 solved at B = 1 is the headline solve's convergence tail. Timed like bench.py's
solve leg (tog_solve_init, then solve_step(chunk) + the blocking batch_stats readback until nothing
is active). With --stats-pass a second, untimed solve reads the statistics row after every step
(backward-pass restarts, line-search trials, AL outer iteration) to explain the step mix.
Run under `rocprofv3 --kernel-trace` and feed the database to tools/tail_trace.py for gaps.
"""
from __future__ import annotations

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
    ap.add_argument("--offset", type=int, default=1457)
    ap.add_argument("--batch", type=int, default=1, help="B > 1: the headline batch (offset 0 .. B-1)")
    ap.add_argument("--chunk", type=int, default=4)
    ap.add_argument("--stats-pass", action="store_true")
    ap.add_argument("--profile", action="store_true", help="HIP-event per-kernel totals (tog_profile)")
    a = ap.parse_args()
    pkg = __graft_entry__.load_package()
    abi = pkg.abi
    prob, opts = pkg.Problems.config_quadrotor(B=a.batch, offset=a.offset if a.batch == 1 else 0)
    solver = pkg.AbstractSolverFor(prob, opts, device=0)
    h = solver.handle
    out = {"offset": a.offset, "batch": a.batch, "chunk": a.chunk}
    # warm: one short solve so code objects are loaded
    h.solve_init(abi.MODE_AL)
    h.solve_step(4)
    h.synchronize()
    h.upload_state(prob)
    if a.profile:
        h.profile(True)
    h.synchronize()
    t0 = time.perf_counter()
    h.solve_init(abi.MODE_AL)
    done = 0
    while done < 20000:
        h.solve_step(a.chunk)
        done += a.chunk
        if h.batch_stats()[0] == 0.0:
            break
    h.synchronize()
    wall = time.perf_counter() - t0
    steps = h.total_steps()
    out.update({"wall_s": wall, "batch_steps": done, "iterations": steps, "ms_per_batch_step": 1e3 * wall / done})
    if a.profile:
        ms, launches = h.profile_read()
        h.profile(False)
        out["kernel_ms_total"] = dict(zip(["jacobian", "backward", "forward", "expansion"], ms.tolist()))
        out["kernel_launches"] = dict(zip(["jacobian", "backward", "forward", "expansion"], launches.tolist()))
        out["kernel_ms_per_step"] = {k: v / done for k, v in out["kernel_ms_total"].items()}
    if a.stats_pass:
        # untimed: the statistics rows after every batch step (per-step active count, line-search trials)
        h.upload_state(prob)
        h.solve_init(abi.MODE_AL)
        rest, trials, al_iters, per_step = [], [], [], []
        for _ in range(done):
            h.solve_step(1)
            S = h.get(abi.FIELD_STATS)
            act = (S[:, abi.STAT_FLAGS].astype(np.int64) & abi.TRAJ_ACTIVE) != 0
            fin = S[:, abi.STAT_TOTAL_STEPS] > 0
            tr = S[:, abi.STAT_LS_TRIALS]
            per_step.append([int(act.sum()), int(np.count_nonzero(act & (tr >= 21))),
                             int(np.count_nonzero(S[:, abi.STAT_BP_RESTARTS] > 0))])
            if a.batch == 1:
                if not act[0]:
                    break
                rest.append(S[0, abi.STAT_BP_RESTARTS])
                trials.append(S[0, abi.STAT_LS_TRIALS])
                al_iters.append(S[0, abi.STAT_AL_ITER])
            elif not act.any():
                break
        out["per_step"] = per_step  # [n_active after the step, of them with 21 trials, with BP restarts]
        if rest:
            rest, trials = np.array(rest), np.array(trials)
            out["bp_restarts"] = {"steps_with_restart": int(np.count_nonzero(rest)), "total": float(rest.sum()),
                                  "hist": np.bincount(np.minimum(rest, 20).astype(int)).tolist()}
            out["ls_trials"] = {"mean": float(trials.mean()), "hist": np.bincount(trials.astype(int)).tolist()}
            out["al_outer_iterations"] = int(max(al_iters) if al_iters else 0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
