"""bench.py — batched iLQR iterations/sec on MI355X (BASELINE.json metric).

One step = one batched AL-iLQR ``step!`` (jacobians -> cost expansion + square-root backward pass
-> forward-pass line search -> bookkeeping / AL dual+penalty update) for every active trajectory of
the per-GPU batch. Workload: BASELINE.json configs[2] (quadrotor n=13 m=4 N=101, AL-iLQR with
u in [0,15] + goal, sqrt backward pass), 8192 trajectories per GPU, synthetic random starts
(SURVEY.md §8(d)); inputs resident in HBM before timing. ``value`` = SURVEY.md §8(d)'s metric: Σ
trajectory-iterations of the WHOLE solve (tog_solve_init until no trajectory is active, the stopping
check included) on all GPUs / max-over-ranks wall time. The `--steps` window (every trajectory
active) is reported beside it as ``window_rate``; ``steps``/``warmup``/``ms_per_step`` describe it.

Multi-GPU: one process per GPU (torch.distributed.run); trajectories are independent so each rank
solves its own shard (weak scaling). The only collective is one RCCL all-reduce per step of the
batch statistics [n_active, Σ cost, max c_max].
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402

METRIC = "iLQR iterations/sec (batched trajectories), quadrotor n=13 m=4 N=101"
# --workload: the headline line is config 3 (BASELINE.json metric); the other BASELINE configs can
# be measured the same way (secondary lines, their own metric string).
WORKLOADS = {
    "quadrotor": ("config_quadrotor", 8192, True,
                  "quadrotor point-to-point, AL-iLQR, u in [0,15] + goal, sqrt backward pass (BASELINE.json configs[2])",
                  "synthetic (seeded random starts: x0[1:3]+N(0,1), U0 = hover + 0.1 N(0,1))"),
    "quadrotor_tv": ("config_quadrotor_tv", 8192, True,
                     "config 3 with a time-varying Objective: 100 stage costs LQRCost(Q w_k, R v_k) + terminal "
                     "(per-knot cost table; the team backward's TV variant)",
                     "synthetic (config 3's seeded starts)"),
    "cartpole": ("config_cartpole", 1024, False,
                 "cartpole swing-up, unconstrained iLQR (BASELINE.json configs[1])",
                 "synthetic (seeded U0 = 0.01 + 0.5 N(0,1), x0 = 0)"),
    "quad_maze": ("config_quad_maze", 8192, True,
                  "quad_obs maze N=201, AL-iLQR, bounds + 4 cylinders + 3 spheres (BASELINE.json configs[3], per-GPU shard)",
                  "synthetic (seeded x0[1:3] ~ U([-5,5]x[-3,0]x[8,12]), U0 = hover + 0.1 N(0,1))"),
    "maze_infeasible": ("config_quadrotor_maze_infeasible", 1024, True,
                        "quadrotor_maze infeasible-start AL phase (SURVEY.md §8(f) row 1): m = 4 + 13 slack controls, "
                        "69 constraint rows per knot, N=101",
                        "synthetic (seeded maze way-points + N(0, 0.5^2), hover U0, slack controls from the guess)"),
    "kuka": ("config_kuka", 4096, True,
             "Kuka iiwa 7-DoF (RBD), AL-iLQR, terminal goal, notebook options (BASELINE.json configs[4])",
             "synthetic (seeded x0[1:7] ~ U(-0.2,0.2), U0 = hold torque at x0)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6  # MI355X public spec, fp64 vector (the local guide has no fp64 row):
#                          256 CU x 4 SIMD x 16 lanes x 2 FLOP x 2.4 GHz


def kernel_bytes(n, m, N, p_stage, p_term, trials, dense_knots=1):
    """Algorithmic HBM bytes per trajectory-step for each kernel (SURVEY.md §8(d) staged design;
    DESIGN.md §4-5 list the terms). The expansion records (k_expand_team) hold Q.x, Q.u, Q.uu per
    knot and Q.xx at the `dense_knots` knots whose AL terms change it (config 3: the terminal one)."""
    K = N - 1
    rec = 8 * (N * (n + m + m * m) + dense_knots * n * n)       # one trajectory's expansion records
    jac = 8 * K * ((n + m) + n * (n + m))                       # read x,u ; write [A|B]
    exp_ = 8 * (N * n + K * m + 2 * (K * p_stage + p_term)) + rec  # read x,u,λ,μ ; write records
    bwd = 8 * (K * (n * (n + m) + m * (n + 1))) + rec           # read [A|B], records ; write K,d
    fwd = 8 * (trials * K * (2 * (n + m) + m * (n + 1))         # per trial: read x,u,K,d ; write x̄,ū
               + 2 * K * (n + m)                                # accept: copy X̄,Ū -> X,U
               + trials * 3 * (K * p_stage + p_term))           # λ, μ read, C written per trial
    return {"jacobian": jac, "backward": bwd, "forward": fwd, "expansion": exp_}


def bwd_flops(n, m, N, p_x, p_u, sqrt=True):
    """Useful fp64 FLOPs of one trajectory's square-root backward pass (per backward launch), counted
    from the operation sequence of backward_pass.jl:87-169 (the oracle's): per knot
      Q.x/Q.u += [A B]ᵀs                2n(n+m)
      S·[A B], S upper-triangular        (n+m)·n(n+1)
      chol_plus QR [Q.xx; S A]           Σ_j 4(n+1)(n-1-j) + 3n   (structured: R top block)
      chol_plus QR [Q.uu; S B; AL rows]  Σ_j 4(n+1+p_u)(m-1-j) + 3(n+p_u)
      AL state rows QR on Q.xx           Σ_j 4(p_x+1)(n-1-j)
      Q.ux += (S B)ᵀ(S A)                2nmn
      Quu_reg QR, two triangular solves  4m³ + 2·2m²(n+1)
      tmp1 = Q.xxᵀ \ Q.uxᵀ, chol_minus   n²m + 6nm²
      S-update operands + QR             2n²m + 2m²n + Σ_j 4(m+1)(n-1-j)
    Divisions and square roots count as one FLOP each. (The std pass is within ~10 % of this.)"""
    tri = lambda rows, cols: sum(4 * (rows + 1) * (cols - 1 - j) for j in range(cols))  # noqa: E731
    per_knot = (2 * n * (n + m) + (n + m) * n * (n + 1) + tri(n, n) + 3 * n
                + tri(n + p_u, m) + 3 * (n + p_u) + (tri(p_x, n) if p_x else 0)
                + 2 * n * m * n + 4 * m ** 3 + 4 * m * m * (n + 1)
                + n * n * m + 6 * n * m * m + 2 * n * n * m + 2 * m * m * n + tri(m, n))
    return per_knot * (N - 1)


def lib_sha16():
    """First 16 hex digits of sha256(libtog.so): the build a PMC summary belongs to."""
    import hashlib

    p = os.path.join(ROOT, "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd", "csrc", "libtog.so")
    try:
        with open(p, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def measured_traffic(kernel, workload="quadrotor"):
    """HBM bytes per launch of `kernel` from the committed PMC summary of THIS build (profiles/*_traffic.json,
    written by tools/rocpd_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    same bench command, FETCH_SIZE x2 per the gfx950 correction, stamped with the sha256 of the libtog.so
    they measured). A summary of another build is never used: (None, reason) then."""
    import glob

    # the headline workload's summaries are <round>_traffic.json; <round>_<workload>_traffic.json
    # (e.g. r4z_quad_maze_traffic.json) belong to the other configs
    def ours(f):
        b = os.path.basename(f)
        if workload == "quadrotor":
            return b.count("_") == 1
        return b.endswith(f"_{workload}_traffic.json") and b.split("_", 1)[1] == f"{workload}_traffic.json"

    sha = lib_sha16()
    match = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        if not ours(f):
            continue
        with open(f) as fh:
            t = json.load(fh)
        if sha is not None and t.get("libtog_sha16") == sha:
            match.append((f, t))
    if not match:
        return None, f"no committed PMC summary of this build (libtog.so sha256[:16] {sha})"
    f, t = match[-1]
    per = t["per_launch"].get(kernel)
    if not per:
        return None, f"{os.path.relpath(f, ROOT)} has no {kernel} entry"
    return round(per["traffic_bytes"]), os.path.relpath(f, ROOT)


def measured_mfma(workload):
    """The matrix-core utilisation of this build's MFMA kernels from a committed PMC summary
    (profiles/*_<workload>_mfma.json, tools/mfma_prof.sh + tools/mfma_summary.py), or None."""
    import glob

    sha = lib_sha16()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_mfma.json")), reverse=True):
        with open(f) as fh:
            t = json.load(fh)
        if sha is not None and t.get("libtog_sha16") == sha:
            out = {"source": os.path.relpath(f, ROOT) + " (committed rocprofv3 passes of this build)",
                   **t["per_kernel"]}
            if "tog::k_kuka_chain<tog::Kuka>" in out or any("k_kuka_chain" in k for k in out):
                # kj_chain_product (csrc/tog_kuka_jac.hpp): J (7 x 14) times T (14 x 21) as two 16x16 output
                # tiles of v_mfma_f64_16x16x4_f64, 4 k-steps each: 7 of 16 rows, 21 of 32 columns, 14 of 16 k
                out["tile_occupancy"] = {"output_rows": "7/16", "output_cols": "21/32", "k": "14/16",
                                         "useful_mac_fraction": round(7 * 21 * 14 / (2 * 16 * 16 * 16), 4)}
            return out
    return None


def host_cpu_info():
    """Host CPU facts for the baseline line: nproc (what the OS shows), the CPUs this process may run
    on (affinity), the cgroup CPU quota (a GPU box's share of a big host) and the model name."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "cpu_model": None}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def cpu_baseline(pkg, orc, seconds=10.0, threads=None):
    """The C oracle ("port" of the reference algorithm) on the host cores: full AL-iLQR solves of
    config-3 trajectories, OpenMP over trajectories (threads pinned, OMP_PROC_BIND=close). Every
    CPU this process may use takes part: the affinity set, capped by the cgroup quota when one
    is set (a GPU box's share of a larger host: oversubscribing the quota only adds contention).
    Bounded sample (~`seconds` of work per run): one warm-up run is discarded (page faults, frequency
    ramp: the first run on a fresh box measured 2-3x slow), then runs repeat until two consecutive runs
    agree within 10 % (at most 5) and the median is reported with its spread. The rate of a run is its
    sustained all-thread throughput, steps ÷ (Σ per-trajectory solve seconds ÷ threads): iteration counts
    are heavy-tailed (a few trajectories run thousands of iterations), so the wall time of a bounded
    sample measures its slowest trajectory rather than the cores (`wall_rates` are reported too)."""
    info = host_cpu_info()
    avail = info["affinity"]
    if info["cgroup_quota_cpus"]:
        avail = max(1, min(avail, int(info["cgroup_quota_cpus"])))
    threads = threads or avail
    # calibration: 2 trajectories per thread, then size the sample to ~`seconds`
    prob, opts = pkg.Problems.config_quadrotor(B=2 * threads, offset=100000)
    t = time.perf_counter()
    orc.solve_batch(prob, opts, nthreads=threads)
    dt = max(time.perf_counter() - t, 1e-3)
    B = int(min(16384, 2 * threads * max(1.0, seconds / dt)))
    B = max(threads, B - B % threads)
    runs = []
    prob, opts = pkg.Problems.config_quadrotor(B=B, offset=150000)
    t = time.perf_counter()
    warm = (orc.solve_batch(prob, opts, nthreads=threads), None)
    warm = (warm[0], time.perf_counter() - t)
    for r in range(5):
        prob, opts = pkg.Problems.config_quadrotor(B=B, offset=200000 + r * B)
        t = time.perf_counter()
        steps, busy = orc.solve_batch(prob, opts, nthreads=threads, busy=True)
        runs.append((steps, time.perf_counter() - t, busy))
        if len(runs) >= 2:
            a, b = (x[0] / (x[2] / threads) for x in runs[-2:])
            if abs(a - b) <= 0.1 * max(a, b):
                break
    rates = [x[0] / (x[2] / threads) for x in runs]
    value = float(np.median(rates))
    # single-thread rate next to the reference's published per-core figures
    p1, o1 = pkg.Problems.config_quadrotor(B=1, offset=300000)
    t1 = time.perf_counter()
    s1 = orc.solve_batch(p1, o1, nthreads=1)
    d1 = time.perf_counter() - t1
    return {"value": value, "unit": "iLQR iterations/s", "cores": threads, "kind": "port",
            "sample": f"{B} config-3 trajectories per run solved to AL convergence by oracle/tog_oracle.c, "
                      f"OpenMP over trajectories; warm-up run ({warm[0]}, {warm[1]:.1f}) discarded; runs (steps, s): "
                      + ", ".join(f"({x[0]}, {x[1]:.1f})" for x in runs) + "; value = median",
            "run_rates": [round(x, 1) for x in rates],
            "wall_rates": [round(x[0] / x[1], 1) for x in runs],
            "spread": round((max(rates) - min(rates)) / value, 3),
            "nproc": info["nproc"], "affinity_cpus": info["affinity"],
            "cgroup_quota_cpus": info["cgroup_quota_cpus"], "cpu_model": info["cpu_model"],
            "single_thread": {"value": s1 / d1, "sample": f"1 trajectory, {s1} iLQR steps, {d1:.1f} s"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="trajectories per GPU (default: the config's)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="quadrotor")
    ap.add_argument("--parts", type=int, default=1,
                    help="single process: split the GPU's batch into this many slices, each on its own stream "
                         "(tog_create_multi over the same device), so one slice's latency-bound line search "
                         "overlaps another's Jacobians")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-solve-leg", action="store_true", help="skip the full-solve timing leg")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--solve-sets", type=int, default=None,
                    help="whole solves on this many disjoint start sets (offsets 0, B, 2B per GPU slice); value is "
                         "set 0's, the others are reported beside it (default: 3 for the headline, else 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("OMP_PROC_BIND", "close")  # the CPU-baseline leg's OpenMP threads are pinned
    os.environ.setdefault("OMP_PLACES", "cores")
    dist = None
    # TOG_BENCH_DIST=1 takes the torch.distributed (RCCL) path even at world size 1, to exercise the
    # multi-rank code (stream interop, stats all-gather, job rate) on a one-GPU box
    if world > 1 or os.environ.get("TOG_BENCH_DIST") == "1":
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    pkg = __graft_entry__.load_package()
    abi = pkg.abi
    cfg_fn, B_default, al_mode, wl_desc, wl_data = WORKLOADS[args.workload]
    mode = abi.MODE_AL if al_mode else abi.MODE_ILQR
    B = args.batch or B_default
    offset, count = pkg.distributed.shard(B * world, rank, world)  # weak scaling: B trajectories per GPU
    prob, opts = getattr(pkg.Problems, cfg_fn)(B=count, offset=offset)
    stream = None
    if dist is not None:
        import torch

        # libtog, the stats reduction and RCCL share one stream. A dedicated stream, not torch's
        # default: its handle is 0 (the null stream), which tog_set_stream reads as "own stream".
        tstream = torch.cuda.Stream(device=local_rank)
        torch.cuda.set_stream(tstream)
        stream = tstream.cuda_stream
    if args.parts > 1 and dist is not None:
        raise SystemExit("--parts is for single-process runs (the multi-rank path sets one shared stream)")
    devices = [local_rank] * args.parts if args.parts > 1 else None
    solver = pkg.AbstractSolverFor(prob, opts, device=local_rank, stream=stream, devices=devices)
    h = solver.handle
    n, m, N = prob.model.n, prob.model.m, prob.N

    stats_t = gathered = None
    if dist is not None:
        stats_t = torch.zeros(3, dtype=torch.float64, device=f"cuda:{local_rank}")
        gathered = torch.zeros(3 * world, dtype=torch.float64, device=f"cuda:{local_rank}")

    def allreduce_stats():
        # batch statistics [n_active, Σ cost, max c_max] of every shard: written on-device by
        # k_batch_stats and exchanged with ONE RCCL collective, stream-ordered (no host sync)
        if dist is None:
            return None
        abi.check(h.lib, h.lib.tog_batch_stats_device(h.h, ctypes.c_void_p(stats_t.data_ptr())))
        return pkg.distributed.reduce_stats(stats_t, gathered, dist)

    def barrier_sync():
        h.synchronize()
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    # ---------------------------------------------------------------- leg 1: step window
    if prob.model.slack:  # infeasible start: slack_controls(prob) before the solve (infeasible.jl:63-80)
        h.slack_controls()
    h.solve_init(mode)
    h.solve_step(args.warmup)
    h.synchronize()
    steps0 = h.total_steps()
    active0 = int(h.batch_stats()[0])
    barrier_sync()
    h.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        h.solve_step(1)
        allreduce_stats()
    barrier_sync()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    ms, launches = h.profile_read()
    h.profile(False)
    steps_done = h.total_steps() - steps0
    active1 = int(h.batch_stats()[0])
    St = h.get(abi.FIELD_STATS)
    trials = float(np.mean(St[:, abi.STAT_LS_TRIALS][St[:, abi.STAT_LS_TRIALS] > 0])) if np.any(
        St[:, abi.STAT_LS_TRIALS] > 0) else 1.0

    if dist is not None:
        window_rate, steps_all, elapsed = pkg.distributed.job_rate(steps_done, elapsed, dist,
                                                                   device=f"cuda:{local_rank}")
    else:
        steps_all = float(steps_done)
        window_rate = steps_all / elapsed
    # roofline for the dominant kernel (largest total device time over the timed region)
    cons = prob.constraints
    p_stage = cons[0].num_constraints("stage") if al_mode else 0
    p_term = cons[N - 1].num_constraints("terminal") if al_mode else 0
    # knots with a dense expansion record: the terminal one, plus every stage knot whose AL rows change
    # Q.xx (sqrt: a row with a state gradient; std: any row)
    sq = bool(pkg.solvers.to_tog_options(opts).square_root)
    p_xrows = max(0, p_stage - 2 * m) if al_mode else 0
    dense = 1 + ((N - 1) if (al_mode and ((p_xrows > 0) if sq else (p_stage > 0))) else 0)
    kb = kernel_bytes(n, m, N, p_stage, p_term, trials, dense)
    names = ["jacobian", "backward", "forward", "expansion"]
    dom = int(np.argmax(ms))
    avg_ms = ms[dom] / max(1, launches[dom])
    # algorithmic bytes per launch = per-trajectory bytes x trajectories processed per launch
    per_launch_traj = steps_done / max(1, launches[dom])
    alg_bytes = kb[names[dom]] * per_launch_traj
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    traffic, tsrc = measured_traffic(names[dom], args.workload)
    # whole step: Σ per-kernel algorithmic bytes of every trajectory-step of the job ÷ the window's wall
    # time, against the job's aggregate HBM peak (world x 8 TB/s)
    step_gbs = sum(kb.values()) * steps_all / elapsed / 1e9 / world
    # backward kernel's useful fp64 FLOP rate against the fp64 vector peak
    p_u = 2 * m if al_mode else 0  # control-bound rows of the stage constraints
    p_x = max(0, p_stage - p_u) if al_mode else 0
    bwd_i = names.index("backward")
    bwd_avg_ms = ms[bwd_i] / max(1, launches[bwd_i])
    bwd_traj = steps_done / max(1, launches[bwd_i])
    flops = bwd_flops(n, m, N, p_x, p_u) * bwd_traj
    flop_rate = flops / (bwd_avg_ms * 1e-3) / 1e12
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_source": (f"{tsrc} (committed PMC passes of this command on this build; not measured "
                                   "in this run)" if traffic is not None else tsrc),
                "libtog_sha16": lib_sha16(),
                "algorithmic_bytes_per_launch": round(alg_bytes), "kernel": names[dom],
                "kernel_ms": {nm_: round(float(ms[i] / max(1, launches[i])), 4) for i, nm_ in enumerate(names)},
                "step_achieved": round(step_gbs, 2),
                "step_frac": round(step_gbs / HBM_PEAK_GBS, 5),
                "step_bytes_per_traj_iter": int(sum(kb.values())),
                "flop_kernel": "backward",
                "flop_achieved_tflops": round(flop_rate, 3),
                "flop_peak_tflops": FP64_PEAK_TFLOPS,
                "flop_frac": round(flop_rate / FP64_PEAK_TFLOPS, 5),
                "flops_per_traj_iter": int(bwd_flops(n, m, N, p_x, p_u))}

    # ---------------------------------------------------------------- leg 2: the whole solve
    solve_leg = None
    solve_sets = None
    if not args.no_solve_leg:
        solve_leg = time_solve(h, abi, mode, prob, dist, allreduce_stats, barrier_sync, local_rank, pkg)
        nsets = args.solve_sets if args.solve_sets is not None else (3 if args.workload == "quadrotor" else 1)
        if nsets > 1:
            # the whole-solve rate depends on each set's slowest trajectories: disjoint start sets of the same
            # size (set s: the job's trajectories s*B*world .. (s+1)*B*world - 1, this rank's contiguous slice)
            solve_sets = [{"offset": 0, "value": solve_leg["value"], "wall_s": solve_leg["wall_s"],
                           "steps": solve_leg["steps"], "max_traj_iterations": solve_leg["traj_iterations"]["max"]}]
            for sidx in range(1, nsets):
                off = sidx * B * world + offset
                prob_s, _ = getattr(pkg.Problems, cfg_fn)(B=count, offset=off)
                r = time_solve(h, abi, mode, prob_s, dist, allreduce_stats, barrier_sync, local_rank, pkg)
                solve_sets.append({"offset": sidx * B * world, "value": r["value"], "wall_s": r["wall_s"],
                                   "steps": r["steps"], "max_traj_iterations": r["traj_iterations"]["max"]})
    # value: SURVEY.md §8(d)'s metric, the whole solve (tog_solve_init until no trajectory is active);
    # the full-batch step window is reported beside it as window_rate
    value = solve_leg["value"] if solve_leg is not None else window_rate
    # the whole solve against the HBM roofline: its rate x the per-iteration algorithmic bytes of the
    # staged step ÷ the job's aggregate peak (the tail runs few trajectories per launch, so this is far
    # below step_frac)
    roofline["solve_frac"] = round(value * sum(kb.values()) / 1e9 / world / HBM_PEAK_GBS, 5)

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1 and args.workload == "quadrotor":
            orc = __graft_entry__.load_oracle()
            cpu = cpu_baseline(pkg, orc, seconds=args.cpu_seconds)
        line = {
            "metric": METRIC if args.workload == "quadrotor" else
            f"iLQR iterations/sec (batched trajectories), {args.workload} n={n} m={m} N={N}", "value": round(value, 2), "unit": "iLQR iterations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": wl_data,
            "config": {"workload": wl_desc, "n": n, "m": m, "N": N,
                       "batch_per_gpu": B, "global_batch": B * world, "parallelism": f"batch-shard x{world}",
                       "streams_per_gpu": args.parts,
                       "mean_line_search_trials": round(trials, 3),
                       "timed_window": {"solve_steps": [args.warmup + 1, args.warmup + args.steps],
                                        "active_at_start": active0, "active_at_end": active1,
                                        "rate": round(window_rate, 2),
                                        "note": "steps / warmup / ms_per_step are this window's (batch "
                                                "steps of the solve with every trajectory active); value "
                                                "is solve_rate, the whole solve"}},
            "window_rate": round(window_rate, 2),
            "solve_rate": solve_leg,
            "solve_rate_sets": (None if solve_sets is None else {
                "sets": solve_sets,
                "mean": round(float(np.mean([x["value"] for x in solve_sets])), 2),
                "min": round(float(np.min([x["value"] for x in solve_sets])), 2),
                "max": round(float(np.max([x["value"] for x in solve_sets])), 2),
                "note": "the whole solve on disjoint start sets of the same size; value is the first set's (offset 0)"}),
            "roofline": roofline,
            "mfma": (measured_mfma(args.workload) if args.workload == "kuka" else None),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def time_solve(h, abi, mode, prob, dist, allreduce_stats, barrier_sync, local_rank, pkg, chunk=4, max_steps=10000):
    """The whole solve, SURVEY.md §8(d): from tog_solve_init (initial rollout + cost) until no
    trajectory of the job is active, including the batch-level stopping check every `chunk` steps
    (the job-wide [n_active, Σ J, max c_max]; over RCCL for several ranks). Same trajectories as the
    window leg (re-initialised from the same U0). Returns Σ steps ÷ max-over-ranks wall time.

    The check is pipelined as tog_solve does it: the next chunk is enqueued before the host waits for
    the previous chunk's statistics (tog_batch_stats_begin / _end; for RCCL a copy into pinned host
    memory behind an event), so the device does not idle during the host round trip. The solve stops one
    chunk after the check that saw no active trajectory (that chunk's kernels return at once)."""
    torch = None
    if dist is not None:
        import torch
    h.upload_state(prob)
    if prob.model.slack:
        h.slack_controls()
    barrier_sync()
    t0 = time.perf_counter()
    h.solve_init(mode)
    B_job = float(prob.B) * (dist.get_world_size() if dist is not None else 1)
    timeline = [(0.0, B_job)]  # (seconds since init, job-wide n_active) at every stopping check

    def begin():
        h.batch_stats_begin()  # local check: also the handle's tail-mode hint
        if dist is None:
            return None
        red = allreduce_stats()
        host = torch.empty(3, dtype=torch.float64, pin_memory=True)
        host.copy_(red, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    def end(tok):
        loc = h.batch_stats_end()
        if tok is None:
            return float(loc[0])
        tok[1].synchronize()
        return float(tok[0][0].item())

    done = chunk
    h.solve_step(chunk)
    tok = begin()
    while True:
        nxt = min(chunk, max_steps - done)
        if nxt > 0:
            h.solve_step(nxt)
        done += nxt
        n_active = end(tok)  # the chunk before `nxt`
        timeline.append((time.perf_counter() - t0, n_active))
        if n_active == 0.0 or nxt == 0:
            break
        tok = begin()
    barrier_sync()
    wall = time.perf_counter() - t0
    # tail share: the fraction of the solve's wall time spent with fewer than 1 % of the job's
    # trajectories active (each check interval counted by the n_active at its start)
    tail = sum(t1 - t0_ for (t0_, a0), (t1, _) in zip(timeline, timeline[1:]) if a0 < 0.01 * B_job)
    bulk_steps = next((i * chunk for i, (_, a) in enumerate(timeline) if a < 0.01 * B_job), done)
    steps = h.total_steps()  # k_init (tog_solve_init) zeroes the per-trajectory counters
    St = h.get(abi.FIELD_STATS)
    conv = int(np.count_nonzero(St[:, abi.STAT_FLAGS].astype(np.int64) &
                                (abi.TRAJ_AL_CONVERGED | abi.TRAJ_CONVERGED)))
    if dist is not None:
        rate, steps_all, wall_all = pkg.distributed.job_rate(steps, wall, dist, device=f"cuda:{local_rank}")
    else:
        rate, steps_all, wall_all = steps / wall, float(steps), wall
    it = St[:, abi.STAT_TOTAL_STEPS]
    return {"value": round(rate, 2), "unit": "iLQR iterations/s", "steps": int(steps_all),
            "wall_s": round(wall_all, 4), "batch_steps": done,
            "ms_per_batch_step": round(1e3 * wall / max(1, done), 4),
            "tail_share": round(tail / wall, 4),
            "tail": {"threshold_active": 0.01 * B_job, "batch_steps_before": bulk_steps,
                     "seconds": round(tail, 4)},
            "traj_iterations": {"min": int(it.min()), "mean": round(float(it.mean()), 2), "max": int(it.max())},
            "converged": conv, "batch": int(prob.B),
            "note": "tog_solve_init .. last trajectory finished; stopping check every 4 steps, pipelined "
                    "(the next chunk is enqueued before the host reads the previous one's statistics)"}


if __name__ == "__main__":
    main()
