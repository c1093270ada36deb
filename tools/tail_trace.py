"""Attribute a kernel trace of tools/tail_solve.py (rocprofv3 --kernel-trace database).

    python tools/tail_trace.py gpurun_out/<dir>/run_results.db [--last 4000] > profiles/r5_tail_trace.txt

Over the last `--last` dispatches (the steady tail): busy time per kernel (calls, total, average),
and the idle time between consecutive dispatches split by the kernel that follows the gap, so that a
host round trip (the gap before the first launch after a blocking readback) shows up apart from the
launch-to-launch latency of a stream-ordered chain.
"""
import collections
import sqlite3
import sys


def short(name):
    name = name.split("(")[0]
    return name[:70]


def main(path, last=4000):
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    rows = rows[-last:]
    t0, t1 = rows[0][1], rows[-1][2]
    span = (t1 - t0) / 1e6
    busy = collections.defaultdict(lambda: [0, 0.0])
    gaps = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for i, (nm, s, e) in enumerate(rows):
        k = short(nm)
        busy[k][0] += 1
        busy[k][1] += (e - s) / 1e6
        if i:
            g = (s - rows[i - 1][2]) / 1e6
            gaps[k][0] += 1
            gaps[k][1] += g
            gaps[k][2] = max(gaps[k][2], g)
    tb = sum(v[1] for v in busy.values())
    tg = sum(v[1] for v in gaps.values())
    print(f"last {len(rows)} dispatches: span {span:.3f} ms, kernels busy {tb:.3f} ms, gaps {tg:.3f} ms")
    nb = busy.get("k_batch_stats", [0])[0] or 1
    print(f"per stopping check (k_batch_stats calls = {nb}): span {span / nb:.4f} ms, busy {tb / nb:.4f}, "
          f"gaps {tg / nb:.4f}")
    print()
    print(f"{'kernel':72s} {'calls':>6s} {'busy_ms':>10s} {'avg_us':>9s} | {'gap_ms_before':>13s} {'avg_gap_us':>10s} "
          f"{'max_gap_us':>10s}")
    for k, (n, t) in sorted(busy.items(), key=lambda kv: -kv[1][1]):
        g = gaps.get(k, [0, 0.0, 0.0])
        print(f"{k:72s} {n:6d} {t:10.3f} {1e3 * t / n:9.2f} | {g[1]:13.3f} {1e3 * g[1] / max(1, g[0]):10.2f} "
              f"{1e3 * g[2]:10.2f}")


def by_width(path, kernel="k_bwd", marker="k_jacobian"):
    """Batch steps (delimited by `marker` dispatches) binned by the launch width of the backward kernel
    (its workgroup count = ceil(n_active) of the last readback in a compacted tail launch): steps, mean
    step time and the mean time of each kernel per step in that bin."""
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
    steps, cur = [], None
    for nm, s, e, gx, wx in rows:
        k = short(nm)
        if k.startswith("void tog::" + marker) or k.startswith(marker):
            if cur:
                steps.append(cur)
            cur = {"t0": s, "t1": e, "w": None, "k": collections.defaultdict(float)}
        if cur is None:
            continue
        cur["t1"] = max(cur["t1"], e)
        cur["k"][k.replace("void tog::", "").split("<")[0]] += (e - s) / 1e3
        if kernel in k and cur["w"] is None:
            cur["w"] = gx // max(1, wx)
    if cur:
        steps.append(cur)
    for a, b in zip(steps, steps[1:]):
        a["dur"] = (b["t0"] - a["t0"]) / 1e6
    steps[-1]["dur"] = (steps[-1]["t1"] - steps[-1]["t0"]) / 1e6
    if len(sys.argv) > 2 and "--dump" in sys.argv:
        import json
        json.dump([[st["w"], round(st["dur"], 4), {k: round(v, 1) for k, v in st["k"].items()}] for st in steps],
                  open(sys.argv[sys.argv.index("--dump") + 1], "w"))
    bins = [(1, 1), (2, 2), (3, 4), (5, 8), (9, 16), (17, 32), (33, 64), (65, 128), (129, 512), (513, 2048),
            (2049, 1 << 30)]
    print()
    print("batch steps binned by the backward launch width (workgroups):")
    print(f"{'width':>12s} {'steps':>6s} {'ms/step':>9s} {'total_s':>8s}  per-kernel us/step")
    for lo, hi in bins:
        sel = [st for st in steps if st["w"] is not None and lo <= st["w"] <= hi]
        if not sel:
            continue
        dur = [st["dur"] for st in sel]
        ks = collections.defaultdict(float)
        for st in sel:
            for k, v in st["k"].items():
                ks[k] += v / len(sel)
        top = ", ".join(f"{k} {v:.0f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1])[:7])
        print(f"{lo:5d}-{hi:<6d} {len(sel):6d} {sum(dur) / len(dur):9.4f} {sum(dur) / len(dur) * len(sel) / 1e3:8.3f}  {top}")


if __name__ == "__main__":
    args = sys.argv[1:]
    last = 4000
    if "--dump" in args:
        i = args.index("--dump")
        del args[i:i + 2]
    if "--last" in args:
        i = args.index("--last")
        last = int(args[i + 1])
        del args[i:i + 2]
    main(args[0], last)
    by_width(args[0])
