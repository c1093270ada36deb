"""Summarise rocprofv3 SQLite outputs (tools/profile.sh) into a text report for profiles/.

    python tools/rocpd_summary.py gpurun_out/prof_r1 > profiles/r1_rocprof_summary.txt

Sections: kernel-trace stats (calls, total/avg duration) and, per kernel, the average FETCH_SIZE /
WRITE_SIZE per dispatch from the separate PMC passes, with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half the bytes of wide reads: x2).
"""
import pathlib
import sqlite3
import sys


def short(name):
    name = name.replace("(tog::DevProblem const*, tog::DevBuffers", "(")
    return name[:90]


def main(d):
    d = pathlib.Path(d)
    out = []
    tr = sqlite3.connect(next((d / "trace").glob("*.db")))
    out.append("== rocprofv3 --kernel-trace --stats (top_kernels)")
    out.append(f"{'kernel':92s} {'calls':>6s} {'total_us':>12s} {'avg_us':>11s} {'pct':>6s}")
    for name, calls, tot, avg, pct in tr.execute("select name,total_calls,total_duration,average,percentage "
                                                 "from top_kernels order by total_duration desc"):
        out.append(f"{short(name):92s} {calls:6d} {tot:12.1f} {avg:11.2f} {pct:6.2f}")
    out.append("")
    out.append("== per-dispatch resources (kernels table)")
    for row in tr.execute("select name, count(*), avg(duration)/1000.0, max(grid_x), max(workgroup_x), "
                          "max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(scratch_size) "
                          "from kernels group by name order by sum(duration) desc limit 8"):
        name, n, avg, gx, wx, v, a, lds, scr = row
        out.append(f"{short(name):92s} n={n} avg_us={avg:.2f} grid={gx} wg={wx} vgpr={v} agpr={a} lds={lds} "
                   f"scratch={scr}")
    for ctr in ("fetch", "write"):
        p = d / ctr
        dbs = list(p.glob("*.db"))
        if not dbs:
            continue
        c = sqlite3.connect(dbs[0])
        out.append("")
        sym = "FETCH_SIZE" if ctr == "fetch" else "WRITE_SIZE"
        corr = 2.0 if ctr == "fetch" else 1.0
        out.append(f"== {sym} per dispatch (KB; pass of its own; gfx950 correction x{corr:g} applied in "
                   f"'corrected_MB')")
        for name, n, avg in c.execute("select kernel_name, count(*), avg(value) from counters_collection "
                                      f"where counter_name='{sym}' group by kernel_name order by sum(value) desc "
                                      "limit 8"):
            out.append(f"{short(name):92s} n={n} avg_KB={avg:.1f} corrected_MB={avg * corr / 1024:.2f}")
    print("\n".join(out))
    return traffic(d)


GROUPS = {"backward": ("k_bwd_team", "k_backward"), "forward": ("k_ls_spec", "k_ls_compact", "k_ls_commit", "k_ls_decide", "k_ls_apply", "k_ls_book"),
          "jacobian": ("k_jacobian", "k_kuka_points", "k_kuka_sjac", "k_kuka_chain"),
          "expansion": ("k_expand_team", "k_expand_u")}


def traffic(d):
    """Per-step HBM bytes of each bench kernel group (one bench "launch" of a group = all its
    dispatches in one step, e.g. forward = 2 x k_ls_spec + k_ls_compact + k_ls_commit): the group's
    summed 2 x FETCH_SIZE + WRITE_SIZE (guide §HBM) over all dispatches, divided by the dispatch count
    of its least frequent kernel (once per step)."""
    res = {}
    for ctr, sym, corr in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        dbs = list((d / ctr).glob("*.db"))
        if not dbs:
            return None
        c = sqlite3.connect(dbs[0])
        tot, cnt = {}, {}
        for name, n, sm in c.execute("select kernel_name, count(*), sum(value) from counters_collection "
                                     f"where counter_name='{sym}' group by kernel_name"):
            for g, keys in GROUPS.items():
                if any(k + "<" in name for k in keys):
                    tot[g] = tot.get(g, 0.0) + sm * 1024.0 * corr
                    cnt[g] = min(cnt.get(g, n), n)
        for g in tot:
            res.setdefault(g, {})[ctr] = tot[g] / max(1, cnt[g])
    for g in res:
        res[g]["traffic_bytes"] = res[g].get("fetch", 0.0) + res[g].get("write", 0.0)
    return res


if __name__ == "__main__":
    import json

    src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r1"
    t = main(src)
    if len(sys.argv) > 2 and t:
        import hashlib

        # stamped with the build the passes measured: bench.py uses a summary only for the same libtog.so
        lib = pathlib.Path(__file__).resolve().parent.parent / "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd" / "csrc" / "libtog.so"
        sha = hashlib.sha256(lib.read_bytes()).hexdigest()[:16]
        pathlib.Path(sys.argv[2]).write_text(json.dumps({"source": src, "libtog_sha16": sha, "per_launch": t}, indent=1) + "\n")


def sq_summary(d):
    """Per-kernel averages of every PMC counter in <d>/sq/*.db (SQ stall/issue analysis)."""
    d = pathlib.Path(d)
    c = sqlite3.connect(next((d / "sq").glob("*.db")))
    rows = c.execute("select kernel_name, counter_name, avg(value), count(*) from counters_collection "
                     "group by kernel_name, counter_name").fetchall()
    by = {}
    for k, ctr, v, n in rows:
        by.setdefault(k, {})[ctr] = v
    for k, ctrs in sorted(by.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = ctrs.get("SQ_WAVE_CYCLES", 0) or 1
        parts = " ".join(f"{ctr}={v:.3g}" for ctr, v in sorted(ctrs.items()))
        frac = {x: ctrs.get(x, 0) / wc for x in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        print(short(k), "\n   ", parts, "\n    fractions of wave-cycles:", {a: round(b, 3) for a, b in frac.items()})
