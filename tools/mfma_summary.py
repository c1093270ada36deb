"""MFMA utilisation of the matrix-core kernels from rocprofv3 databases (tools/mfma_prof.sh):

    python tools/mfma_summary.py <prof_dir> <out.json> [kernel-substring ...]

<prof_dir>/trace/*.db  a --kernel-trace pass (per-dispatch durations)
<prof_dir>/mfma/*.db   a --pmc pass: SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE

Per kernel (averages per dispatch): fp64 matrix FLOPs = 512 x SQ_INSTS_VALU_MFMA_MOPS_F64 (one
v_mfma_f64_16x16x4_f64 = 2,048 FLOPs = 4 units), their rate over the traced duration against the fp64 matrix
peak, and the busy-cycle utilisation SQ_VALU_MFMA_BUSY_CYCLES / (1,024 SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs; MI355X_MICROARCH.md, DVFS note). The
output is stamped with sha256(libtog.so)[:16] so that bench.py reports it only for the build it measured."""
import hashlib
import json
import pathlib
import sqlite3
import sys

FP64_MATRIX_PEAK_TFLOPS = 78.6  # MI355X fp64 matrix (= vector) peak: 256 CU x 128 FLOP/clk x 2.4 GHz
SIMDS = 1024


def main(d, out, pats):
    d = pathlib.Path(d)
    tr = sqlite3.connect(next((d / "trace").glob("*.db")))
    dur = {name: (n, avg_ns) for name, n, avg_ns in tr.execute(
        "select name, count(*), avg(duration) from kernels group by name")}
    pc = sqlite3.connect(next((d / "mfma").glob("*.db")))
    ctr = {}
    for k, c, v in pc.execute("select kernel_name, counter_name, avg(value) from counters_collection "
                              "group by kernel_name, counter_name"):
        ctr.setdefault(k, {})[c] = v
    res = {}
    for k, cs in ctr.items():
        if pats and not any(p in k for p in pats):
            continue
        mops = cs.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        if not mops:
            continue
        tk = next((n for n in dur if n.split("(")[0] == k.split("(")[0]), None)
        n_disp, avg_ns = dur[tk] if tk else (0, None)
        flops = 512.0 * mops
        cycles = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        r = {"dispatches_traced": n_disp, "avg_ms": (avg_ns / 1e6) if avg_ns else None,
             "mfma_f64_mops_per_dispatch": mops, "fp64_matrix_flops_per_dispatch": flops,
             "mfma_f64_instructions_per_dispatch": flops / 2048.0,
             "mfma_busy_cycles_per_dispatch": busy, "kernel_cycles_per_dispatch": cycles,
             "busy_util": (busy / (SIMDS * cycles)) if cycles else None}
        if avg_ns:
            tf = flops / (avg_ns * 1e-9) / 1e12
            r.update({"achieved_tflops": tf, "peak_tflops": FP64_MATRIX_PEAK_TFLOPS,
                      "flop_frac": tf / FP64_MATRIX_PEAK_TFLOPS,
                      "effective_clock_ghz": cycles / (avg_ns * 1e-9) / 1e9 if cycles else None})
        res[k.split("(")[0]] = r
    lib = pathlib.Path(__file__).resolve().parent.parent / \
        "trajectoryoptimization.jl-c79d492b-0548-5874-b488-5a62c1d9d0ca_amd" / "csrc" / "libtog.so"
    sha = hashlib.sha256(lib.read_bytes()).hexdigest()[:16]
    pathlib.Path(out).write_text(json.dumps({"source": str(d), "libtog_sha16": sha, "per_kernel": res}, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
