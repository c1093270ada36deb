"""One-line digest of bench.py JSON lines: value, window rate, per-kernel ms, roofline fraction.
  python tools/bench_summary.py gpurun_out/<tag>/bench_*.log"""
import json
import sys

for path in sys.argv[1:]:
    line = [l for l in open(path).read().strip().split("\n") if l.startswith("{")][-1]
    d = json.loads(line)
    r = d.get("roofline") or {}
    s = d.get("solve_rate") or {}
    print(f"{path}: value {d['value']:.0f} window {d.get('window_rate', 0):.0f} ms/step {d['ms_per_step']:.3f} "
          f"kernels {r.get('kernel_ms')} frac {r.get('frac')} step_frac {r.get('step_frac')} "
          f"tail_share {s.get('tail_share')} wall {s.get('wall_s')}")
