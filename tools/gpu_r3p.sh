#!/bin/bash
# Duo backward prefetch check: the backward/tail parity subset, the B=1 tail bench and the default bench.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r3p}
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_tail.py tests/test_line_search_modes.py tests/test_config3_full.py tests/test_quad_maze.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $OUT/tail_b1.log 2>&1 || { tail -20 $OUT/tail_b1.log; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 - <<PY
import json
for f in ("$OUT/bench.log", "$OUT/tail_b1.log"):
    l = [x for x in open(f) if x.startswith("{")][-1]
    d = json.loads(l)
    sr = d.get("solve_rate") or {}
    print(f, "value", d["value"], "window", d.get("window_rate"), "ms/step", d["ms_per_step"],
          d["roofline"]["kernel_ms"], "solve", {k: sr.get(k) for k in ("wall_s", "batch_steps", "tail_share", "ms_per_batch_step", "converged")})
PY
