#!/bin/bash
# Round-3 final evidence on the committed build: smoke, the GPU suite, the default bench (whole solve + window
# + CPU baseline), the B=1 tail bench, then the kernel trace and PMC traffic passes of the bench window.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r3q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $OUT/tail_b1.log 2>&1 || { tail -20 $OUT/tail_b1.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
[ -n "$NO_PROF" ] || TAG=$TAG NO_SQ=1 bash tools/profile_round.sh
