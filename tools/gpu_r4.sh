#!/bin/bash
# Round-4 GPU check: smoke, the GPU suite (optionally a -k filter), optional benches.
#   TAG=r4a [K="expr"] [BENCH="quadrotor kuka"] [TAIL=1] bash tools/gpu_r4.sh
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r4a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  KARG=()
  [ -n "$K" ] && KARG=(-k "$K")
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread "${KARG[@]}" > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
for w in $BENCH; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$w.log 2>&1 || { tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-400
done
if [ -n "$TAIL" ]; then
  timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $OUT/tail_b1.log 2>&1 || { tail -20 $OUT/tail_b1.log; exit 1; }
  tail -1 $OUT/tail_b1.log | cut -c1-400
fi
exit 0
