#!/bin/bash
# Round-4: the GPU suite without -x (every failure listed), after an optional diagnostic.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r4d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python tools/diag_trace.py $DIAG > $OUT/diag.txt 2>&1 || { tail -30 $OUT/diag.txt; exit 1; }
  head -40 $OUT/diag.txt
fi
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread "${KARG[@]}" > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head -30
tail -1 $OUT/gpu_tests.log
exit $rc
