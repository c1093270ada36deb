#!/bin/bash
# Quick GPU iteration: the given test files (-m gpu), then the B=1 tail kernel trace (tools/gpu_tailprof.sh).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gradient_types.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
[ -n "$NO_PROF" ] || bash tools/gpu_tailprof.sh
