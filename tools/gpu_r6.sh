#!/bin/bash
# Round 6 GPU step: targeted tests (-x), optionally the whole GPU suite (SUITE=1), then bench lines.
#   TAG=r6b TESTS="tests/test_time_varying.py" BENCH="quadrotor:--no-solve-leg quadrotor_tv:--no-solve-leg" bash tools/gpu_r6.sh
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r6x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log; grep -E "FAILED|Error" $OUT/tests.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SUITE" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
  rc=$?; tail -2 $OUT/suite.log; grep -E "FAILED|ERROR" $OUT/suite.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for spec in $BENCH; do
  wl=${spec%%:*}; args=${spec#*:}; [ "$args" = "$spec" ] && args=""
  args=${args//,/ }
  timeout -k 10 600 python bench.py --workload $wl --no-cpu-baseline $args > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail $OUT/bench_$wl.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1])
print('$wl', 'value', d['value'], 'window', d['window_rate'], 'ms/step', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])"
done
