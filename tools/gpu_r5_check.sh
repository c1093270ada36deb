#!/bin/bash
# Round 5 check: targeted tests first (-x), then the whole GPU suite, the headline tail trace and the bench.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
FIRST=${FIRST:-tests/test_history.py tests/test_line_search_modes.py tests/test_tail.py}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $FIRST > $OUT/first.log 2>&1
rc=$?; tail -3 $OUT/first.log; grep -E "FAILED|Error" $OUT/first.log | head -20
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOSUITE" ]; then
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
  rc=$?; tail -2 $OUT/suite.log; grep -E "FAILED|ERROR" $OUT/suite.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$TRACE" ]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/tools/tail_solve.py" --batch 8192) > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
  DB=$(find $OUT/trace -name "*.db" | head -1)
  python3 tools/tail_trace.py "$DB" --last 8000 > $OUT/tail_trace.txt || exit 1
  rm -rf $OUT/trace
  cat $OUT/tail_trace.txt
fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:---cpu-seconds 4} > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
s=d['solve_rate'];print('value',d['value'],'window',d['window_rate'],'ms/step',d['ms_per_step'],'solve',s['wall_s'],s['batch_steps'],s['steps'],s['ms_per_batch_step'],'tail',s['tail'])
print('kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])"
