#!/bin/bash
# Round 5: targeted GPU tests, the team MFMA microbenchmark, then the bench line of each workload in WLS
# (window + whole solve). Outputs in gpurun_out/<TAG>/.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
FIRST=${FIRST:-tests/test_quad_maze.py tests/test_kuka.py tests/test_time_varying.py}
if [ -n "$FIRST" ] && [ "$FIRST" != none ]; then
  timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $FIRST > $OUT/first.log 2>&1
  rc=$?; tail -3 $OUT/first.log; grep -E "FAILED|Error" $OUT/first.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$MICRO" ]; then
  timeout -k 10 60 tools/microbench/team_mfma_ab > $OUT/team_mfma_ab.txt 2>&1 || { cat $OUT/team_mfma_ab.txt; exit 1; }
  cat $OUT/team_mfma_ab.txt
fi
if [ -n "$SQW" ]; then  # one SQ counter pass over a short bench window of workload $SQW
  TAG=${TAG}sq STEPS=3 BENCH_ARGS="--workload $SQW --no-solve-leg" bash tools/profile_sq.sh > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
  python3 -c "import sys; sys.path.insert(0, 'tools'); import rocpd_summary as r; r.sq_summary('gpurun_out/prof_${TAG}sq')" > $OUT/sq_$SQW.txt || exit 1
  rm -rf gpurun_out/prof_${TAG}sq
  head -8 $OUT/sq_$SQW.txt
fi
for w in ${WLS:-quad_maze kuka quadrotor}; do
  timeout -k 10 400 python bench.py --workload $w --cpu-seconds 4 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail $OUT/bench_$w.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1])
s=d['solve_rate'];print('$w value',d['value'],'window',d['window_rate'],'ms/step',d['ms_per_step'],'solve',s['wall_s'],s['batch_steps'],s['steps'])
print('  kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'],'step_frac',d['roofline']['step_frac'],'solve_frac',d['roofline'].get('solve_frac'))"
done
