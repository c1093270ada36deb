#!/bin/bash
# Round 6 A/B step: the GPU suite on the in-tree build (SUITE=1), then window-rate A/B of the in-tree
# libtog.so against ab_var/base/libtog.so on one box (base, main, base, main per workload).
#   TAG=r6k SUITE=1 WLS="quadrotor quad_maze" bash tools/gpu_r6_ab.sh
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r6ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$SUITE" ]; then
  timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
  rc=$?; tail -2 $OUT/suite.log; grep -E "FAILED|ERROR" $OUT/suite.log | head -20
  [ $rc -eq 0 ] || exit $rc
fi
for wl in ${WLS:-quadrotor}; do
  for v in ${VARS:-base main base main}; do
    if [ $v = main ]; then unset TOG_LIBRARY; else export TOG_LIBRARY=$PWD/ab_var/$v/libtog.so; fi
    timeout -k 10 300 python bench.py --workload $wl --no-solve-leg --no-cpu-baseline --steps ${STEPS:-10} \
      > $OUT/ab_${wl}_$v.json 2> $OUT/ab_${wl}_$v.err || { tail $OUT/ab_${wl}_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/ab_${wl}_$v.json').read().strip().splitlines()[-1]);print('$wl $v',d['window_rate'],d['roofline']['kernel_ms'])"
  done
done
if [ -n "$TAIL" ]; then  # config 3's slowest trajectory alone (B = 1): the headline's tail step
  for v in ${VARS:-base main base main}; do
    if [ $v = main ]; then unset TOG_LIBRARY; else export TOG_LIBRARY=$PWD/ab_var/$v/libtog.so; fi
    timeout -k 10 200 python tools/tail_solve.py --offset 1457 --profile > $OUT/tail_$v.json 2> $OUT/tail_$v.err || { tail $OUT/tail_$v.err; exit 1; }
    echo "tail $v $(tail -c 600 $OUT/tail_$v.json)"
  done
fi
unset TOG_LIBRARY
if [ -n "$HEADLINE" ]; then
  timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('headline',d['value'],d['window_rate'],d['roofline']['kernel_ms'])"
fi
