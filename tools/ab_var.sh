#!/bin/bash
# A/B of libtog variants (ab_var/<v>/libtog.so, TOG_LIBRARY) on the config-4 bench window, same box.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r5r}; mkdir -p $OUT
for v in ${VARS:-main v1 v2 v3 main}; do
  vv=${v%_d}; if [ $vv = main ]; then unset TOG_LIBRARY; else export TOG_LIBRARY=$PWD/ab_var/$vv/libtog.so; fi
  if [ $vv != $v ]; then export TOG_DENSE_RECORDS=1; else unset TOG_DENSE_RECORDS; fi
  timeout -k 10 300 python bench.py --workload ${WL:-quad_maze} --no-solve-leg --no-cpu-baseline --steps 10 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail $OUT/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1]);print('$v',d['window_rate'],d['roofline']['kernel_ms'])"
done
