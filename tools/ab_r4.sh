#!/bin/bash
# A/B of the config-4 bench window: the round-4 build (ab_r4/, staged from commit dc391d8) against this tree,
# same box, back to back.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-r5q}; mkdir -p $OUT
for v in r4 now r4b nowb; do
  case $v in r4|r4b) D=ab_r4 ;; *) D=. ;; esac
  timeout -k 10 300 python $D/bench.py --workload quad_maze --no-solve-leg --no-cpu-baseline --steps 10 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail $OUT/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_$v.json').read().strip().splitlines()[-1]);print('$v',d['window_rate'],d['roofline']['kernel_ms'])"
done
