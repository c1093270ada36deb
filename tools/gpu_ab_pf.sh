#!/bin/bash
# A/B of the backward's next-knot prefetch (TOG_BWD_PF, ab_libs/pf*): parity of the variants, then the
# default bench window for the main build and each variant
cd "$(dirname "$0")/.." || exit 1
o=gpurun_out/abpf; mkdir -p $o
export TMPDIR=/tmp
set -o pipefail
for v in pf1 pf2; do
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_quad_maze.py tests/test_line_search_modes.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/parity_$v.log 2>&1 || { tail -30 $o/parity_$v.log; exit 1; }
  tail -1 $o/parity_$v.log
done
for v in base pf0 pf1 pf2 base; do
  lib=""; [ $v != base ] && lib=ab_libs/$v/libtog.so
  TOG_LIBRARY=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve-leg > $o/bench_$v.log 2>&1 || { tail -20 $o/bench_$v.log; exit 1; }
  python -c "import json; l=[x for x in open('$o/bench_$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
