#!/bin/bash
# A/B of the bulk k_ls_spec row tables (LDS copy vs constant-space reads, TOG_SPEC_RT=global): window bench
# of each, then the rollout/line-search parity subset.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${TAG:-abrt}
mkdir -p $OUT
set -o pipefail
for v in lds global; do
  if [ $v = global ]; then export TOG_SPEC_RT=global; else unset TOG_SPEC_RT; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve-leg > $OUT/bench_$v.log 2>&1 || { tail -20 $OUT/bench_$v.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('$OUT/bench_$v.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$v', d['window_rate'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
unset TOG_SPEC_RT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_line_search_modes.py tests/test_quad_maze.py tests/test_tail.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
