#!/bin/bash
# A/B of the LLVM scheduling strategy for the quadrotor kernels (ab_libs/ilp: -amdgpu-sched-strategy=max-ilp):
# parity of the variant, then the default bench window for the main build and the variant
cd "$(dirname "$0")/.." || exit 1
o=gpurun_out/absched; mkdir -p $o
export TMPDIR=/tmp
set -o pipefail
TOG_LIBRARY=ab_libs/ilp/libtog.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_quad_maze.py tests/test_line_search_modes.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/parity_ilp.log 2>&1 || { tail -30 $o/parity_ilp.log; exit 1; }
tail -1 $o/parity_ilp.log
for v in base ilp base ilp; do
  lib=""; [ $v != base ] && lib=ab_libs/$v/libtog.so
  TOG_LIBRARY=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve-leg > $o/bench_$v.log 2>&1 || { tail -20 $o/bench_$v.log; exit 1; }
  python -c "import json; l=[x for x in open('$o/bench_$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
