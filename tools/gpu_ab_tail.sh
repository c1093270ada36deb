#!/bin/bash
# A/B of the tail backward variant (ab_libs/<v>/libtog.so from tools/ab_quad.sh): parity of two variants,
# the one-trajectory tail bench per variant, and section timers of the profiled builds.
cd "$(dirname "$0")/.." || exit 1
o=gpurun_out/abtail; mkdir -p $o
export TMPDIR=/tmp
set -o pipefail
for v in ${PARITY:-pf1tri0 pf0tri1}; do
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $o/parity_$v.log 2>&1 || { tail -30 $o/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $o/parity_$v.log)"
done
for v in base ${VARIANTS:-pf0tri0 pf1tri0 pf0tri1} base; do
  lib=""; [ $v != base ] && lib=ab_libs/$v/libtog.so
  TOG_LIBRARY=$lib timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $o/tail_$v.log 2>&1 || { tail -20 $o/tail_$v.log; exit 1; }
  python -c "import json; l=[x for x in open('$o/tail_$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
for v in ${PROFS:-prof11 prof00}; do
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 300 python tools/bwd_prof.py 3 4 > $o/bwdprof_$v.log 2>&1 || { tail -20 $o/bwdprof_$v.log; exit 1; }
  echo "== $v"; head -12 $o/bwdprof_$v.log; grep "\[A B\]" $o/bwdprof_$v.log
done
