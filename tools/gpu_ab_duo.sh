#!/bin/bash
# A/B of the tail backward (k_bwd_duo) variants in ab_libs/: GPU parity of the new variant, the one-trajectory
# tail bench per variant, and the per-wave section timers of the profiled builds.
#   NEW=duo_v2 OLD=duo_v1 PROFS="prof prof2" bash tools/gpu_ab_duo.sh
cd "$(dirname "$0")/.." || exit 1
o=gpurun_out/abduo; mkdir -p $o
export TMPDIR=/tmp
set -o pipefail
NEW=${NEW:-duo_v2}
for v in $NEW; do
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_tail.py tests/test_gpu_parity.py tests/test_config3_full.py} -m gpu -x -q --timeout 300 --timeout-method thread > $o/parity_$v.log 2>&1 || { tail -30 $o/parity_$v.log; exit 1; }
  echo "$v $(tail -n 1 $o/parity_$v.log)"
done
for v in ${VARIANTS:-${OLD:-duo_v1} $NEW ${OLD:-duo_v1} $NEW}; do
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $o/tail_$v.log 2>&1 || { tail -20 $o/tail_$v.log; exit 1; }
  python -c "import json; l=[x for x in open('$o/tail_$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
for pv in ${PROFS:-prof:duo prof2:duo}; do
  v=${pv%%:*}; kind=${pv##*:}
  TOG_LIBRARY=ab_libs/$v/libtog.so timeout -k 10 300 python tools/duo_prof.py 10 $kind > $o/duoprof_$v.log 2>&1 || { tail -20 $o/duoprof_$v.log; exit 1; }
  echo "== $v"; cat $o/duoprof_$v.log
done
