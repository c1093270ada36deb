#!/bin/bash
# GPU box: backward-kernel section timers (TOG_BWD_PROF build in ab/libtog_prof.so) at several batch sizes
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for b in ${BATCHES:-1 8192}; do
  TOG_LIBRARY=ab_libs/prof/libtog.so timeout -k 10 300 python tools/bwd_prof.py ${STEPS:-3} $b > gpurun_out/bwd_prof_b$b.log 2>&1 || exit $?
done
