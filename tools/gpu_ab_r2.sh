#!/bin/bash
# Backward-pass section profile (TOG_BWD_PROF build) and the MFMA A/B (tools/mfma_ab.py), each step timed.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
set -o pipefail
TOG_LIBRARY=build_ab/prof/libtog.so timeout -k 10 300 python tools/bwd_prof.py 3 8192 > gpurun_out/ab/bwd_prof_b8192.log 2>&1 || exit 1
TOG_LIBRARY=build_ab/prof/libtog.so timeout -k 10 300 python tools/bwd_prof.py 3 4 > gpurun_out/ab/bwd_prof_b4.log 2>&1 || exit 1
timeout -k 10 400 python tools/mfma_ab.py team-valu > gpurun_out/ab/mfma_team.json 2> gpurun_out/ab/mfma_team.err || exit 1
TOG_BWD=lds timeout -k 10 400 python tools/mfma_ab.py lds-valu > gpurun_out/ab/mfma_lds.json 2> gpurun_out/ab/mfma_lds.err || exit 1
TOG_BWD=lds TOG_LIBRARY=build_ab/mfma/libtog.so timeout -k 10 400 python tools/mfma_ab.py lds-mfma > gpurun_out/ab/mfma_mfma.json 2> gpurun_out/ab/mfma_mfma.err || exit 1
cat gpurun_out/ab/*.json
