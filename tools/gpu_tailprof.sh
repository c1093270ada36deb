#!/bin/bash
# Kernel trace of the one-trajectory tail step (and the counter list for later PMC passes).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-tail}
S=gpurun_out/summ_$TAG
mkdir -p "$S"
export TMPDIR=/tmp
ROOT=$(pwd)
set -o pipefail
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > "$ROOT/$S/avail.txt" 2>&1) || true
grep -i -E "icache|ifetch|SQC_|INST_LEVEL|WAIT_INST" "$S/avail.txt" | head -60 > "$S/avail_inst.txt" || true
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG/trace" -o run -- python3 "$ROOT/bench.py" --batch ${BATCH:-1} --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg) \
  > "$S/trace.log" 2>&1 || { tail -20 "$S/trace.log"; exit 1; }
find gpurun_out/prof_$TAG -name "*.db" | head
python3 tools/rocpd_summary.py gpurun_out/prof_$TAG > "$S/rocprof_summary.txt" || exit 1
rm -rf gpurun_out/prof_$TAG
head -24 "$S/rocprof_summary.txt"
