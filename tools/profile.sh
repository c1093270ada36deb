#!/bin/bash
# GPU-box profiling of bench.py: kernel-trace stats, then two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE — they do not fit one pass on gfx950). Outputs under gpurun_out/prof_<tag>/.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-5}
ARGS="--steps $STEPS --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
ROOT=$(pwd)
set -o pipefail
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/bench.py" $ARGS) \
  > "$OUT/trace.log" 2>&1 || { echo "kernel-trace pass failed"; tail -20 "$OUT/trace.log"; exit 1; }
(cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/fetch" -o run -- python3 "$ROOT/bench.py" $ARGS) \
  > "$OUT/fetch.log" 2>&1 || { echo "FETCH_SIZE pass failed"; tail -20 "$OUT/fetch.log"; exit 1; }
(cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/write" -o run -- python3 "$ROOT/bench.py" $ARGS) \
  > "$OUT/write.log" 2>&1 || { echo "WRITE_SIZE pass failed"; tail -20 "$OUT/write.log"; exit 1; }
find "$OUT" -name "*.csv" | head -20
tail -2 "$OUT/trace.log"
