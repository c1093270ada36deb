#!/bin/bash
# One rocprofv3 PMC pass with SQ stall/issue counters over a short bench run (no tracing domains).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-sq}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
CTRS=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"}
(cd /tmp && timeout -k 10 600 rocprofv3 --pmc $CTRS -d "$ROOT/$OUT/sq" -o run -- python3 "$ROOT/bench.py" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}) \
  > "$OUT/sq.log" 2>&1 || { echo "SQ pass failed"; tail -30 "$OUT/sq.log"; exit 1; }
tail -2 "$OUT/sq.log"
