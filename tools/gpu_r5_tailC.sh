#!/bin/bash
# Round 5: per-step trace of the headline solve + the per-step statistics of the same (deterministic) solve.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/tools/tail_solve.py" --batch 8192) > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
DB=$(find $OUT/trace -name "*.db" | head -1)
python3 tools/tail_trace.py "$DB" --last 8000 --dump $OUT/steps.json > $OUT/tail_trace.txt || exit 1
rm -rf $OUT/trace
timeout -k 10 300 python3 tools/tail_solve.py --batch 8192 --stats-pass > $OUT/stats.json 2> $OUT/stats.err || { tail $OUT/stats.err; exit 1; }
ls -la $OUT
