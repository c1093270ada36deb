#!/bin/bash
# Round 5: kernel trace of the headline solve (B = 8192), attributed over its last dispatches (the tail).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/tools/tail_solve.py" --batch 8192) > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
DB=$(find $OUT/trace -name "*.db" | head -1)
python3 tools/tail_trace.py "$DB" --last 8000 > $OUT/tail_trace.txt || exit 1

rm -rf $OUT/trace
grep -v "^\[" $OUT/trace.log | tail -3
cat $OUT/tail_trace.txt
