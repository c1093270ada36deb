#!/bin/bash
# Round 5: attribute the headline solve's tail step (config 3's slowest trajectory solved alone).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
OFF=${OFF:-1457}
timeout -k 10 200 python tools/tail_solve.py --offset $OFF --stats-pass > $OUT/tail_solve.json 2> $OUT/tail_solve.err || { tail -20 $OUT/tail_solve.err; exit 1; }
cat $OUT/tail_solve.json
timeout -k 10 200 python tools/tail_solve.py --offset $OFF --profile > $OUT/tail_solve_prof.json 2>> $OUT/tail_solve.err || exit 1
cat $OUT/tail_solve_prof.json
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/tools/tail_solve.py" --offset $OFF) > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
DB=$(find $OUT/trace -name "*.db" | head -1)
python3 tools/tail_trace.py "$DB" --last 8000 > $OUT/tail_trace.txt || exit 1
rm -rf $OUT/trace
cat $OUT/tail_trace.txt
