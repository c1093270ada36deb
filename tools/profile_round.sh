#!/bin/bash
# Round profile on the GPU box, summarised there (the rocprofv3 databases are too large to copy back):
#   TAG=r2 bash tools/profile_round.sh            -> gpurun_out/summ_<TAG>/{rocprof_summary.txt,traffic.json,sq.txt}
# kernel-trace + FETCH_SIZE + WRITE_SIZE passes (tools/profile.sh) and one SQ pass (tools/profile_sq.sh) over
# the bench window (--no-solve-leg: the whole-solve leg would add thousands of tail-step dispatches).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r2}
S=gpurun_out/summ_$TAG
mkdir -p "$S"
set -o pipefail
export BENCH_ARGS="--no-solve-leg ${BENCH_ARGS:-}"
TAG=$TAG STEPS=${STEPS:-20} bash tools/profile.sh > "$S/profile.log" 2>&1 || { tail -20 "$S/profile.log"; exit 1; }
python3 tools/rocpd_summary.py gpurun_out/prof_$TAG "$S/traffic.json" > "$S/rocprof_summary.txt" || exit 1
if [ -z "$NO_SQ" ]; then
  TAG=${TAG}sq STEPS=3 bash tools/profile_sq.sh > "$S/sq.log" 2>&1 || { tail -20 "$S/sq.log"; exit 1; }
  python3 -c "import sys; sys.path.insert(0, 'tools'); import rocpd_summary as r; r.sq_summary('gpurun_out/prof_${TAG}sq')" \
    > "$S/sq.txt" || exit 1
fi
grep -h -E "avg_ms|\"value\"" gpurun_out/prof_$TAG/trace.log | tail -1 > "$S/bench_line.json" || true
rm -rf gpurun_out/prof_$TAG gpurun_out/prof_${TAG}sq
head -30 "$S/rocprof_summary.txt"
