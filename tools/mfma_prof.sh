#!/bin/bash
# MFMA utilisation of the Kuka bench (config 5): a kernel-trace pass and one PMC pass of the MFMA counters,
# summarised on the box into gpurun_out/mfma_<TAG>.json (tools/mfma_summary.py).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r6}
OUT=gpurun_out/prof_mfma_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
ARGS="--workload kuka --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-solve-leg"
set -o pipefail
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run -- python3 "$ROOT/bench.py" $ARGS) \
  > "$OUT/trace.log" 2>&1 || { echo "kernel-trace pass failed"; tail -20 "$OUT/trace.log"; exit 1; }
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d "$ROOT/$OUT/mfma" -o run -- python3 "$ROOT/bench.py" $ARGS) > "$OUT/mfma.log" 2>&1 || { echo "MFMA pass failed"; tail -20 "$OUT/mfma.log"; exit 1; }
python3 tools/mfma_summary.py "$OUT" "gpurun_out/mfma_${TAG}_kuka.json" k_kuka_chain || exit 1
rm -rf "$OUT/trace" "$OUT/mfma"
