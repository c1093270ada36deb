#!/bin/bash
# Round 5 final checks on the GPU box, in two parts (each fits one gpurun call):
#   PART=suite bash tools/gpu_final_r5.sh   -> the whole -m gpu suite, then smoke()
#   PART=bench bash tools/gpu_final_r5.sh   -> the default bench line, the round profile of its window
#                                             (kernel trace, FETCH/WRITE, SQ) and the B = 1 tail line
# Outputs in gpurun_out/final5/. Every GPU step has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/final5
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
if [ "${PART:-suite}" = suite ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
else
  timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  tail -c 600 $OUT/bench.log
  TAG=r5f NO_SQ=1 bash tools/profile_round.sh > $OUT/pr_r5f.log 2>&1 || { tail -20 $OUT/pr_r5f.log; exit 1; }
  timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > $OUT/tail_b1.log 2>&1 \
    || { tail -20 $OUT/tail_b1.log; exit 1; }
  tail -c 300 $OUT/tail_b1.log
fi
