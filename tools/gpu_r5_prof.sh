#!/bin/bash
# Round 5 profiles of the bench window for configs 3, 4 and 5: per workload the
# kernel-trace stats, FETCH_SIZE and WRITE_SIZE passes (traffic.json) and one SQ pass; the Kuka SQ pass adds
# the fp64 matrix-core counters. Summaries land in gpurun_out/summ_<TAG>_<workload>/.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5k}
WLS=${WLS:-"quadrotor quad_maze kuka"}
for w in $WLS; do
  if [ "$w" = kuka ]; then
    export CTRS="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
  else
    unset CTRS
  fi
  TAG=${TAG}_$w BENCH_ARGS="--workload $w" STEPS=${STEPS:-10} bash tools/profile_round.sh || exit 1
done
