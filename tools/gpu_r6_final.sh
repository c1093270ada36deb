#!/bin/bash
# Round 6 final measurement, part PART (1: smoke + GPU suite + headline profile passes; 2: secondary profiles,
# MFMA, bench lines with the stamped PMC summaries copied into profiles/ on the box, IROS maze).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
T=${TAG:-r6z}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ "$PART" = 1 ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
  cat $OUT/smoke.txt
  timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/suite.log 2>&1
  rc=$?; tail -2 $OUT/suite.log; grep -E "FAILED|ERROR" $OUT/suite.log | head -20
  [ $rc -eq 0 ] || exit $rc
  TAG=$T bash tools/profile_round.sh || exit 1
  exit 0
fi
BENCH_ARGS="--workload quad_maze" TAG=${T}q NO_SQ=1 bash tools/profile_round.sh > /dev/null || exit 1
BENCH_ARGS="--workload kuka" TAG=${T}k NO_SQ=1 bash tools/profile_round.sh > /dev/null || exit 1
TAG=$T bash tools/mfma_prof.sh > /dev/null || exit 1
# this build's PMC summaries where bench.py looks for them
cp gpurun_out/summ_${T}/traffic.json profiles/${T}_traffic.json 2>/dev/null
cp gpurun_out/summ_${T}q/traffic.json profiles/${T}_quad_maze_traffic.json || exit 1
cp gpurun_out/summ_${T}k/traffic.json profiles/${T}_kuka_traffic.json || exit 1
cp gpurun_out/mfma_${T}_kuka.json profiles/${T}_kuka_mfma.json || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
for wl in cartpole quad_maze kuka maze_infeasible quadrotor_tv; do
  timeout -k 10 600 python bench.py --workload $wl --no-cpu-baseline > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail $OUT/bench_$wl.err; exit 1; }
done
timeout -k 10 600 python tools/iros_maze.py --batch 256 --out $OUT/iros_maze_b256.json > /dev/null || exit 1
timeout -k 10 300 python tools/iros_maze.py --batch 1 --out $OUT/iros_maze_b1.json > /dev/null || exit 1
python3 - <<PY
import json
for f in ["bench", "bench_cartpole", "bench_quad_maze", "bench_kuka", "bench_maze_infeasible", "bench_quadrotor_tv"]:
    d = json.loads(open("$OUT/%s.json" % f).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, "value", d["value"], "window", d["window_rate"], "ms/step", d["ms_per_step"], "frac", r["frac"], "traffic", r["traffic"], "kernel_ms", r["kernel_ms"])
PY
