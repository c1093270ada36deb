#!/bin/bash
# Round-end evidence: full GPU suite, default bench (window + whole-solve leg + CPU baseline), profile of the
# bench window (trace, FETCH/WRITE, SQ), Kuka trace, tail bench. Each GPU step under its own limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/final
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || { tail -30 gpurun_out/final/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || { tail -20 gpurun_out/final/bench.log; exit 1; }
TAG=r2c bash tools/profile_round.sh > gpurun_out/final/pr_r2c.log 2>&1 || exit 1
TAG=r2ckuka STEPS=10 NO_SQ=1 BENCH_ARGS="--workload kuka" bash tools/profile_round.sh > gpurun_out/final/pr_r2ckuka.log 2>&1 || exit 1
for w in cartpole quad_maze maze_infeasible; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > gpurun_out/final/bench_$w.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > gpurun_out/final/tail_b1.log 2>&1 || exit 1
tail -c 800 gpurun_out/final/bench.log
