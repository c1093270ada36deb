#!/bin/bash
# Secondary bench lines for the other BASELINE configs (GPU box). Each step has its own time limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for w in ${WORKLOADS:-cartpole kuka quad_maze maze_infeasible}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_$w.log 2>&1 || { echo "bench $w failed ($?)"; tail -20 gpurun_out/bench_$w.log; exit 1; }
  tail -1 gpurun_out/bench_$w.log
done
