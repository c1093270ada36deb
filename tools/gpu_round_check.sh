#!/bin/bash
# gpu_round_check.sh <tag>: round-end check of the committed tree: GPU suite, smoke, default bench (window + solve + CPU baseline),
# the multi-rank bench path at world 1 (RCCL stats exchange), each step under its own limit.
cd "$(dirname "$0")/.." || exit 1
t=${1:-r2}
mkdir -p gpurun_out/$t
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$t/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$t/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$t/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$t/smoke.log 2>&1 || { tail -20 gpurun_out/$t/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/$t/bench.log 2>&1 || { tail -20 gpurun_out/$t/bench.log; exit 1; }
TOG_BENCH_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/$t/bench_dist1.log 2>&1 || { tail -20 gpurun_out/$t/bench_dist1.log; exit 1; }
tail -c 1200 gpurun_out/$t/bench.log
