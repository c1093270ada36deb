#!/bin/bash
# f64 latency microbenchmark + quick parity subset + benches (tools/gpu_r3.sh with TESTS)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/${TAG:-r3}
timeout -k 10 60 tools/microbench/lat_f64 > gpurun_out/${TAG:-r3}/lat_f64.txt 2>&1 || exit 1
cat gpurun_out/${TAG:-r3}/lat_f64.txt
TESTS="${TESTS:-tests/test_gpu_parity.py tests/test_quad_maze.py tests/test_step_api.py}" bash tools/gpu_r3.sh
