#!/bin/bash
# Quick GPU iteration: the core parity tests, then the default bench window (no solve leg) + kernel trace.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_golden.py tests/test_quad_maze.py tests/test_step_api.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_quick.log 2>&1 || { tail -30 gpurun_out/gpu_quick.log; exit 1; }
tail -2 gpurun_out/gpu_quick.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve-leg ${BENCH_ARGS:-} > gpurun_out/bench_q.log 2>&1 || { tail -20 gpurun_out/bench_q.log; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_q.log') if x.startswith('{')][-1]; d=json.loads(l)
print('value', d['value'], 'ms/step', d['ms_per_step'], d['roofline']['kernel_ms'])"
if [ -n "$TRACE" ]; then TAG=q NO_SQ=1 STEPS=20 bash tools/profile_round.sh > gpurun_out/pr_q.log 2>&1 && head -16 gpurun_out/summ_q/rocprof_summary.txt; fi
