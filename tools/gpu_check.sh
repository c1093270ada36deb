#!/bin/bash
# GPU-box check: parity tests, then a short bench, then (optionally) a rocprofv3 kernel trace.
# Stops at the first GPU fault / abort / timeout (exit codes other than pytest's 0/1).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
{ echo "nproc: $(nproc)"; echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)";
  python3 -c 'import os; print("affinity:", len(os.sched_getaffinity(0)))';
  grep -m1 "model name" /proc/cpuinfo; } > gpurun_out/hostinfo.txt 2>&1
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout ${PER_TEST_TIMEOUT:-300} --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
if [ $brc -ne 0 ]; then echo "bench exit $brc: stopping"; exit $brc; fi
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  echo "rocprof exit $?"
  find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
