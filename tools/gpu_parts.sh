#!/bin/bash
# gpu_parts.sh <tag>: generic-cost GPU tests, then the stream-split (--parts) A/B on the Kuka and quadrotor workloads
cd "$(dirname "$0")/.." || exit 1
t=${1:-parts}
mkdir -p gpurun_out/$t
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_generic_cost.py -x -v --timeout 120 --timeout-method thread > gpurun_out/$t/gc_tests.log 2>&1 || { tail -30 gpurun_out/$t/gc_tests.log; exit 1; }
tail -1 gpurun_out/$t/gc_tests.log
for w in kuka quadrotor; do
  for p in 1 2; do
    timeout -k 10 300 python bench.py --workload $w --steps 10 --parts $p --no-cpu-baseline --no-solve-leg > gpurun_out/$t/bench_${w}_p$p.log 2>&1 || { tail -20 gpurun_out/$t/bench_${w}_p$p.log; exit 1; }
    python -c "import json,sys; l=[x for x in open('gpurun_out/$t/bench_${w}_p$p.log') if x.startswith('{')][-1]; d=json.loads(l); print('$w', $p, d['value'], d['ms_per_step'], d['roofline'].get('kernel_ms'))"
  done
done
