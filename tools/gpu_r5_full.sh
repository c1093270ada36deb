#!/bin/bash
# Round 5: the whole GPU suite (no -x: every failure listed), the smoke, the B = 1 tail probe and the bench.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r5h}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests "${KARG[@]}" > $OUT/suite.log 2>&1
rc=$?; tail -2 $OUT/suite.log; grep -E "FAILED|ERROR" $OUT/suite.log | head -30
[ $rc -eq 0 ] || [ -n "$KEEPGOING" ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 200 python tools/tail_solve.py --offset 1457 --profile > $OUT/tail_b1.json 2> $OUT/tail_b1.err || { tail $OUT/tail_b1.err; exit 1; }
cat $OUT/tail_b1.json
timeout -k 10 400 python bench.py --cpu-seconds 4 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
s=d['solve_rate'];print('value',d['value'],'window',d['window_rate'],'ms/step',d['ms_per_step'],'solve',s['wall_s'],s['batch_steps'],s['steps'],s['ms_per_batch_step'])
print('kernel_ms',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'])"
