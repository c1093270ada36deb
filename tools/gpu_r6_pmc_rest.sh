#!/bin/bash
# Round 6: PMC traffic summaries (FETCH_SIZE / WRITE_SIZE passes, stamped with the libtog.so hash) for the
# secondary workloads that had none, copied where bench.py looks for them, then those bench lines again.
#   TAG=r6x bash tools/gpu_r6_pmc_rest.sh
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
T=${TAG:-r6x}
mkdir -p gpurun_out/$T
for wl in ${WLS:-cartpole maze_infeasible quadrotor_tv}; do
  BENCH_ARGS="--workload $wl" TAG=${T}_$wl NO_SQ=1 bash tools/profile_round.sh > /dev/null || exit 1
  cp gpurun_out/summ_${T}_$wl/traffic.json profiles/${T}_${wl}_traffic.json || exit 1
  timeout -k 10 600 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/$T/bench_${wl}_pmc.json \
    2> gpurun_out/$T/bench_${wl}_pmc.err || { tail gpurun_out/$T/bench_${wl}_pmc.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/$T/bench_${wl}_pmc.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$wl', d['value'], d['window_rate'], r['kernel'], r['frac'], r['traffic'], r.get('algorithmic_bytes_per_launch'))"
done
