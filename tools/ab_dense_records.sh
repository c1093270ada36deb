cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out/r5m
for v in dense packed; do
  if [ $v = dense ]; then export TOG_DENSE_RECORDS=1; else unset TOG_DENSE_RECORDS; fi
  timeout -k 10 300 python bench.py --workload quad_maze --no-solve-leg --no-cpu-baseline --steps 10 > gpurun_out/r5m/bench_$v.json 2> gpurun_out/r5m/bench_$v.err || { tail gpurun_out/r5m/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r5m/bench_$v.json').read().strip().splitlines()[-1]);print('$v',d['window_rate'],d['roofline']['kernel_ms'])"
done
