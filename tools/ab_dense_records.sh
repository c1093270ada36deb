cd $GRAFT_REPO_ROOT || exit 1
OUTD=gpurun_out/${TAG:-r5m}; mkdir -p $OUTD
for v in dense packed; do
  if [ $v = dense ]; then export TOG_DENSE_RECORDS=1; else unset TOG_DENSE_RECORDS; fi
  timeout -k 10 300 python bench.py --workload quad_maze --no-solve-leg --no-cpu-baseline --steps 10 > $OUTD/bench_$v.json 2> $OUTD/bench_$v.err || { tail $OUTD/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUTD/bench_$v.json').read().strip().splitlines()[-1]);print('$v',d['window_rate'],d['roofline']['kernel_ms'])"
done
