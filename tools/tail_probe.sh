cd /root/repo || exit 1
mkdir -p gpurun_out/tail
export TMPDIR=/tmp
for b in 1 64 1024; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tail/bench_b$b.log 2>&1 || exit $?
done
ROOT=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/tail/prof" -o run -- python3 "$ROOT/bench.py" --batch 1 --steps 10 --warmup 2 --no-cpu-baseline) > gpurun_out/tail/prof.log 2>&1 || exit $?
find gpurun_out/tail/prof -name "*stats*"
