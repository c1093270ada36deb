mkdir -p gpurun_out/r4g
export TMPDIR=/tmp
K='models_equal_oracle and kuka'
(cd ab_libs/r3tree && timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3) > gpurun_out/r4g/r3.txt 2>&1
TOG_LS=replay timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/replay.txt
TOG_LS_NOPEND=1 timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/nopend.txt
TOG_BWD=lds timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/lds.txt
for f in r3 replay nopend lds; do echo "== $f"; cat gpurun_out/r4g/$f.txt; done
# Kuka bench: the stage-chain Jacobian (default) against the dual-staged A/B, then the profile of the default
timeout -k 10 300 python bench.py --workload kuka --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r4g/bench_kuka.txt 2>&1 || exit 1
TOG_KUKA_JAC=dual timeout -k 10 300 python bench.py --workload kuka --steps 10 --warmup 2 --no-cpu-baseline --no-solve-leg > gpurun_out/r4g/bench_kuka_dual.txt 2>&1 || exit 1
tail -1 gpurun_out/r4g/bench_kuka.txt | cut -c1-300
tail -1 gpurun_out/r4g/bench_kuka_dual.txt | cut -c1-300
TAG=r4gkuka NO_SQ=1 STEPS=10 BENCH_ARGS="--workload kuka" bash tools/profile_round.sh > gpurun_out/r4g/prof.txt 2>&1 || { tail -5 gpurun_out/r4g/prof.txt; exit 1; }
head -24 gpurun_out/summ_r4gkuka/rocprof_summary.txt
