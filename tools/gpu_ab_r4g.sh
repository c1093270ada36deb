mkdir -p gpurun_out/r4g
export TMPDIR=/tmp
K='models_equal_oracle and kuka'
(cd ab_libs/r3tree && timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3) > gpurun_out/r4g/r3.txt 2>&1
TOG_LS=replay timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/replay.txt
TOG_LS_NOPEND=1 timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/nopend.txt
TOG_BWD=lds timeout -k 10 300 python -m pytest tests/test_minimum_time.py -k "$K" -m gpu -q -p no:cacheprovider 2>&1 | tail -3 > gpurun_out/r4g/lds.txt
for f in r3 replay nopend lds; do echo "== $f"; cat gpurun_out/r4g/$f.txt; done
