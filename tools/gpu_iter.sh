set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_kuka.py tests/test_quad_maze.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_sub.log 2>&1 || { tail -20 gpurun_out/gpu_tests_sub.log; exit 1; }
tail -2 gpurun_out/gpu_tests_sub.log
timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-solve-leg > gpurun_out/bench.log 2>&1 || exit 1
tail -c 600 gpurun_out/bench.log
TOG_LIBRARY=build_ab/prof/libtog.so timeout -k 10 300 python tools/bwd_prof.py 3 8192 > gpurun_out/bwd_prof_b8192.log 2>&1 || exit 1
TOG_LIBRARY=build_ab/prof/libtog.so timeout -k 10 300 python tools/bwd_prof.py 3 4 > gpurun_out/bwd_prof_b4.log 2>&1 || exit 1
cat gpurun_out/bwd_prof_b8192.log gpurun_out/bwd_prof_b4.log
