# Round-3 A/B: a level's first 240 tasks by value + the rest by pointer (tree) vs all-by-pointer levels beyond
# 240 tasks (libptzba_prev.so); config 3, then config 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py -k "not config4_" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03hy_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03hy_tests.log; exit 1; }
tail -1 gpurun_out/r03hy_tests.log
VARIANTS="default prev" bash tools/gpu_lib_ab.sh || exit 1
BENCH_ARGS="--config config4 --steps 10 --warmup 2 --no-accuracy" VARIANTS="default prev" bash tools/gpu_lib_ab.sh || exit 1
