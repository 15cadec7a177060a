# Round-3: blocked back-solve task records by value: parity subset, then config-3 and config-4 A/B against the
# pointer-only records (PTZBA_BSB_TASKS_PTR=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py tests/test_gpu_config3.py -k "not config4_" -x -q --timeout 400 --timeout-method thread > gpurun_out/r03bv_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03bv_tests.log; exit 1; }
tail -1 gpurun_out/r03bv_tests.log
VARIANTS="default ENV_PTZBA_BSB_TASKS_PTR=1" bash tools/gpu_lib_ab.sh || exit 1
BENCH_ARGS="--config config4 --steps 10 --warmup 2 --no-accuracy" VARIANTS="default ENV_PTZBA_BSB_TASKS_PTR=1" bash tools/gpu_lib_ab.sh || exit 1
