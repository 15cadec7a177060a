# Round-3: GPU tests touched by the default blocked back-solve (config 3, distributed, grid, two-level order),
# then config-4 A/B: 2 x 2 trailing blocks (default) vs one task per tile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py tests/test_gpu_config3.py tests/test_gpu_distributed.py tests/test_gpu_stream.py -k "not config4_" -x -q --timeout 400 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r03z_tests.log; exit 1; }
tail -2 gpurun_out/r03z_tests.log
BENCH_ARGS="--config config4 --steps 10 --warmup 2 --no-accuracy" VARIANTS="default ENV_PTZBA_CHOL_BLOCKS=0" bash tools/gpu_lib_ab.sh || exit 1
