# Round-3: two-level dissection parity at a small size, grid tests incl. 2 x 2 trailing blocks, then
# config-3 A/B (HEAD library libptzba_base.so vs the tree) and config-4 A/B (blocks vs per-tile tasks)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py -k "not config4_" -x -v --timeout 300 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -3 gpurun_out/r03x_tests.log
VARIANTS="default base" bash tools/gpu_lib_ab.sh || exit 1
BENCH_ARGS="--config config4 --steps 10 --warmup 2 --no-accuracy" VARIANTS="default ENV_PTZBA_CHOL_BLOCKS=0" bash tools/gpu_lib_ab.sh || exit 1
