# Round-3: parity of the two-level dissection (config 3, small oracle problem, multi-rank), of the 2 x 2
# trailing blocks (grid) and of the chunk-pair K2 (mf2), then config-3 A/B: HEAD~ library (libptzba_base.so)
# vs the tree, the one-level order, the blocked back-solve, the chunk-pair K2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py tests/test_gpu_config3.py tests/test_gpu_ba.py tests/test_gpu_distributed.py -k "not config4_" -x -v --timeout 400 --timeout-method thread > gpurun_out/r03y_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r03y_tests.log; exit 1; }
tail -3 gpurun_out/r03y_tests.log
VARIANTS="default base ENV_PTZBA_ND_DEPTH=1 ENV_PTZBA_BACKSOLVE=blk ENV_PTZBA_SCHUR=mf2" bash tools/gpu_lib_ab.sh || exit 1
