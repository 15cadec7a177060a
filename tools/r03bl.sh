# Round-3: 2 x 2 trailing blocks in every plan (also DT = 1): GPU parity subset, then config-3 A/B (blocks on /
# off, one-level order)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested2.py tests/test_gpu_config4.py tests/test_gpu_config3.py tests/test_gpu_ba.py tests/test_gpu_stream.py tests/test_gpu_ekf.py -k "not config4_" -x -q --timeout 400 --timeout-method thread > gpurun_out/r03bl_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03bl_tests.log; exit 1; }
tail -1 gpurun_out/r03bl_tests.log
VARIANTS="default ENV_PTZBA_CHOL_BLOCKS=0 ENV_PTZBA_ND_DEPTH=1" bash tools/gpu_lib_ab.sh || exit 1
