set -o pipefail
VARIANTS="default ENV_PTZBA_NO_FUSED_PREP=1" TESTS="tests/test_gpu_ba.py tests/test_gpu_config3.py tests/test_gpu_ekf.py tests/test_gpu_distributed.py tests/test_gpu_stream.py tests/test_gpu_maps.py tests/test_gpu_config4.py" bash tools/gpu_lib_ab.sh
