set -o pipefail
VARIANTS="default nofold" TESTS="tests/test_gpu_ba.py tests/test_gpu_config3.py tests/test_gpu_stream.py" bash tools/gpu_lib_ab.sh
