set -o pipefail
VARIANTS="default k1issue k1atomic" TESTS="tests/test_gpu_ba.py tests/test_gpu_ekf.py tests/test_gpu_config3.py" bash tools/gpu_lib_ab.sh
