# Round-3 A/B: vectorised k_schur_reduce (SR_VEC 1, the tree) against the scalar reduce (libptzba_srvec0.so)
set -o pipefail
mkdir -p gpurun_out
TESTS="tests/test_gpu_ba.py tests/test_gpu_config3.py" VARIANTS="default srvec0" bash tools/gpu_lib_ab.sh
