# Round-3 A/B: two-level nested dissection at config 3 (default) vs the one-level order (PTZBA_ND_DEPTH=1);
# parity: config-3, BA and multi-rank GPU tests first
set -o pipefail
mkdir -p gpurun_out
TESTS="tests/test_gpu_config3.py tests/test_gpu_ba.py tests/test_gpu_distributed.py" VARIANTS="default ENV_PTZBA_ND_DEPTH=1" bash tools/gpu_lib_ab.sh
