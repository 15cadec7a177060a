set -o pipefail
mkdir -p gpurun_out
PTZBA_LIB=$PWD/pan-tilt-zoom-slam_amd/libptzba_plain.so timeout -k 10 300 python -u -m pytest tests/test_gpu_config3.py -k "longer or residual" tests/test_gpu_ba.py -x -q --timeout 120 --timeout-method thread > gpurun_out/plain_tests.log 2>&1 || { tail -30 gpurun_out/plain_tests.log; exit 1; }
tail -3 gpurun_out/plain_tests.log
ALT=$PWD/pan-tilt-zoom-slam_amd/libptzba_plain.so bash tools/ab_libs.sh
