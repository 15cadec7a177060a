# K1 change check on one box: phase timing of the K1_TIMING build, the K1 / BA GPU tests, then a same-box
# A/B of the tree's library against $ALT (tools/ab_libs.sh)
set -o pipefail
mkdir -p gpurun_out
PTZBA_LIB=$PWD/pan-tilt-zoom-slam_amd/libptzba_k1t.so timeout -k 10 200 python tools/k1_timing.py > gpurun_out/k1t.txt 2>&1 || { tail gpurun_out/k1t.txt; exit 1; }
cat gpurun_out/k1t.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_config3.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k1_tests.log 2>&1 || { tail -30 gpurun_out/k1_tests.log; exit 1; }
tail -1 gpurun_out/k1_tests.log
bash tools/ab_libs.sh
