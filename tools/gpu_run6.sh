set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_camera.py tests/test_gpu_ba.py -x -q -m gpu -k "not config2 and not dedup" > gpurun_out/t6.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
bash tools/schur_variants.sh
