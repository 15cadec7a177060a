#!/bin/bash
# round-4 pass F: schedule bitwise tests, rank-tree distributed tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_ba.py -k "knobs or single_launch" > gpurun_out/r04f_knob_tests.log 2>&1 || { tail -30 gpurun_out/r04f_knob_tests.log; exit 1; }
tail -1 gpurun_out/r04f_knob_tests.log
timeout -k 10 870 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_distributed.py > gpurun_out/r04f_dist_tests.log 2>&1 || { tail -40 gpurun_out/r04f_dist_tests.log; exit 1; }
tail -1 gpurun_out/r04f_dist_tests.log
