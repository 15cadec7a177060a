#!/bin/bash
# round-4 pass K: the keyframe-path host changes (resident descriptor sets, lazy keyframe lists, vectorised cap,
# set_problem bitmap / counting sort / 64K-item threads) under the front-end / stream / map / BA tests, the config-5
# stream, then the K2 item-count A/B (fewer, larger work items)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_stream.py tests/test_gpu_maps.py tests/test_gpu_ba.py tests/test_gpu_config3.py > gpurun_out/r04k_tests.log 2>&1 || { tail -40 gpurun_out/r04k_tests.log; exit 1; }
tail -1 gpurun_out/r04k_tests.log
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04k_demo_stream.json 2> gpurun_out/r04k_demo_stream.err || { tail -20 gpurun_out/r04k_demo_stream.err; exit 1; }
cat gpurun_out/r04k_demo_stream.json
REPS=2 STEPS=200 AB_ENVS="PTZBA_S2_ITEMS=128 PTZBA_S2_ITEMS=192 PTZBA_S2_ITEMS=256 PTZBA_S2_ITEMS=320" bash tools/r04ab.sh || exit 1
