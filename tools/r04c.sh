#!/bin/bash
# round-4 config-5 keyframe-path pass: stream/map/front-end GPU tests, then a cProfile'd stream run with the
# set_problem phase timers, then the plain stream demo
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_maps.py tests/test_gpu_frontend.py tests/test_gpu_ba.py > gpurun_out/r04c_tests.log 2>&1 || { tail -30 gpurun_out/r04c_tests.log; exit 1; }
tail -2 gpurun_out/r04c_tests.log
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python tools/profile_stream.py gpurun_out/r04c_stream_prof.txt --frames 150 > gpurun_out/r04c_stream_prof.json 2> gpurun_out/r04c_setup_timing.txt || exit 1
cat gpurun_out/r04c_stream_prof.json
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04c_demo_stream.json 2> gpurun_out/r04c_demo_stream.err || exit 1
cat gpurun_out/r04c_demo_stream.json
