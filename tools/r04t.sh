#!/bin/bash
# round-4 pass T: the sliding-window SIFT column pass (bit-exact vs the oracle, timing), the front-end tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frontend.py > gpurun_out/r04t_tests.log 2>&1 || { tail -40 gpurun_out/r04t_tests.log; exit 1; }
tail -1 gpurun_out/r04t_tests.log
timeout -k 10 300 python tools/sift_bench.py > gpurun_out/r04t_sift.txt 2>&1 || { tail -20 gpurun_out/r04t_sift.txt; exit 1; }
cat gpurun_out/r04t_sift.txt
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04t_demo_stream.json 2> gpurun_out/r04t_demo_stream.err || { tail -20 gpurun_out/r04t_demo_stream.err; exit 1; }
cat gpurun_out/r04t_demo_stream.json
PTZ_SIFT_COLS_SW=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04t_demo_stream_colsw.json 2> gpurun_out/r04t_demo_stream_colsw.err || { tail -20 gpurun_out/r04t_demo_stream_colsw.err; exit 1; }
cat gpurun_out/r04t_demo_stream_colsw.json
