#!/bin/bash
# round-4 pass V: the fused native matcher and the sliding-window row blur (tests, SIFT timing), the config-5 stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_stream.py tests/test_gpu_maps.py > gpurun_out/r04v_tests.log 2>&1 || { tail -40 gpurun_out/r04v_tests.log; exit 1; }
tail -1 gpurun_out/r04v_tests.log
timeout -k 10 300 python tools/sift_bench.py > gpurun_out/r04v_sift.txt 2>&1 || { tail -20 gpurun_out/r04v_sift.txt; exit 1; }
cat gpurun_out/r04v_sift.txt
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04v_demo_stream.json 2> gpurun_out/r04v_demo_stream.err || { tail -20 gpurun_out/r04v_demo_stream.err; exit 1; }
cat gpurun_out/r04v_demo_stream.json
PTZ_SIFT_ROWS_SW=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04v_demo_stream_rows.json 2> gpurun_out/r04v_demo_stream_rows.err || { tail -20 gpurun_out/r04v_demo_stream_rows.err; exit 1; }
cat gpurun_out/r04v_demo_stream_rows.json
