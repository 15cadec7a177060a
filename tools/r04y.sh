#!/bin/bash
# config-5 keyframe path: the stream with the slack allocations, its set_problem phase times, and a host profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04y_demo_stream.json 2> gpurun_out/r04y_demo_stream.err || { tail -20 gpurun_out/r04y_demo_stream.err; exit 1; }
cat gpurun_out/r04y_demo_stream.json
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > /dev/null 2> gpurun_out/r04y_stream_setup_timing.txt || { tail -20 gpurun_out/r04y_stream_setup_timing.txt; exit 1; }
timeout -k 10 400 python tools/profile_stream.py gpurun_out/r04y_stream_host_profile.txt > gpurun_out/r04y_profiled_stream.json 2>&1 || { tail -20 gpurun_out/r04y_profiled_stream.json; exit 1; }
echo done
