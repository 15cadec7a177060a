#!/bin/bash
# round-4 pass R: the full GPU suite on the current tree, the config-5 stream and its host profile (callers)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04r_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04r_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04r_gpu_tests.log
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04r_demo_stream.json 2> gpurun_out/r04r_demo_stream.err || { tail -20 gpurun_out/r04r_demo_stream.err; exit 1; }
cat gpurun_out/r04r_demo_stream.json
timeout -k 10 300 python tools/profile_stream.py gpurun_out/r04r_stream_prof.txt > gpurun_out/r04r_stream_prof.json 2> gpurun_out/r04r_stream_prof.err || { tail -20 gpurun_out/r04r_stream_prof.err; exit 1; }
