#!/bin/bash
# keyframe-path checks: the GPU tests that cover it (maps, stream, front-end, drop-in BA), then the stream twice and
# once with set_problem's phase times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_maps.py tests/test_gpu_stream.py tests/test_gpu_frontend.py tests/test_gpu_ba.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z3_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z3_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z3_gpu_tests.log
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z3_demo_stream_$k.json 2> gpurun_out/r04z3_demo_stream_$k.err || { tail -20 gpurun_out/r04z3_demo_stream_$k.err; exit 1; }
  cat gpurun_out/r04z3_demo_stream_$k.json
done
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > /dev/null 2> gpurun_out/r04z3_stream_setup_timing.txt || { tail -20 gpurun_out/r04z3_stream_setup_timing.txt; exit 1; }
echo done
