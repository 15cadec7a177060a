#!/bin/bash
# config-5 stream twice after the feature-count fix (keyframe path timing, box variance)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z2_demo_stream_$k.json 2> gpurun_out/r04z2_demo_stream_$k.err || { tail -20 gpurun_out/r04z2_demo_stream_$k.err; exit 1; }
  cat gpurun_out/r04z2_demo_stream_$k.json
done
