#!/bin/bash
# SIFT per-frame host trims (cached tables, pinned image upload): the front-end / stream GPU tests, the stream twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_stream.py tests/test_gpu_maps.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z6_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z6_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z6_gpu_tests.log
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z6_demo_stream_$k.json 2> gpurun_out/r04z6_demo_stream_$k.err || { tail -20 gpurun_out/r04z6_demo_stream_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04z6_demo_stream_$k.json')); print(d['fps_end_to_end'], d['tracking_ms'], d['keyframe_ba_ms'])"
done
