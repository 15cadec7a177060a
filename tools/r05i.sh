#!/bin/bash
# round 5: stream / map / drop-in tests after the first-keyframe warm-up, then the stream twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r05i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_maps.py tests/test_gpu_ba.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1 2; do
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/${T}_demo_stream_$k.json 2> gpurun_out/${T}_demo_stream_$k.err || { tail -20 gpurun_out/${T}_demo_stream_$k.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_demo_stream_$k.json').read()); print(round(d['fps_end_to_end'],1), d['tracking_ms'], d['keyframe_ba_ms'], d.get('keyframe_ba_slowest_breakdown_ms'))"
done
echo done
