#!/bin/bash
# round 5: stream keyframe spikes vs Python's cyclic GC (default vs gc.freeze), two runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05j}
for g in default freeze default freeze; do
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py --gc $g > gpurun_out/${T}_demo_stream_$g.json 2> gpurun_out/${T}_demo_stream_$g.err || { tail -20 gpurun_out/${T}_demo_stream_$g.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_demo_stream_$g.json').read()); print('$g', round(d['fps_end_to_end'],1), d['tracking_ms'], d['keyframe_ba_ms'], d['gc_pauses_ms'])"
done
echo done
