#!/bin/bash
# round 5: front-end tests (empty sets, >255 values), the stream with its slowest-keyframe breakdown, bench + stream leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r05h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_fe_tests.log 2>&1 || { tail -30 gpurun_out/${T}_fe_tests.log; exit 1; }
tail -1 gpurun_out/${T}_fe_tests.log
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/${T}_demo_stream.json 2> gpurun_out/${T}_demo_stream.err || { tail -20 gpurun_out/${T}_demo_stream.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_demo_stream.json').read()); print(d['fps_end_to_end'], d['keyframe_ba_ms'], d.get('keyframe_ba_slowest_breakdown_ms'), d.get('keyframe_ba_breakdown_ms'))"
timeout -k 10 400 python bench.py --steps 300 --no-cpu-baseline --no-cold --no-secondary > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), d['config5'])"
echo done
