#!/bin/bash
# pass Z4: batched set_problem uploads (one staged copy + one scatter launch) -- the full GPU suite, smoke, the default
# bench line, the stream twice and once with set_problem's phase times (batched and PTZBA_STAGE_BATCH=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04z4_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z4_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z4_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z4_smoke.log 2>&1 || { tail gpurun_out/r04z4_smoke.log; exit 1; }
tail -1 gpurun_out/r04z4_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04z4_bench.json 2> gpurun_out/r04z4_bench.err || { tail gpurun_out/r04z4_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04z4_bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernel_ms'], round(d['roofline']['frac'],3), d['dropin_call'])"
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z4_demo_stream_$k.json 2> gpurun_out/r04z4_demo_stream_$k.err || { tail -20 gpurun_out/r04z4_demo_stream_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04z4_demo_stream_$k.json')); print(d['fps_end_to_end'], d['keyframe_ba_ms'], {k: round(v, 2) for k, v in d['keyframe_ba_breakdown_ms'].items()})"
done
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > /dev/null 2> gpurun_out/r04z4_stream_setup_timing.txt || { tail -20 gpurun_out/r04z4_stream_setup_timing.txt; exit 1; }
PTZBA_STAGE_BATCH=0 PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > /dev/null 2> gpurun_out/r04z4_stream_setup_timing_nobatch.txt || { tail -20 gpurun_out/r04z4_stream_setup_timing_nobatch.txt; exit 1; }
echo done
