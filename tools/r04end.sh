#!/bin/bash
# round-4 closing check on the last code commit: the full GPU suite, smoke, the default bench line, the stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04end_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04end_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04end_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04end_smoke.log 2>&1 || { tail gpurun_out/r04end_smoke.log; exit 1; }
tail -1 gpurun_out/r04end_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04end_bench.json 2> gpurun_out/r04end_bench.err || { tail gpurun_out/r04end_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04end_bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernel_ms'], round(d['roofline']['frac'],3))"
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04end_demo_stream_$k.json 2> gpurun_out/r04end_demo_stream_$k.err || { tail -20 gpurun_out/r04end_demo_stream_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04end_demo_stream_$k.json')); print(d['fps_end_to_end'], d['keyframe_ba_ms'])"
done
