#!/bin/bash
# round-4 pass Z (slack allocations, streamed set_problem segments, table feature counts): the full GPU suite, smoke, the default bench line (as the driver runs it),
# the config-5 stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || { tail gpurun_out/r04z_smoke.log; exit 1; }
tail -1 gpurun_out/r04z_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || { tail gpurun_out/r04z_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04z_bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernel_ms'], round(d['roofline']['frac'],3))"
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z_demo_stream.json 2> gpurun_out/r04z_demo_stream.err || { tail -20 gpurun_out/r04z_demo_stream.err; exit 1; }
cat gpurun_out/r04z_demo_stream.json
