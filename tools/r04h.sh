#!/bin/bash
# round-4 pass H: full GPU suite, config-4 bench with the set_problem phase timing, config-5 stream (fused SIFT blur)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r04h_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04h_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04h_gpu_tests.log
PTZBA_SETUP_TIMING=1 timeout -k 10 600 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-cold > gpurun_out/r04h_bench_config4.json 2> gpurun_out/r04h_bench_config4.err || { tail -20 gpurun_out/r04h_bench_config4.err; exit 1; }
grep "set_problem" gpurun_out/r04h_bench_config4.err | head -10
timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04h_demo_stream.json 2> gpurun_out/r04h_demo_stream.err || exit 1
cat gpurun_out/r04h_demo_stream.json
