#!/bin/bash
# round-4 pass P: keyframe-path host changes and supercolumn plans under the GPU tests, the config-5 stream, the SIFT
# phase times, then the config-3 A/B: supercolumns (two- and one-level orders), K2 item counts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_gpu_stream.py tests/test_gpu_maps.py tests/test_gpu_ba.py tests/test_gpu_nested2.py > gpurun_out/r04p_tests.log 2>&1 || { tail -40 gpurun_out/r04p_tests.log; exit 1; }
tail -1 gpurun_out/r04p_tests.log
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04p_demo_stream.json 2> gpurun_out/r04p_demo_stream.err || { tail -20 gpurun_out/r04p_demo_stream.err; exit 1; }
cat gpurun_out/r04p_demo_stream.json
PTZ_SIFT_TIMING=1 timeout -k 10 300 python tools/sift_bench.py > gpurun_out/r04p_sift.txt 2> gpurun_out/r04p_sift_timing.txt || { tail -20 gpurun_out/r04p_sift_timing.txt; exit 1; }
cat gpurun_out/r04p_sift.txt
tail -7 gpurun_out/r04p_sift_timing.txt
REPS=1 STEPS=200 AB_ENVS="PTZBA_CHOL_SUPER=1 PTZBA_CHOL_SUPER=1,PTZBA_ND_DEPTH=1 PTZBA_S2_ITEMS=192 PTZBA_S2_ITEMS=256 PTZBA_S2_ITEMS=320" bash tools/r04ab.sh || exit 1
