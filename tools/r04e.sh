#!/bin/bash
# round-4 pass E: config-3 schedule knobs (bitwise), coherent-traffic A/B, kernel trace of the config-5 stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_config3.py -k "knobs" tests/test_gpu_ba.py -k "knobs or single_launch" > gpurun_out/r04e_tests.log 2>&1 || { tail -30 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
REPS=2 AB_ENVS="PTZBA_CHOL_COH=1" bash tools/r04ab.sh || exit 1
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04e_demo_stream.json 2> gpurun_out/r04e_setup_timing.txt || exit 1
cat gpurun_out/r04e_demo_stream.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04e_stream_prof -o stream -- python pan-tilt-zoom-slam_amd/demo_stream.py --frames 100 > gpurun_out/r04e_stream.json 2> gpurun_out/r04e_stream.err || { tail -20 gpurun_out/r04e_stream.err; exit 1; }
find gpurun_out/r04e_stream_prof -name "*stats*" | head
