#!/bin/bash
# round-4 pass D: single-launch factorisation tests + A/B, kernel trace of the config-5 stream
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TESTS="tests/test_gpu_ba.py -k single_launch" REPS=3 AB_ENVS="PTZBA_CHOL_PERSIST=1" bash tools/r04ab.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_config3.py -k "knobs" > gpurun_out/r04d_tests3.log 2>&1 || { tail -30 gpurun_out/r04d_tests3.log; exit 1; }
tail -2 gpurun_out/r04d_tests3.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d_stream_prof -o stream -- python pan-tilt-zoom-slam_amd/demo_stream.py --frames 100 > gpurun_out/r04d_stream.json 2> gpurun_out/r04d_stream.err || { tail -20 gpurun_out/r04d_stream.err; exit 1; }
cat gpurun_out/r04d_stream.json
find gpurun_out/r04d_stream_prof -name "*stats*" | head
