#!/bin/bash
# round-4 final measurement pass: rocprofv3 stats, PMC traffic of K1 / K2, the bench line with this run's traffic,
# PMC calibration, smoke, config-4 bench (tools/r04b.sh with TAG=r04s), then the config-5 stream with the
# set_problem phase timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r04s bash tools/r04b.sh || exit 1
cd "$GRAFT_REPO_ROOT" || exit 1
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04s_demo_stream.json 2> gpurun_out/r04s_demo_stream.err || { tail -20 gpurun_out/r04s_demo_stream.err; exit 1; }
cat gpurun_out/r04s_demo_stream.json
