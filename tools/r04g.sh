#!/bin/bash
# round-4 pass G: coherent / single-launch A/B, stream setup timing, per-rank device times at configs 3 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
REPS=2 AB_ENVS="PTZBA_CHOL_COH=0 PTZBA_CHOL_PERSIST=2" bash tools/r04ab.sh || exit 1
PTZBA_SETUP_TIMING=1 timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04g_demo_stream.json 2> gpurun_out/r04g_setup_timing.txt || exit 1
cat gpurun_out/r04g_demo_stream.json
timeout -k 10 400 python tools/dist_model.py --config config3 --worlds 1,2,3,4,8 > gpurun_out/r04g_dist_model_c3.jsonl || exit 1
timeout -k 10 600 python tools/dist_model.py --config config4 --worlds 1,2,4,8 --trials 10 > gpurun_out/r04g_dist_model_c4.jsonl || exit 1
python tools/dist_predict.py gpurun_out/r04g_dist_model_c3.jsonl gpurun_out/r04g_dist_model_c4.jsonl
