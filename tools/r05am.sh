#!/bin/bash
# round 5: per-rank device times of the rank-tree solve on the current kernels (tools/dist_model.py, configs 3 and 4),
# then the collectives model (dist_predict) and the split-separator model (dist_split_model)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python tools/dist_model.py --config config3 --worlds 1,2,4,8 > gpurun_out/r05am_dist_model_c3.jsonl || exit 1
timeout -k 10 700 python tools/dist_model.py --config config4 --worlds 1,2,4,8 --trials 10 > gpurun_out/r05am_dist_model_c4.jsonl || exit 1
python tools/dist_predict.py gpurun_out/r05am_dist_model_c3.jsonl gpurun_out/r05am_dist_model_c4.jsonl > gpurun_out/r05am_dist_predict.jsonl || exit 1
cat gpurun_out/r05am_dist_predict.jsonl
