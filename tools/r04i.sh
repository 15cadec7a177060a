#!/bin/bash
# round-4 pass I: rank-tree plans with delayed updates / blocks -- distributed GPU tests, per-rank device times at
# config 4 and 3; SIFT fused-blur A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/sift_bench.py > gpurun_out/r04i_sift.txt 2>&1 || { tail gpurun_out/r04i_sift.txt; exit 1; }
cat gpurun_out/r04i_sift.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_distributed.py > gpurun_out/r04i_dist_tests.log 2>&1 || { tail -40 gpurun_out/r04i_dist_tests.log; exit 1; }
tail -1 gpurun_out/r04i_dist_tests.log
timeout -k 10 500 python tools/dist_model.py --config config4 --worlds 1,2,4,8 --trials 10 > gpurun_out/r04i_dist_model_c4.jsonl || exit 1
timeout -k 10 200 python tools/dist_model.py --config config3 --worlds 2,4,8 > gpurun_out/r04i_dist_model_c3.jsonl || exit 1
python tools/dist_predict.py gpurun_out/r04i_dist_model_c3.jsonl gpurun_out/r04i_dist_model_c4.jsonl
