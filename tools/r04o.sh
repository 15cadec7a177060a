#!/bin/bash
# round-4 pass O: supercolumn plans on the GPU (exactness, config-3 A/B) and the SIFT phase times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nested2.py > gpurun_out/r04o_tests.log 2>&1 || { tail -40 gpurun_out/r04o_tests.log; exit 1; }
tail -1 gpurun_out/r04o_tests.log
PTZ_SIFT_TIMING=1 timeout -k 10 300 python tools/sift_bench.py > gpurun_out/r04o_sift.txt 2> gpurun_out/r04o_sift_timing.txt || { tail -20 gpurun_out/r04o_sift_timing.txt; exit 1; }
cat gpurun_out/r04o_sift.txt
tail -7 gpurun_out/r04o_sift_timing.txt
REPS=2 STEPS=200 AB_ENVS="PTZBA_CHOL_SUPER=1 PTZBA_CHOL_SUPER=1,PTZBA_ND_DEPTH=1" bash tools/r04ab.sh || exit 1
