#!/bin/bash
# round-4 pass J: single-launch factorisation variants (polling pressure, levels per launch) and K2 work-item targets
# against the defaults; the fused-prepare bitwise test
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ba.py -k "fused_prepare" > gpurun_out/r04j_tests.log 2>&1 || { tail -30 gpurun_out/r04j_tests.log; exit 1; }
tail -1 gpurun_out/r04j_tests.log
REPS=2 STEPS=200 AB_ENVS="PTZBA_CHOL_PERSIST=2,PTZBA_CHOL_SPIN_SLEEP=8 PTZBA_CHOL_PERSIST=2,PTZBA_CHOL_GROUP=2 PTZBA_CHOL_PERSIST=2,PTZBA_CHOL_GROUP=2,PTZBA_CHOL_SPIN_SLEEP=4 PTZBA_S2_ITEMS=256 PTZBA_S2_ITEMS=384 PTZBA_S2_ITEMS=768" bash tools/r04ab.sh || exit 1
