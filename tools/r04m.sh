#!/bin/bash
# round-4 pass M: supercolumn factorisation (PTZBA_CHOL_SUPER=1, chol_super): exactness on the GPU (two-level and
# one-level orders, continuation records), then the config-3 A/B against the default plan
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nested2.py > gpurun_out/r04m_tests.log 2>&1 || { tail -40 gpurun_out/r04m_tests.log; exit 1; }
tail -1 gpurun_out/r04m_tests.log
REPS=2 STEPS=200 AB_ENVS="PTZBA_CHOL_SUPER=1 PTZBA_CHOL_SUPER=1,PTZBA_ND_DEPTH=1" bash tools/r04ab.sh || exit 1
