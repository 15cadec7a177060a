#!/bin/bash
# round 5: the whole GPU suite on the current build (one pytest process), log under gpurun_out/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05t}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/${T}_gpu_tests.log; exit $rc
