#!/bin/bash
# round 5: the GN start + huber curvature switch -- GPU suite, then the defaults study
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/r05d_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05d_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r05d_gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/ftol_study.py defaults > gpurun_out/r05d_defaults.jsonl 2> gpurun_out/r05d_defaults.err || { tail gpurun_out/r05d_defaults.err; exit 1; }
echo done
