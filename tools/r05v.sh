#!/bin/bash
# round 5: K1 waves-per-block A/B (bench only), then the distributed GPU tests (incl. config 4 at world 8: ranks over gloo, one device)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V="default wpb8 wpb16" NOTESTS=1 TAG=r05u bash tools/r05p.sh || exit 1
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py \
  > gpurun_out/r05v_c4w8.log 2>&1; rc=$?; tail -3 gpurun_out/r05v_c4w8.log; exit $rc
