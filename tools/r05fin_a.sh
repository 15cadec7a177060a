#!/bin/bash
# round-5 final pass, part A (one MI355X): the whole GPU test suite and smoke() on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05fin}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 \
  || { echo TESTFAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 \
  || { echo SMOKEFAIL; tail gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
