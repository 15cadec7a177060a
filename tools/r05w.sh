#!/bin/bash
# round 5: set_problem's device front -- BA / config-3 / config-4 / distributed GPU tests, then set_problem timing at
# configs 3 and 4 (tools/setup_time.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05w}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_ba.py \
  tests/test_gpu_config3.py tests/test_gpu_config4.py tests/test_gpu_stream.py > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python tools/setup_time.py config3 2 > gpurun_out/${T}_setup_c3.jsonl || exit 1
timeout -k 10 400 python tools/setup_time.py config4 2 > gpurun_out/${T}_setup_c4.jsonl || exit 1
cat gpurun_out/${T}_setup_c3.jsonl gpurun_out/${T}_setup_c4.jsonl
