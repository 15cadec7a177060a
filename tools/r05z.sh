#!/bin/bash
# round 5: kernel trace of a short config-3 bench (rocprofv3 --kernel-trace): per-kernel durations and the gaps between
# consecutive kernels of one LM iteration (tools/trace_gaps.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05z_trace -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold --stream-frames 0 > gpurun_out/r05z_bench.log 2>&1 || { tail gpurun_out/r05z_bench.log; exit 1; }
find gpurun_out/r05z_trace -name "*kernel_trace.csv" | head -3
