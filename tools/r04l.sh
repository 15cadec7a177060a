#!/bin/bash
# round-4 pass L: where a 1080p GPU SIFT detection spends its ~2.2 ms -- host phase times (PTZ_SIFT_TIMING) and the
# rocprofv3 kernel summary of the same benchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
PTZ_SIFT_TIMING=1 timeout -k 10 300 python tools/sift_bench.py > gpurun_out/r04l_sift.txt 2> gpurun_out/r04l_sift_timing.txt || { tail -20 gpurun_out/r04l_sift_timing.txt; exit 1; }
cat gpurun_out/r04l_sift.txt
tail -8 gpurun_out/r04l_sift_timing.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04l_prof -o sift -- python tools/sift_bench.py > gpurun_out/r04l_prof.log 2>&1 || { tail -20 gpurun_out/r04l_prof.log; exit 1; }
find gpurun_out/r04l_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04l_sift_kernel_stats.csv
head -25 gpurun_out/r04l_sift_kernel_stats.csv | cut -c1-160
