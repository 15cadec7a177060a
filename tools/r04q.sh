#!/bin/bash
# round-4 pass Q: supercolumn plans with one sweep copy per kernel (exactness, config-3 A/B), where the config-5
# keyframe path spends its host time (cProfile of the stream), the SIFT kernels (rocprofv3 stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_nested2.py tests/test_gpu_ba.py -k "supercolumn or lazy or drop" > gpurun_out/r04q_tests.log 2>&1 || { tail -40 gpurun_out/r04q_tests.log; exit 1; }
tail -1 gpurun_out/r04q_tests.log
REPS=2 STEPS=200 AB_ENVS="PTZBA_CHOL_SUPER=1" bash tools/r04ab.sh || exit 1
timeout -k 10 300 python tools/profile_stream.py gpurun_out/r04q_stream_prof.txt > gpurun_out/r04q_stream_prof.json 2> gpurun_out/r04q_stream_prof.err || { tail -20 gpurun_out/r04q_stream_prof.err; exit 1; }
cat gpurun_out/r04q_stream_prof.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04q_sift_prof -o sift --output-format csv -- python tools/sift_bench.py > gpurun_out/r04q_sift_prof.log 2>&1 || { tail -20 gpurun_out/r04q_sift_prof.log; exit 1; }
f=$(find gpurun_out/r04q_sift_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04q_sift_kernel_stats.csv
head -16 gpurun_out/r04q_sift_kernel_stats.csv | cut -c1-150
