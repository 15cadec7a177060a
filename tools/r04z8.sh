#!/bin/bash
# SIFT row pass over 4 rows per workgroup: the front-end / stream GPU tests, SIFT wall time and kernel stats, the stream
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_stream.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z8_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z8_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z8_gpu_tests.log
timeout -k 10 300 python tools/sift_bench.py --default > gpurun_out/r04z8_sift_bench.txt 2>&1 || { tail gpurun_out/r04z8_sift_bench.txt; exit 1; }
cat gpurun_out/r04z8_sift_bench.txt
PTZ_SIFT_ROWS4=0 timeout -k 10 300 python tools/sift_bench.py --default > gpurun_out/r04z8_sift_bench_rows1.txt 2>&1 || { tail gpurun_out/r04z8_sift_bench_rows1.txt; exit 1; }
cat gpurun_out/r04z8_sift_bench_rows1.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z8_prof -o run --output-format csv -- python tools/sift_bench.py --default > gpurun_out/r04z8_prof.log 2>&1 || { tail gpurun_out/r04z8_prof.log; exit 1; }
python -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/r04z8_prof/run_kernel_stats.csv')))
for r in rows: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), round(float(r['TotalDurationNs']) / 23e6, 3), 'ms/call')
"
for k in 1 2; do
  timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py > gpurun_out/r04z8_demo_stream_$k.json 2> gpurun_out/r04z8_demo_stream_$k.err || { tail -20 gpurun_out/r04z8_demo_stream_$k.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r04z8_demo_stream_$k.json')); print(d['fps_end_to_end'], d['tracking_ms'], d['keyframe_ba_ms'])"
done
