#!/bin/bash
# GPU SIFT on a rendered 1080p frame: wall time per call, then rocprofv3 kernel stats of the default variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/sift_bench.py --default > gpurun_out/r04z7_sift_bench.txt 2>&1 || { tail gpurun_out/r04z7_sift_bench.txt; exit 1; }
cat gpurun_out/r04z7_sift_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z7_prof -o run --output-format csv -- python tools/sift_bench.py --default > gpurun_out/r04z7_prof.log 2>&1 || { tail gpurun_out/r04z7_prof.log; exit 1; }
python -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/r04z7_prof/run_kernel_stats.csv')))
for r in rows: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), round(float(r['TotalDurationNs']) / 23e6, 3), 'ms/call')
"
