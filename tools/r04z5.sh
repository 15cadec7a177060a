#!/bin/bash
# K2 reduce with its index loads in one round trip and 8 splits in flight: the K2 / Cholesky / config-3 GPU tests,
# rocprofv3 stats of a short bench, the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_config3.py tests/test_gpu_nested2.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04z5_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04z5_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04z5_gpu_tests.log
BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-cold --no-secondary"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z5_prof_stats -o run --output-format csv -- python bench.py $BARGS > gpurun_out/r04z5_prof_stats.log 2>&1 || { echo PROFFAIL; tail gpurun_out/r04z5_prof_stats.log; exit 1; }
find gpurun_out/r04z5_prof_stats -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    if 'schur' in r['Name'] or 'linearize' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
timeout -k 10 600 python bench.py > gpurun_out/r04z5_bench.json 2> gpurun_out/r04z5_bench.err || { tail gpurun_out/r04z5_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04z5_bench.json').read().strip().splitlines()[-1]); print(round(d['value'],1), d['ms_per_step'], d['kernel_ms'], round(d['roofline']['frac'],3))"
