#!/bin/bash
# round 5: GPU suite after the knob pruning, SIFT timing, short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r05g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/${T}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; }
timeout -k 10 120 python -u tools/sift_bench.py > gpurun_out/${T}_sift.txt 2>&1 || { tail gpurun_out/${T}_sift.txt; exit 1; }
cat gpurun_out/${T}_sift.txt
timeout -k 10 300 python bench.py --steps 300 --no-cpu-baseline --no-cold > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), d['accuracy']['rmse_vs_oracle_optimum']['bench_solve_ftol_1e-4'], d['kernel_ms'])"
echo done
