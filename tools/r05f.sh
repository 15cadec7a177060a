#!/bin/bash
# round 5: GPU suite, defaults study, default bench line, rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-r05f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > gpurun_out/${T}_gpu_tests.log 2>&1; rc=$?
tail -1 gpurun_out/${T}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/${T}_gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/ftol_study.py defaults > gpurun_out/${T}_defaults.jsonl 2> gpurun_out/${T}_defaults.err || { tail gpurun_out/${T}_defaults.err; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), d['accuracy']['rmse_vs_oracle_optimum']['bench_solve_ftol_1e-4'], d['kernel_ms'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/${T}_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof.log || { tail gpurun_out/${T}_prof.log; exit 1; }
head -14 gpurun_out/${T}_prof/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
echo done
