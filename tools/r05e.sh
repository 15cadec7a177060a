#!/bin/bash
# round 5: default bench line + rocprofv3 kernel stats of a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.err || { tail -20 gpurun_out/r05e_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r05e_bench.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), d['accuracy']['rmse_vs_oracle_optimum']['bench_solve_ftol_1e-4'], d['kernel_ms'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r05e_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05e_prof -o run --output-format csv -- python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/r05e_prof_bench.json 2> gpurun_out/r05e_prof.log || { tail gpurun_out/r05e_prof.log; exit 1; }
head -14 gpurun_out/r05e_prof/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120
echo done
