#!/bin/bash
# round 5: the XCD-local factorisation tail (k_chol_xcd) -- bitwise tests against one launch per level, then bench A/B
# (PTZBA_CHOL_XCD=0 vs the default) and a kernel-trace summary of the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05x1}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  "tests/test_gpu_config3.py::test_config3_schedule_knobs_bitwise_equal" \
  "tests/test_gpu_ba.py::test_single_launch_schedules_bitwise_equal" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
for rep in 1 2; do
for v in 0 auto ${EXTRA}; do
  if [ $v = auto ]; then unset PTZBA_CHOL_XCD; else export PTZBA_CHOL_XCD=$v; fi
  timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-accuracy --no-secondary --stream-frames 0 > gpurun_out/${T}_$v$rep.json 2> gpurun_out/${T}_$v$rep.err || { tail gpurun_out/${T}_$v$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${T}_$v$rep.json').read().strip().splitlines()[-1]); print('xcd=$v', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d.get('kernel_ms', {}).items()} if isinstance(d.get('kernel_ms'), dict) else '')"
done
done
unset PTZBA_CHOL_XCD
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-cold --no-secondary --stream-frames 0 > gpurun_out/${T}_prof.log 2>&1 || { echo PROFFAIL; tail gpurun_out/${T}_prof.log; exit 1; }
f=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1)
head -14 "$f" | cut -d, -f1-6
