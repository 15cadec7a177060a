# K2 A/B on one MI355X: fp32 GPU parity tests with the default (MFMA) Schur kernel, then the bench with
# PTZBA_SCHUR=valu and the default alternately; prints it/s and the Schur kernel time of each.
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_ba.py tests/test_gpu_config3.py}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/sab_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/sab_tests.log; exit 1; }
tail -1 gpurun_out/sab_tests.log
for v in valu mfma valu mfma; do
  PTZBA_SCHUR=$v timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-secondary --no-cold > gpurun_out/sab_$v.json 2> gpurun_out/sab_$v.err || { echo BENCHFAIL $v; tail gpurun_out/sab_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sab_$v.json').read().strip().splitlines()[-1]); print('$v it/s', round(d['value'],1), 'kernel_ms', {k: round(x,4) for k,x in d['kernel_ms'].items()}, 'acc', d.get('accuracy',{}).get('rmse_fp32_vs_fp64'))"
done
