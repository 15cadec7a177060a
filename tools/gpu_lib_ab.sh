# Library A/B on one MI355X: optional GPU parity tests (TESTS=...), then the config-3 bench for each
# variant in VARIANTS (default = the tree's libptzba.so, NAME = libptzba_NAME.so, ENV_X=Y = the tree's
# library with that environment variable set), twice, alternating.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/lab_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/lab_tests.log; exit 1; }
  tail -1 gpurun_out/lab_tests.log
fi
for rep in 1 2; do
  for v in $VARIANTS; do
    L=$P/libptzba.so; E=""
    case $v in default) ;; ENV_*) E=${v#ENV_} ;; *) L=$P/libptzba_$v.so ;; esac
    env $E PTZBA_LIB=$L timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-secondary --no-cold $BENCH_ARGS > gpurun_out/lab_$v.json 2> gpurun_out/lab_$v.err || { echo BENCHFAIL $v; tail gpurun_out/lab_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/lab_$v.json').read().strip().splitlines()[-1]); print('$v it/s', round(d['value'],1), {k: round(x,4) for k,x in d['kernel_ms'].items()}, d.get('accuracy',{}).get('rmse_fp32_vs_fp64'))"
  done
done
