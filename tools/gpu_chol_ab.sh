# Cholesky potrf variants on one MI355X: per-level phase timing of CS_TIMING builds (CST_LIBS, names of
# libptzba_NAME.so), GPU tests on the default build, then short benches of the default and BENCH_LIBS.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
for v in $CST_LIBS; do
  echo "== timing $v"
  PTZBA_LIB=$P/libptzba_$v.so timeout -k 10 120 python tools/chol_timing.py > gpurun_out/ct_$v.log 2>&1 || { tail gpurun_out/ct_$v.log; exit 1; }
  sed -n 1,3p gpurun_out/ct_$v.log
done
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ca_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/ca_tests.log; exit 1; }
  tail -1 gpurun_out/ca_tests.log
fi
for v in default $BENCH_LIBS; do
  L=$P/libptzba.so; [ $v = default ] || L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-accuracy > gpurun_out/cb_$v.json 2> gpurun_out/cb_$v.err || { tail gpurun_out/cb_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/cb_$v.json').read().strip().splitlines()[-1]); print('$v it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],3), d['kernel_ms'])"
done
