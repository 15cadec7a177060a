# LDS aliasing of the Cholesky sweep buffer (3 workgroups per CU): factorisation tests (BA small configs, grid,
# EKF signed factor), then config-4 per-trial groups and the config-3 bench, tree library vs the
# CHOL_LB_ALIAS=0 variant (libptzba_lbown.so), alternating.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P=$PWD/pan-tilt-zoom-slam_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ekf.py \
  "tests/test_gpu_config4.py::test_grid_gauss_newton_step_is_exact" > gpurun_out/r03o_tests.txt 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03o_tests.txt; exit 1; }
tail -1 gpurun_out/r03o_tests.txt
for v in default lbown default lbown; do
  L=$P/libptzba.so; [ $v != default ] && L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03o_c4_$v.jsonl 2> gpurun_out/r03o_c4_$v.err || { echo FAIL $v; tail gpurun_out/r03o_c4_$v.err; exit 1; }
  echo c4 $v; cut -c1-210 gpurun_out/r03o_c4_$v.jsonl
done
for v in default lbown default lbown; do
  L=$P/libptzba.so; [ $v != default ] && L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-secondary --no-cold --no-accuracy > gpurun_out/r03o_c3_$v.json 2> gpurun_out/r03o_c3_$v.err || { echo BFAIL $v; tail gpurun_out/r03o_c3_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r03o_c3_$v.json').read().strip().splitlines()[-1]); print('c3 $v it/s', round(d['value'],1), {k: round(x,4) for k,x in d['kernel_ms'].items()})"
done
