# Register-direct trailing tasks (CHOL_TRAIL_DIRECT): factorisation / EKF tests, then config-4 per-trial groups
# and the config-3 bench, tree library vs the LDS-staged variant (libptzba_tstage.so), alternating.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P=$PWD/pan-tilt-zoom-slam_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ekf.py \
  "tests/test_gpu_config4.py::test_grid_gauss_newton_step_is_exact" "tests/test_gpu_config4.py::test_grid_delayed_trailing_updates_exact" \
  > gpurun_out/r03s_tests.txt 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03s_tests.txt; exit 1; }
tail -1 gpurun_out/r03s_tests.txt
for v in default tstage default tstage; do
  L=$P/libptzba.so; [ $v != default ] && L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03s_c4_$v.jsonl 2> gpurun_out/r03s_c4_$v.err || { echo FAIL $v; tail gpurun_out/r03s_c4_$v.err; exit 1; }
  echo c4 $v; cut -c1-210 gpurun_out/r03s_c4_$v.jsonl
done
VARIANTS="default tstage" bash tools/gpu_lib_ab.sh
