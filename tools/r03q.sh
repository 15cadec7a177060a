# Delayed trailing updates (DT = 2, config 4's default): grid exactness (forced), factorisation / EKF tests,
# config-4 LM test, then config-4 per-trial groups DT = 2 vs DT = 1 (PTZBA_CHOL_DELAY=1) alternating, and the
# config-4 bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ba.py tests/test_gpu_ekf.py \
  "tests/test_gpu_config4.py::test_grid_gauss_newton_step_is_exact" "tests/test_gpu_config4.py::test_grid_delayed_trailing_updates_exact" \
  > gpurun_out/r03q_tests.txt 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03q_tests.txt; exit 1; }
tail -1 gpurun_out/r03q_tests.txt
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_config4.py -k "lm_three" \
  > gpurun_out/r03q_tests_c4.txt 2>&1 || { echo C4TFAIL; tail -30 gpurun_out/r03q_tests_c4.txt; exit 1; }
grep -E "kernel ms|passed|failed" gpurun_out/r03q_tests_c4.txt | tail -2 | cut -c1-400
for v in 2 1 2 1; do
  PTZBA_CHOL_DELAY=$v timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03q_c4_dt$v.jsonl 2> gpurun_out/r03q_c4_dt$v.err || { echo FAIL $v; tail gpurun_out/r03q_c4_dt$v.err; exit 1; }
  echo c4 DT=$v; cut -c1-210 gpurun_out/r03q_c4_dt$v.jsonl
done
timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/r03q_bench_config4.json 2> gpurun_out/r03q_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/r03q_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03q_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
