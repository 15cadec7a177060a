# Blocked right-looking back substitution (large systems): parity on the grid problems (single rank natural /
# nested, forced; part-owned 2 ranks, forced), config-4 3-iteration LM test (now blocked by default), then the
# config-4 bench line and its per-kernel model.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_config4.py -k "grid" \
  > gpurun_out/r03m_tests_grid.txt 2>&1 || { echo GRIDFAIL; tail -30 gpurun_out/r03m_tests_grid.txt; exit 1; }
tail -3 gpurun_out/r03m_tests_grid.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_distributed.py -k "grid" \
  > gpurun_out/r03m_tests_dist_grid.txt 2>&1 || { echo DISTFAIL; tail -30 gpurun_out/r03m_tests_dist_grid.txt; exit 1; }
tail -3 gpurun_out/r03m_tests_dist_grid.txt
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_config4.py -k "lm_three" \
  > gpurun_out/r03m_tests_c4.txt 2>&1 || { echo C4TFAIL; tail -30 gpurun_out/r03m_tests_c4.txt; exit 1; }
grep -E "kernel ms|passed|failed" gpurun_out/r03m_tests_c4.txt | tail -3
timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/r03m_bench_config4.json 2> gpurun_out/r03m_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/r03m_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03m_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
