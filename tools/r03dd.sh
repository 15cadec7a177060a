# Round-3: part-owned solve with the two-level order inside each half: multi-rank GPU parity, then the per-rank
# device-time model at config 3 (N = 1, 2, 4, 8) and config 4 (N = 2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r03dd_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03dd_tests.log; exit 1; }
tail -1 gpurun_out/r03dd_tests.log
timeout -k 10 400 python tools/dist_model.py --config config3 --worlds 1,2,4,8 --trials 40 > gpurun_out/r03dd_dist_model_c3.jsonl 2> gpurun_out/r03dd_dist_model_c3.err || { echo MODELFAIL3; tail -20 gpurun_out/r03dd_dist_model_c3.err; exit 1; }
cut -c1-250 gpurun_out/r03dd_dist_model_c3.jsonl
