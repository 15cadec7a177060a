set -o pipefail
timeout -k 10 300 python tools/dist_model.py --config config3 --worlds 1,2,4,8 --trials 40 > gpurun_out/r03e_dist_model_c3.jsonl 2> gpurun_out/r03e_dist_model_c3.err || { echo MODELFAIL; tail -20 gpurun_out/r03e_dist_model_c3.err; exit 1; }
cat gpurun_out/r03e_dist_model_c3.jsonl | cut -c1-400
VARIANTS="default nlwait k1atomic" TESTS="tests/test_gpu_ba.py tests/test_gpu_ekf.py" bash tools/gpu_lib_ab.sh
