set -o pipefail
timeout -k 10 900 python tools/dist_model.py --config config4 --worlds 1,2,8 --trials 6 > gpurun_out/r03i_dist_model_c4.jsonl 2> gpurun_out/r03i_dist_model_c4.err || { echo MODELFAIL; tail -20 gpurun_out/r03i_dist_model_c4.err; exit 1; }
cut -c1-420 gpurun_out/r03i_dist_model_c4.jsonl
