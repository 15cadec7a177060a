# Round-3 end: per-rank device time of the N-way part-owned solve on one MI355X (tools/dist_model.py), configs 3 and 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/dist_model.py --config config3 --worlds 1,2,4,8 --trials 40 > gpurun_out/r03dm_dist_model_c3.jsonl 2> gpurun_out/r03dm_dist_model_c3.err || { echo MODELFAIL3; tail -20 gpurun_out/r03dm_dist_model_c3.err; exit 1; }
cut -c1-300 gpurun_out/r03dm_dist_model_c3.jsonl
timeout -k 10 700 python tools/dist_model.py --config config4 --worlds 1,2,8 --trials 6 > gpurun_out/r03dm_dist_model_c4.jsonl 2> gpurun_out/r03dm_dist_model_c4.err || { echo MODELFAIL4; tail -20 gpurun_out/r03dm_dist_model_c4.err; exit 1; }
cut -c1-300 gpurun_out/r03dm_dist_model_c4.jsonl
