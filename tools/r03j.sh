set -o pipefail
for n in 64 128 256; do
  PTZBA_S2_ITEMS=$n timeout -k 10 300 python tools/dist_model.py --config config3 --worlds 2,8 --trials 30 > gpurun_out/r03j_items$n.jsonl 2> gpurun_out/r03j_items$n.err || { echo MODELFAIL; tail -20 gpurun_out/r03j_items$n.err; exit 1; }
  echo "S2_ITEMS=$n"; python -c "
import json
for l in open('gpurun_out/r03j_items$n.jsonl'):
    d=json.loads(l); print(d['world'], d['rank'], round(d['wall_ms_per_trial'],4), d['kernel_ms'], d['solver']['schur_items'])"
done
timeout -k 10 900 python tools/dist_model.py --config config4 --worlds 1,2,8 --trials 6 > gpurun_out/r03i_dist_model_c4.jsonl 2> gpurun_out/r03i_dist_model_c4.err || { echo MODELFAIL4; tail -20 gpurun_out/r03i_dist_model_c4.err; exit 1; }
cut -c1-420 gpurun_out/r03i_dist_model_c4.jsonl
