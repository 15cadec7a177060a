# Config-4 trailing-task anatomy (timing-only CHOL_VARIANT builds): 3 = trailing tasks return at once,
# 6 = no panel-tile reads, 7 = no C tile read/write; then the config-3 A/B of the blocked back-solve.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
for v in default cv3 cv6 cv7; do
  L=$P/libptzba.so; [ $v != default ] && L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03p_c4_$v.jsonl 2> gpurun_out/r03p_c4_$v.err || { echo FAIL $v; tail gpurun_out/r03p_c4_$v.err; exit 1; }
  echo c4 $v; cut -c1-210 gpurun_out/r03p_c4_$v.jsonl
done
VARIANTS="default ENV_PTZBA_BACKSOLVE=blk" bash tools/gpu_lib_ab.sh
