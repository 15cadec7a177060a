# Config-4 factorisation anatomy: per-trial kernel groups (tools/dist_model.py, N = 1, fixed damping) for the
# tree's library and for timing-only variants of k_chol_step: CHOL_VARIANT=3 (trailing tasks return at once),
# =1 (no potrf/trsm sweep).  Numerics of the variants are meaningless; only the level durations matter.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
for v in default cv3 cv1; do
  L=$P/libptzba.so; [ $v != default ] && L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 300 python tools/dist_model.py --config config4 --worlds 1 --trials 6 > gpurun_out/r03n_$v.jsonl 2> gpurun_out/r03n_$v.err || { echo FAIL $v; tail gpurun_out/r03n_$v.err; exit 1; }
  echo $v; cat gpurun_out/r03n_$v.jsonl | cut -c1-330
done
