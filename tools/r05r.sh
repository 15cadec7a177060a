#!/bin/bash
# round 5: K1 ablations (timing-only builds, wrong results): 1 no frame-table staging, 2 no phase-A projection,
# 3 no record stream (phase B), 4 no phase C -- each timed alone by tools/k1_time.py against the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in default abl1 abl2 abl3 abl4 default; do
  L=pan-tilt-zoom-slam_amd/libptzba.so; [ $v != default ] && L=pan-tilt-zoom-slam_amd/libptzba_$v.so
  PTZBA_LIB=$PWD/$L timeout -k 10 120 python tools/k1_time.py $v 200 || exit 1
done
