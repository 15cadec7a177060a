#!/bin/bash
# round 5: A/B of the product build (default) against variant libraries (V="default orig ...": libptzba_<v>.so):
# bench it/s + K1 HIP events, then (NOTESTS unset) the GPU BA tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05l}
for rep in 1 2; do
for v in ${V:-default orig}; do
  L=pan-tilt-zoom-slam_amd/libptzba.so; [ $v != default ] && L=pan-tilt-zoom-slam_amd/libptzba_$v.so
  PTZBA_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-accuracy --no-secondary --stream-frames 0 > gpurun_out/${T}_$v$rep.json 2> gpurun_out/${T}_$v$rep.err || { tail gpurun_out/${T}_$v$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${T}_$v$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), 'K1 ms', round(r['k1_avg_ms'],5), 'frac', round(r['frac'],4), 'cold', round(r['cold_cache']['frac'],4))"
done
done
[ -n "$NOTESTS" ] && exit 0
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ba.py tests/test_gpu_config3.py tests/test_gpu_stream.py tests/test_gpu_nested2.py tests/test_gpu_distributed.py > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_tests.log; exit $rc
