# Same-box A/B/C of the tree's library and variant libraries ($VARIANTS, pan-tilt-zoom-slam_amd/libptzba_NAME.so)
# on the headline bench: parity tests of each variant's BA path first, then two alternating bench rounds.
set -o pipefail
mkdir -p gpurun_out
for v in $VARIANTS; do
  PTZBA_LIB=$PWD/pan-tilt-zoom-slam_amd/libptzba_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab3_$v.log 2>&1 || { echo "TESTFAIL $v"; tail -20 gpurun_out/ab3_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab3_$v.log)"
done
for r in 1 2; do
  for v in cur $VARIANTS; do
    L=$PWD/pan-tilt-zoom-slam_amd/libptzba.so; [ $v = cur ] || L=$PWD/pan-tilt-zoom-slam_amd/libptzba_$v.so
    PTZBA_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/ab3_$v$r.json 2> gpurun_out/ab3_$v$r.err || { echo ABFAIL; tail gpurun_out/ab3_$v$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab3_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', round(d['value'],1), {k: round(x*1e3,1) for k, x in d['kernel_ms'].items()})"
  done
done
