# K1 thread-coarsening A/B (K1_COARSE was 0 by default then) on one MI355X: GPU tests on libptzba_c1.so (tools/build_variant.sh c1
# ba_kernels.hip -DK1_COARSE=1), then benches of the default build and c1.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
PTZBA_LIB=$P/libptzba_c1.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/kc_tests.log 2>&1 || { tail -30 gpurun_out/kc_tests.log; exit 1; }
tail -1 gpurun_out/kc_tests.log
for v in default c1; do
  L=$P/libptzba.so; [ $v = default ] || L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/kc_$v.json 2> gpurun_out/kc_$v.err || { tail gpurun_out/kc_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/kc_$v.json').read().strip().splitlines()[-1]); print('$v it/s', round(d['value'],1), 'k1 ms', round(d['roofline']['k1_avg_ms'],4), 'frac', round(d['roofline']['frac'],3), d['accuracy']['rmse_fp32_vs_fp64'], d['accuracy']['iters_fp32'])"
done
