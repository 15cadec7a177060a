# K1 knob sweep on one MI355X: bench.py with the default build and the libptzba_{w3,w5,u2,u4}.so variants
# (tools/build_variant.sh NAME ba_kernels.hip "-DK1_MIN_WAVES=N" / "-DK1_UNROLL=N"); prints it/s and the K1 average.
set -o pipefail
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
for v in default w3 w5 u2 u4 default; do
  L=$P/libptzba.so; [ $v = default ] || L=$P/libptzba_$v.so
  PTZBA_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-accuracy > gpurun_out/ks_$v.json 2> gpurun_out/ks_$v.err || { tail gpurun_out/ks_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ks_$v.json').read().strip().splitlines()[-1]); print('$v it/s', round(d['value'],1), 'k1 ms', round(d['roofline']['k1_avg_ms'],4), 'frac', round(d['roofline']['frac'],3))"
done
