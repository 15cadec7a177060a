# K1 variant sweep on one box: phase timing (K1_TIMING builds) and 30-iteration benches of each variant
# library (tools/build_variant.sh NAME ba_kernels.hip "<defines>" and tNAME with -DK1_TIMING)
set -o pipefail
mkdir -p gpurun_out
for v in $K1_VARIANTS; do
  PTZBA_LIB=$PWD/pan-tilt-zoom-slam_amd/libptzba_t$v.so timeout -k 10 200 python tools/k1_timing.py > gpurun_out/t$v.txt 2>&1 || { tail gpurun_out/t$v.txt; exit 1; }
  echo "== $v"; sed -n 2,6p gpurun_out/t$v.txt
done
for r in 1 2; do
  for v in $K1_VARIANTS; do
    PTZBA_LIB=$PWD/pan-tilt-zoom-slam_amd/libptzba_$v.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/v_$v$r.json 2> gpurun_out/v_$v$r.err || { tail gpurun_out/v_$v$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/v_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', round(d['value'],1), {k: round(x*1e3,1) for k, x in d['kernel_ms'].items()})"
  done
done
