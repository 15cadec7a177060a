# Schur timing ablation (libptzba_s1 = no LDS atomics, libptzba_s2 = no partner loads); timings only.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2; do
  if [ $v = 0 ]; then L=pan-tilt-zoom-slam_amd/libptzba.so; else L=pan-tilt-zoom-slam_amd/libptzba_s$v.so; fi
  PTZBA_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-accuracy > gpurun_out/sa$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sa$v.json')); print('variant $v', d['kernel_ms'])"
done
