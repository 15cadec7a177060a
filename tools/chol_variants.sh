# Cholesky ablation: CHOL_VARIANT 1 = no fused potrf+TRSM, 3 = no trailing update, 4 = no panel GEMMs, 5 = empty kernel (timing only).
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 3 4 5; do
  if [ $v = 0 ]; then L=pan-tilt-zoom-slam_amd/libptzba.so; else L=pan-tilt-zoom-slam_amd/libptzba_c$v.so; fi
  PTZBA_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-accuracy > gpurun_out/cv$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/cv$v.json')); print('variant $v', d['kernel_ms'])"
done
