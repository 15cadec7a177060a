# Same-box A/B of two builds of libptzba on the headline bench (config 3): alternating runs of the
# default library and $ALT (PTZBA_LIB), each a full bench process.  Usage: ALT=path/to/lib.so bash tools/ab_libs.sh
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in cur alt; do
    L=""; [ $v = alt ] && L="$ALT"
    PTZBA_LIB=${L:-$PWD/pan-tilt-zoom-slam_amd/libptzba.so} timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || { echo ABFAIL; tail gpurun_out/ab_$v$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', round(d['value'],1), {k: round(x*1e3,1) for k, x in d['kernel_ms'].items()})"
  done
done
