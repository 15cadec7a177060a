# BASELINE configs 4 and 5 on this round's tree: config-4 bench line (N = 1), the config-5 stream demo, and a
# 2-rank part-owned config-4 rehearsal over gloo on one device.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/r03l_bench_config4.json 2> gpurun_out/r03l_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/r03l_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r03l_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
timeout -k 10 600 python pan-tilt-zoom-slam_amd/demo_stream.py --frames 300 > gpurun_out/r03l_demo_stream.json 2> gpurun_out/r03l_demo_stream.err || { echo DEMOFAIL; tail -20 gpurun_out/r03l_demo_stream.err; exit 1; }
tail -c 1500 gpurun_out/r03l_demo_stream.json
