# Round-3 final measurement pass: tools/gpu_measure.sh (all GPU tests, rocprofv3 stats,
# PMC passes, bench line with the full CPU baseline, PMC calibration, K2 traffic), then smoke() and the
# config-4 bench line.
set -o pipefail
export TAG=${TAG:-r03end}
bash tools/gpu_measure.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKEFAIL; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${TAG}_bench_config4.json 2> gpurun_out/${TAG}_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/${TAG}_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
