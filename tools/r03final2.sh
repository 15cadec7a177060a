# Round-3 final pass, second half (the first stopped at the PMC calibration: its binary had not been rebuilt):
# PMC byte calibration, smoke(), the config-4 bench line
set -o pipefail
export TAG=${TAG:-r03z}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_fetch -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_fetch.log 2>&1 || { echo CALFAIL; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_write -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_write.log 2>&1 || { echo CALFAIL; exit 1; }
python tools/pmc_calib_summary.py gpurun_out/${TAG}_cal_fetch gpurun_out/${TAG}_cal_write gpurun_out/${TAG}_pmc_calib.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKEFAIL; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${TAG}_bench_config4.json 2> gpurun_out/${TAG}_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/${TAG}_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3))"
