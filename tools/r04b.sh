# Round-4 measurement pass on one MI355X: rocprofv3 kernel stats, the two PMC passes of K1 / K2 traffic, the bench
# line with this run's traffic, PMC byte calibration, smoke(), config-4 bench (with the set_problem phase timing),
# config-5 stream.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${TAG:-r04b}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-cold --no-secondary"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_stats -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_prof_stats.log 2>&1 || { echo PROFFAIL; tail gpurun_out/${TAG}_prof_stats.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_pmc_write.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${TAG}_pmc_write.log; exit 1; }
K1NAME="k_linearize<float, 1"  # (substring: the FTL instantiation <float, 1, true> at config 3)
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "$K1NAME" config3/pair/fp32/huber gpurun_out/${TAG}_k1_traffic.json > /dev/null || { echo TRAFFICFAIL; exit 1; }
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "k_schur_mf" config3/pair/fp32/huber/k2 gpurun_out/${TAG}_k2_traffic.json 1024 > /dev/null || { echo K2TRAFFICFAIL; exit 1; }
timeout -k 10 900 python bench.py --traffic-json gpurun_out/${TAG}_k1_traffic.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCHFAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 3000 gpurun_out/${TAG}_bench.json
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_fetch -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_fetch.log 2>&1 || { echo CALFAIL; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_write -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_write.log 2>&1 || { echo CALFAIL; exit 1; }
python tools/pmc_calib_summary.py gpurun_out/${TAG}_cal_fetch gpurun_out/${TAG}_cal_write gpurun_out/${TAG}_pmc_calib.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKEFAIL; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
PTZBA_SETUP_TIMING=1 timeout -k 10 900 python bench.py --config config4 --steps 8 --warmup 2 --no-cpu-baseline --no-accuracy --no-cold > gpurun_out/${TAG}_bench_config4.json 2> gpurun_out/${TAG}_bench_config4.err || { echo C4FAIL; tail -20 gpurun_out/${TAG}_bench_config4.err; exit 1; }
grep "set_problem" gpurun_out/${TAG}_bench_config4.err | head -20
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), 'it/s', d['kernel_ms'], round(d['roofline']['frac'],3), d.get('dropin_call'))"
