#!/bin/bash
# round-5 final pass, part B (one MI355X): rocprofv3 kernel stats, K1 / K2 HBM traffic from separate FETCH_SIZE /
# WRITE_SIZE passes (MI355X_MICROARCH.md), the PMC width calibration, then the default bench line with that traffic
# and the config-4 bench (drop-in set_problem timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05fin}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-cold --no-secondary --stream-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_stats -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${T}_prof_stats.log 2>&1 || { echo PROFFAIL; tail gpurun_out/${T}_prof_stats.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${T}_pmc_fetch -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${T}_pmc_fetch.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${T}_pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${T}_pmc_write -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${T}_pmc_write.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${T}_pmc_write.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write "k_linearize<float, 1, true>" config3/pair/fp32/huber gpurun_out/${T}_k1_traffic.json > /dev/null || { echo TRAFFICFAIL; exit 1; }
python tools/pmc_traffic.py gpurun_out/${T}_pmc_fetch gpurun_out/${T}_pmc_write "k_schur_mf" config3/pair/fp32/huber/k2 gpurun_out/${T}_k2_traffic.json 1024 > /dev/null || { echo K2TRAFFICFAIL; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${T}_cal_fetch -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${T}_cal_fetch.log 2>&1 || { echo CALFAIL; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${T}_cal_write -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${T}_cal_write.log 2>&1 || { echo CALFAIL; exit 1; }
python tools/pmc_calib_summary.py gpurun_out/${T}_cal_fetch gpurun_out/${T}_cal_write gpurun_out/${T}_pmc_calib.json || { echo CALSUMFAIL; exit 1; }
timeout -k 10 500 python bench.py --traffic-json gpurun_out/${T}_k1_traffic.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCHFAIL; tail gpurun_out/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), 'K1', round(r['k1_avg_ms']*1e3,2), 'frac', round(r['frac'],4), 'traffic', r['traffic'], 'cold', round(r['cold_cache']['frac'],4))"
timeout -k 10 500 python bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-accuracy --no-cold --stream-frames 0 > gpurun_out/${T}_bench_config4.json 2> gpurun_out/${T}_bench_config4.err || { echo C4BENCHFAIL; tail gpurun_out/${T}_bench_config4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${T}_bench_config4.json').read().strip().splitlines()[-1]); print('config4', round(d['value'],2), d.get('dropin_call'))"
