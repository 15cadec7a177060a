# Round measurement on one MI355X (run through gpurun): GPU tests, bench line, rocprofv3 kernel
# stats, and HBM traffic of K1 from two separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots").  Every GPU step has its own time limit
# and the script stops at the first failure.
set -o pipefail
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-cold --no-secondary --config4-steps 0 --stream-frames 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_stats -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_prof_stats.log 2>&1 || { echo PROFFAIL; tail gpurun_out/${TAG}_prof_stats.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${TAG}_pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py $BARGS > gpurun_out/${TAG}_pmc_write.log 2>&1 || { echo PMCFAIL; tail gpurun_out/${TAG}_pmc_write.log; exit 1; }
# the bench line's traffic field comes from this run's PMC passes
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "k_linearize<float, 1," config3/pair/fp32/huber gpurun_out/${TAG}_k1_traffic.json 0 1172736 > /dev/null || { echo TRAFFICFAIL; exit 1; }
timeout -k 10 400 python bench.py --traffic-json gpurun_out/${TAG}_k1_traffic.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCHFAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
# PMC byte-count calibration of the access widths K1 uses (1 GiB streams and a cache-resident table)
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_fetch -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_fetch.log 2>&1 || { echo CALFAIL; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_cal_write -o run --output-format csv -- ./tools/pmc_calib.bin > gpurun_out/${TAG}_cal_write.log 2>&1 || { echo CALFAIL; exit 1; }
python tools/pmc_calib_summary.py gpurun_out/${TAG}_cal_fetch gpurun_out/${TAG}_cal_write gpurun_out/${TAG}_pmc_calib.json
# K2 (matrix-core Schur kernel) traffic from the same PMC passes
python tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "k_schur_mf" config3/pair/fp32/huber/k2 gpurun_out/${TAG}_k2_traffic.json 1024 131072 > /dev/null || { echo K2TRAFFICFAIL; exit 1; }
cat gpurun_out/${TAG}_k2_traffic.json
