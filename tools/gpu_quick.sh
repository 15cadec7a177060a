# Iteration loop on one MI355X: GPU tests, then a short profiled bench; prints the top kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/q_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy > gpurun_out/q_bench.json 2> gpurun_out/q_prof.log || { echo PROFFAIL; tail gpurun_out/q_prof.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/q_bench.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],3))"
head -9 gpurun_out/q_prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
if [ -n "$AB_LIB" ]; then
  PTZBA_LIB=$AB_LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_prof_ab -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy > gpurun_out/q_bench_ab.json 2> gpurun_out/q_prof_ab.log || { echo ABFAIL; tail gpurun_out/q_prof_ab.log; exit 1; }
  echo "A/B variant $AB_LIB"; python -c "import json; d=json.loads(open('gpurun_out/q_bench_ab.json').read().strip().splitlines()[-1]); print('it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],3))"
  head -9 gpurun_out/q_prof_ab/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-110
fi
