# A/B on one MI355X: GPU tests, then two short profiled benches (default, and with $AB_ENV set,
# e.g. AB_ENVS="PTZBA_LIB=/root/repo/pan-tilt-zoom-slam_amd/libptzba_x.so"); prints it/s and the top kernels of each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/ab_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  rm -rf gpurun_out/ab_prof_$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_prof_$1 -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_EXTRA > gpurun_out/ab_bench_$1.json 2> gpurun_out/ab_prof_$1.log || { echo PROFFAIL $1; tail gpurun_out/ab_prof_$1.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab_bench_$1.json').read().strip().splitlines()[-1]); print('$1 it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],3), 'acc', d.get('accuracy',{}).get('rmse_fp32_vs_fp64'), d.get('accuracy',{}).get('iters_fp32'))"
  python -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/ab_prof_$1/run_kernel_stats.csv')))[:8]: print('  ', r['Name'][:50].ljust(50), r['Calls'].rjust(5), '%9.2f us' % (float(r['AverageNs'])/1e3))"
}
run A
# AB_ENVS: space-separated VAR=value settings, one variant run each (B1, B2, ...)
k=0
for kv in $AB_ENVS; do k=$((k+1)); ( export $kv; echo "variant B$k: $kv"; run B$k ) || exit 1; done
