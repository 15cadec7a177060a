# Round-3 GPU pass on one MI355X (run through gpurun): GPU tests, smoke(), one bench line.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCHFAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.json
fi
