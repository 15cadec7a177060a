# Multi-rank rehearsals on one MI355X (through gpurun): the distributed GPU tests (part-owned solve through
# the library with a gloo hook, the library's own RCCL communicator at one rank), then bench.py --gpus 2 over
# gloo on one device (the driver's N > 1 runs use RCCL across devices).
set -o pipefail
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 600 --timeout-method thread > gpurun_out/${TAG}_dist_tests.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/${TAG}_dist_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_dist_tests.log
if [ -z "$NO_BENCH" ]; then
  PTZBA_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_n2_gloo.json 2> gpurun_out/${TAG}_bench_n2_gloo.err || { echo BENCHFAIL; tail -30 gpurun_out/${TAG}_bench_n2_gloo.err; exit 1; }
  tail -1 gpurun_out/${TAG}_bench_n2_gloo.json | cut -c1-1500
fi
