# Round-2 measurement pass on one MI355X (through gpurun): GPU tests, the default bench line, an N=2
# gloo rehearsal of `bench.py --gpus 2`, the fp64 K1 A/B (coarsening / occupancy) and rocprofv3 stats.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${TAG:-r02}
STAGES=${STAGES:-tests,bench,dist,ab64,prof}
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
has() { case ",$STAGES," in *",$1,"*) return 0;; esac; return 1; }
if has grid; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_config4.py -k grid -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_grid.log 2>&1 || { echo GRIDFAIL; tail -40 gpurun_out/${TAG}_grid.log; exit 1; }
  tail -3 gpurun_out/${TAG}_grid.log
fi
if has c4; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_config4.py -k config4 -x -v -s --timeout 800 --timeout-method thread > gpurun_out/${TAG}_c4.log 2>&1 || { echo C4FAIL; tail -40 gpurun_out/${TAG}_c4.log; exit 1; }
  grep -E "config4|set_problem|passed|failed" gpurun_out/${TAG}_c4.log | cut -c1-1500
fi
if has stream; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ekf.py tests/test_gpu_stream.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/${TAG}_stream.log 2>&1 || { echo STREAMFAIL; grep -v "^tracking\|^overlap" gpurun_out/${TAG}_stream.log | tail -60; exit 1; }
  grep -E "passed|failed|rmse" gpurun_out/${TAG}_stream.log
fi
if has demo; then
  timeout -k 10 600 python -u pan-tilt-zoom-slam_amd/demo_stream.py --frames 300 --window 30 --keyframe-every 5 > gpurun_out/${TAG}_demo_stream.json 2> gpurun_out/${TAG}_demo_stream.err || { echo DEMOFAIL; tail -30 gpurun_out/${TAG}_demo_stream.err; exit 1; }
  cat gpurun_out/${TAG}_demo_stream.json
fi
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_gpu_tests.log
fi
if has bench; then
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  tail -c 3000 gpurun_out/${TAG}_bench.json
fi
if has c4bench; then
  timeout -k 10 900 python -u bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${TAG}_c4bench.json 2> gpurun_out/${TAG}_c4bench.err || { echo C4BENCHFAIL; tail -20 gpurun_out/${TAG}_c4bench.err; exit 1; }
  tail -c 3000 gpurun_out/${TAG}_c4bench.json
fi
if has dist; then
  PTZBA_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_dist2.json 2> gpurun_out/${TAG}_dist2.err || { echo DISTFAIL; tail -20 gpurun_out/${TAG}_dist2.err; exit 1; }
  tail -c 1500 gpurun_out/${TAG}_dist2.json
fi
if has ab64; then
  for v in default nc64 w3_64; do
    L=$P/libptzba.so; [ $v = default ] || L=$P/libptzba_$v.so
    PTZBA_LIB=$L timeout -k 10 300 python bench.py --precision fp64 --loss linear --steps 30 --warmup 3 --no-cpu-baseline --no-accuracy --no-secondary > gpurun_out/${TAG}_ab64_$v.json 2> gpurun_out/${TAG}_ab64_$v.err || { echo AB64FAIL; tail gpurun_out/${TAG}_ab64_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/${TAG}_ab64_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v it/s', round(d['value'],1), 'k1 ms', round(r['k1_avg_ms'],4), 'frac', round(r['frac'],3), 'cold', r.get('cold_cache',{}).get('k1_avg_ms'))"
  done
fi
if has c4prof; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4prof -o run --output-format csv -- python bench.py --config config4 --steps 3 --warmup 1 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${TAG}_c4prof.log 2>&1 || { echo C4PROFFAIL; tail gpurun_out/${TAG}_c4prof.log; exit 1; }
  head -14 gpurun_out/${TAG}_c4prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
fi
if has prof; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_stats -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --no-secondary --no-cold > gpurun_out/${TAG}_prof_stats.log 2>&1 || { echo PROFFAIL; tail gpurun_out/${TAG}_prof_stats.log; exit 1; }
  head -14 gpurun_out/${TAG}_prof_stats/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
fi
