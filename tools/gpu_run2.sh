set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_camera.py tests/test_gpu_ba.py -x -q -m gpu -k "not config2 and not dedup" > gpurun_out/t5.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t5.log; exit 1; }
tail -3 gpurun_out/t5.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo BENCHFAIL; tail gpurun_out/bench5.err; exit 1; }
cat gpurun_out/bench5.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-accuracy > gpurun_out/prof5.log 2>&1 || { echo PROFFAIL; tail gpurun_out/prof5.log; exit 1; }
find gpurun_out/prof5 -name "*stats*" | head
