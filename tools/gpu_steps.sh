# One parameterised GPU session (run through gpurun); replaces the per-round r0N*.sh scripts.
#   TAG=r06x STEPS="tests ct bench prof ab" AB_LIBS="name1 name2" TESTS="tests/test_gpu_ba.py" bash tools/gpu_steps.sh
# steps (each GPU step under its own time limit; the script stops at the first failure):
#   tests   pytest -m gpu ($TESTS, default: the whole suite)
#   ct      Cholesky sweep accounting of the CS_TIMING variant libptzba_cst.so (tools/chol_timing.py)
#   bench   short bench of the default library (no CPU baseline / accuracy / stream legs)
#   prof    rocprofv3 --kernel-trace --stats of that bench (config $CFG, default config3)
#   ab      short bench of every libptzba_NAME.so in $AB_LIBS against the default, alternating twice
#   dist    world-N gloo rehearsal of bench.py on one device (N in $DIST_N, default "2 8")
#   full    the default bench.py line (what the driver runs)
#   stream  demo_stream.py (config 5) with each argument set of $STREAM_ARGS (';'-separated), 300 frames
set -o pipefail
TAG=${TAG:-r06}
CFG=${CFG:-config3}
mkdir -p gpurun_out
P=$PWD/pan-tilt-zoom-slam_amd
BARGS="--steps ${BSTEPS:-100} --warmup 5 --no-cpu-baseline --no-accuracy --stream-frames 0 --no-cold"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'it/s', round(d['value'],1), 'ms/it', round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['kernel_ms'].items()})" "$1" "$2"; }
for st in $STEPS; do
  case $st in
  tests)
    timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAILED|Error|error" gpurun_out/${TAG}_tests.log | head -20; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
    tail -1 gpurun_out/${TAG}_tests.log ;;
  ct)
    PTZBA_LIB=$P/libptzba_cst.so timeout -k 10 240 python tools/chol_timing.py --json gpurun_out/${TAG}_sweep.json > gpurun_out/${TAG}_ct.log 2>&1 || { echo CTFAIL; tail -20 gpurun_out/${TAG}_ct.log; exit 1; }
    cat gpurun_out/${TAG}_ct.log ;;
  bench)
    timeout -k 10 300 python bench.py --config $CFG $BARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCHFAIL; tail gpurun_out/${TAG}_bench.err; exit 1; }
    summ gpurun_out/${TAG}_bench.json default ;;
  prof)
    cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
    rm -rf gpurun_out/${TAG}_prof
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --stream-frames 0 --no-cold --no-secondary > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { echo PROFFAIL; tail gpurun_out/${TAG}_prof.err; exit 1; }
    head -14 gpurun_out/${TAG}_prof/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150 ;;
  ab)
    for rep in 1 2; do
      for v in default $AB_LIBS; do
        L=$P/libptzba.so; [ $v = default ] || L=$P/libptzba_$v.so
        PTZBA_LIB=$L timeout -k 10 300 python bench.py --config $CFG $BARGS > gpurun_out/${TAG}_ab_${v}_$rep.json 2> gpurun_out/${TAG}_ab_${v}_$rep.err || { echo ABFAIL $v; tail gpurun_out/${TAG}_ab_${v}_$rep.err; exit 1; }
        summ gpurun_out/${TAG}_ab_${v}_$rep.json "$v#$rep"
      done
    done ;;
  dist)
    for n in ${DIST_N:-2 8}; do
      PTZBA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-accuracy --stream-frames 0 --no-cold ${DIST_ARGS} > gpurun_out/${TAG}_dist$n.json 2> gpurun_out/${TAG}_dist$n.err || { echo DISTFAIL $n; tail -20 gpurun_out/${TAG}_dist$n.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('world', d['n_gpus'], 'it/s', round(d['value'],1), d['config']['parallelism'], json.dumps(d.get('collective_fit')), json.dumps([{k: r[k] for k in ('rank','kernel_ms','collective_ms_per_iteration','n_collectives_per_iteration','factorisation_ms_net')} for r in d.get('per_rank') or []])[:1500])" gpurun_out/${TAG}_dist$n.json
    done ;;
  stream)
    IFS=';' read -ra SA <<< "${STREAM_ARGS:- }"
    k=0
    for args in "${SA[@]}"; do
      k=$((k + 1))
      timeout -k 10 300 python pan-tilt-zoom-slam_amd/demo_stream.py --frames 300 --window 30 $args > gpurun_out/${TAG}_stream$k.json 2> gpurun_out/${TAG}_stream$k.err || { echo STREAMFAIL; tail gpurun_out/${TAG}_stream$k.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'fps', round(d['fps_end_to_end'],1), 'kf', {k: round(v,2) for k,v in d['keyframe_ba_ms'].items()}, 'set_problem', round(d['keyframe_ba_breakdown_ms'].get('solve_set_problem_s',0),2), {k: round(v,3) for k,v in d['keyframe_ba_breakdown_ms'].items() if k.startswith('solve_setup_')})" gpurun_out/${TAG}_stream$k.json "[$args]"
    done ;;
  full)
    timeout -k 10 900 python bench.py ${FULL_ARGS} > gpurun_out/${TAG}_full.json 2> gpurun_out/${TAG}_full.err || { echo FULLFAIL; tail gpurun_out/${TAG}_full.err; exit 1; }
    summ gpurun_out/${TAG}_full.json full ;;
  *) echo "unknown step $st"; exit 2 ;;
  esac
done
