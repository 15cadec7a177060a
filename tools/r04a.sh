# Round 4 pass A: full GPU tests, then the plain bench for the defaults and the A/B knobs of this round's changes
# (K1 frame tables in LDS, k_trial dense-slot walk, C-driven restart loop), then the config-5 stream demo.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a_gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r04a_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04a_gpu_tests.log
REPS=${REPS:-2} AB_ENVS="PTZBA_K1_FTL=0 PTZBA_TRIAL_DPL=0 PTZBA_BENCH_PYLOOP=1 PTZBA_CHOL_XCD=1 PTZBA_K2_FOLD=2 PTZBA_BS_PERSIST=1 PTZBA_RED_BLOCKS=8 PTZBA_LIB=$GRAFT_REPO_ROOT/pan-tilt-zoom-slam_amd/libptzba_k1o5.so" bash tools/r04ab.sh || exit 1
timeout -k 10 600 python pan-tilt-zoom-slam_amd/demo_stream.py --frames 300 > gpurun_out/r04a_demo_stream.json 2> gpurun_out/r04a_demo_stream.err || { echo DEMOFAIL; tail -20 gpurun_out/r04a_demo_stream.err; exit 1; }
tail -c 1800 gpurun_out/r04a_demo_stream.json
