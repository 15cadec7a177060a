# Round-3 config-3 A/B on one box: HEAD~3 library (libptzba_base.so) vs the tree, the one-level order, the
# blocked back-solve, the chunk-pair K2
set -o pipefail
mkdir -p gpurun_out
VARIANTS="default base ENV_PTZBA_ND_DEPTH=1 ENV_PTZBA_BACKSOLVE=blk ENV_PTZBA_SCHUR=mf2" bash tools/gpu_lib_ab.sh || exit 1
