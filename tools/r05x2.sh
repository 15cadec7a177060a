#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05x2
for rep in 1 2; do
for v in 0 s64 s32 s16; do
  unset PTZBA_CHOL_XCD PTZBA_CX_SLOTS
  case $v in 0) export PTZBA_CHOL_XCD=0;; s64) export PTZBA_CX_SLOTS=64;; s32) export PTZBA_CX_SLOTS=32;; s16) export PTZBA_CX_SLOTS=16;; esac
  timeout -k 10 200 python bench.py --steps 300 --no-cpu-baseline --no-accuracy --no-secondary --stream-frames 0 > gpurun_out/${T}_$v$rep.json 2> gpurun_out/${T}_$v$rep.err || { tail gpurun_out/${T}_$v$rep.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${T}_$v$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['kernel_ms'].items()})"
done
done
