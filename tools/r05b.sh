#!/bin/bash
# Huber curvature factor x damping start at the reference's ftol=1e-4 stop (config 2 / 3, fp32 + Huber)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 LAMS=1e-12,1e-6
for hc in 1 0.5 0.3 0.1 0.03; do
  PTZBA_HUBER_CURV=$hc timeout -k 10 200 python -u tools/ftol_study.py config2 config3 huber-only >> gpurun_out/r05b_ftol_study.jsonl 2>> gpurun_out/r05b_ftol_study.err || exit 1
done
echo done
