#!/bin/bash
# round-4 final pass, part 2: the SIFT / front-end / stream GPU tests and the stream on the last code commit
# (tools/r04z6.sh), then rocprofv3 kernel stats, K1 / K2 PMC traffic, the bench line with this run's traffic, PMC
# calibration, smoke, config-4 bench (tools/r04b.sh with TAG=r04fin)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04z6.sh || exit 1
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=r04fin bash tools/r04b.sh
