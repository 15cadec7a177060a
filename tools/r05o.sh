#!/bin/bash
# round 5: where K1's wave cycles go (SQ counters): parked on waits, issue-stalled, or issuing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r05o_pmc1 gpurun_out/r05o_pmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES --kernel-include-regex k_linearize -d gpurun_out/r05o_pmc1 -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold --stream-frames 0 > gpurun_out/r05o_b1.json 2> gpurun_out/r05o_b1.err || { tail gpurun_out/r05o_b1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --kernel-include-regex k_linearize -d gpurun_out/r05o_pmc2 -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-accuracy --no-secondary --no-cold --stream-frames 0 > gpurun_out/r05o_b2.json 2> gpurun_out/r05o_b2.err || { tail gpurun_out/r05o_b2.err; exit 1; }
ls gpurun_out/r05o_pmc1 gpurun_out/r05o_pmc2
echo done
