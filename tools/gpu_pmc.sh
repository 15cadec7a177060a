# PMC passes (one rocprofv3 run per pass, counters within the gfx950 slot limits) over a short bench;
# per-kernel averages of every counter -> gpurun_out/pmc_<tag>_summary.txt
set -o pipefail
TAG=${TAG:-x}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
BARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-accuracy --no-cold --no-secondary --config4-steps 0 --stream-frames 0"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES" ${PMC_EXTRA:+"$PMC_EXTRA"}; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${TAG}_$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- python bench.py $BARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo PMCFAIL $i; tail gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_* > gpurun_out/pmc_${TAG}_summary.txt && cat gpurun_out/pmc_${TAG}_summary.txt
