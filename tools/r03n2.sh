# End of round 3: bench.py --gpus 2 rehearsal on one device (two ranks, gloo exchanges) with the final tree's
# part-owned order (each half in the two-level order)
set -o pipefail
mkdir -p gpurun_out
PTZBA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/r03n2_bench_n2_gloo.json 2> gpurun_out/r03n2_bench_n2_gloo.err || { echo DISTFAIL; tail -20 gpurun_out/r03n2_bench_n2_gloo.err; exit 1; }
tail -1 gpurun_out/r03n2_bench_n2_gloo.json | cut -c1-1500
