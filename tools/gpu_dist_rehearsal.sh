# N=2 rehearsal of bench.py's sharded protocol on a one-GPU box: two ranks share the device and
# all-reduce through gloo (the packed exchange, the scalars, max-over-ranks timing).
set -o pipefail
mkdir -p gpurun_out
PTZBA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { echo DISTFAIL; tail -20 gpurun_out/dist2.err; exit 1; }
tail -1 gpurun_out/dist2.json
