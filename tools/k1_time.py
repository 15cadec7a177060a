"""Time K1 alone: n back-to-back h.linearize() launches at config 3 (fp32 + Huber), HIP events on the handle's stream
(torch's current stream, attached with set_stream).  PTZBA_LIB selects a variant library (ablation builds:
tools/r05r.sh).  Prints one line: variant, mean us per launch."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "default"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
p = synthetic.make_problem("config3", seed=0)
h = ptzba.BAHandle(0)
h.set_stream(torch.cuda.current_stream().cuda_stream)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
              loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays)
for _ in range(10):
    h.linearize()
torch.cuda.synchronize()
res = []
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        h.linearize()
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) * 1e3 / n)
print(f"{tag:10s} K1 us per launch (3 reps of {n}): " + " ".join(f"{x:.2f}" for x in res), flush=True)
