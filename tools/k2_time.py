"""Time K2 (k_schur_mf + k_schur_reduce: the bench's "schur" group, HIP events around every launch) alone at config 3
(fp32 + Huber): n ptzba_build_reduced calls after one linearisation.  PTZBA_LIB selects a variant library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "default"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
p = synthetic.make_problem("config3", seed=0)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
              loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays)
h.linearize()
for _ in range(5):
    h.build_reduced(1e-4)
h.sync()
res = []
for rep in range(3):
    h.reset_kernel_times(True, groups=2, stride=1)
    for _ in range(n):
        h.build_reduced(1e-4)
    res.append(h.kernel_times()["schur"][0] * 1e3)
h.reset_kernel_times(False)
print(f"{tag:10s} K2 us per build (3 reps of {n}): " + " ".join(f"{x:.2f}" for x in res), flush=True)
