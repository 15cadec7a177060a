"""Debug A/B: LM scalars of one linearise + step (several lambdas) and the first iterations of a solve at config 3
(fp32 / fp64, Huber) for the library PTZBA_LIB points at; writes gpurun_out/scal_<tag>.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

tag = sys.argv[1]
p = synthetic.make_problem("config3", seed=0)
out = {}
for name, prec in (("fp32", ptzba.FP32), ("fp64", ptzba.FP64)):
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    for lam in (1e-4, 1e-2):
        h.step(lam)
        out[f"{name}_step{lam}"] = h.read_scalars()
    res = ptzba.LMSolver(h, ftol=1e-10, xtol=1e-12, max_iter=60).run()
    ptz, rays = h.get_state()
    out[f"{name}_res"] = np.array([res.status, res.cost, res.njev, res.nfev])
    out[f"{name}_ptz"] = ptz
    print(tag, name, res, flush=True)
    h.close()
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/scal_{tag}.npz", **out)
