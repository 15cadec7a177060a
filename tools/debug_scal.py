import sys, numpy as np
sys.path.insert(0, "pan-tilt-zoom-slam_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import ptzba, synthetic
from oracle import ptz_oracle as orc
for cfg in ("config1",):
    p = synthetic.make_problem(cfg, seed=0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v)
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    s = h.read_scalars()
    x = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    r = orc.compute_residual_records(x, p.n_pose, p.u, p.v, p.frame.astype(np.int64), p.landmark.astype(np.int64), p.xy)
    print(cfg, "cost gpu", s[0], "oracle", 0.5 * np.sum(r * r))
    h.build_reduced(1e-3); h.solve_reduced()
    s = h.read_scalars()
    print("scalars after solve", s)
    sp, n, scp = h.exchange()
    import torch
    from bench import _DevArray
    t = torch.as_tensor(_DevArray(scp, 8), device="cuda:0").cpu().numpy()
    print("raw scal", t)
