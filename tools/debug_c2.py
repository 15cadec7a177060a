import sys, numpy as np
sys.path.insert(0, "pan-tilt-zoom-slam_amd"); sys.path.insert(0, ".")
import ptzba, synthetic
d = np.load("tests/golden/config2_optimum.npz")
p = synthetic.make_problem("config2", seed=0)
xt = d["x_tight"]; ptz_t = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
for prec in (0, 1):
    for kw in (dict(ftol=1e-12, xtol=1e-12), dict(ftol=0.0, xtol=1e-10), dict(ftol=0, xtol=0, max_iter=60)):
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec)
        h.set_state(p.init_ptz, p.init_rays)
        res = ptzba.LMSolver(h, **kw).run()
        ptz, rays = h.get_state()
        print(prec, kw, res, "rmse", synthetic.pose_rmse(ptz, ptz_t), "lam", res.lam, "last", res.history[-3:])
        h.close()
