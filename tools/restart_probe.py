import sys, time, os
sys.path.insert(0, "pan-tilt-zoom-slam_amd")
import numpy as np, ptzba, synthetic
p = synthetic.make_problem("config3", seed=0)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32, loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays); h.save_state()
for rep in range(3):
    h.restore_state(); ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100).run()
h.sync()
ts=[]; its=0
t0=time.perf_counter()
for rep in range(10):
    a=time.perf_counter(); h.restore_state(); r=ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100).run(); b=time.perf_counter()
    ts.append(b-a); its+=r.njev
h.sync(); t1=time.perf_counter()
print("per solve ms", [round(x*1e3,2) for x in ts], "iters", its, "total", round((t1-t0)*1e3,2), "ms ->", round(its/(t1-t0),1), "it/s")
