import sys, numpy as np
sys.path.insert(0, "pan-tilt-zoom-slam_amd"); sys.path.insert(0, ".")
import ptzba, synthetic
from oracle import ptz_oracle as orc
p = synthetic.make_problem(sys.argv[1] if len(sys.argv) > 1 else "config1", seed=0)
fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=0)
h.set_state(p.init_ptz, p.init_rays)
prev = None
for it in range(12):
    ptz0, rays0 = h.get_state()
    x0 = np.concatenate([ptz0[1:].reshape(-1), rays0.reshape(-1)])
    h.linearize(); c = h.read_scalars()[0]
    h.build_reduced(0.0); h.solve_reduced(); s = h.read_scalars(); h.accept(True)
    ptz1, rays1 = h.get_state()
    dx_gpu = np.concatenate([(ptz1 - ptz0)[1:].reshape(-1), (rays1 - rays0).reshape(-1)])
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm)
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    from scipy.sparse.linalg import spsolve
    H = (J.T @ J).tocsc(); g = J.T @ r
    dx = spsolve(H, -g)
    print(f"it {it} cost {c:.10f} trial {s[1]:.10f} |dx| {np.abs(dx).max():.3e} |dx_gpu-dx| {np.abs(dx_gpu-dx).max():.3e} "
          f"argmax {np.argmax(np.abs(dx_gpu-dx))} n_pose3={3*(p.n_pose-1)}")
