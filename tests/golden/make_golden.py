"""
Generate golden fixtures by RUNNING THE REFERENCE (build container only; /root/reference does not
exist on the GPU box).  Recipe = SURVEY §8c: the reference's Python hot path is imported in place
with stub modules for its three import-time blockers (cv2, pyflann, the ctypes RF module), and its
OpenCV front-end (`detect_compute_sift`, `match_sift_features`) is monkeypatched with synthetic
ground-truth correspondences.  Everything downstream runs unmodified: matching-graph bookkeeping
incl. the random.shuffle cap, landmark ids, x0 init, scipy trf, keyframe assembly, EKF update.

Nothing from /root/reference is copied: only numeric inputs/outputs are written (tests/golden/*.npz).
Bytecode writing is disabled so no reference .pyc lands anywhere.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--quick]
"""
import argparse
import os
import random
import sys
import time
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/slam_system"

import numpy as np  # noqa: E402


def install_stubs():
    cv2 = types.ModuleType("cv2")
    cv2.imwrite = lambda *a, **k: True
    cv2.line = lambda *a, **k: None
    sys.modules["cv2"] = cv2
    sys.modules["pyflann"] = types.ModuleType("pyflann")
    for name in ["rf_map", "rf_map.python_package", "rf_map.python_package.backup"]:
        m = types.ModuleType(name)
        m.__path__ = []
        sys.modules[name] = m
    rf = types.ModuleType("rf_map.python_package.backup.rf_map")
    rf.RFMap = object
    sys.modules["rf_map.python_package.backup.rf_map"] = rf
    sys.path.insert(0, REF)


install_stubs()
import importlib.util  # noqa: E402

# the build's own generator (numpy only), loaded by path so the product's same-named modules never
# shadow the reference's on sys.path
_spec = importlib.util.spec_from_file_location("synthetic", os.path.join(REPO, "pan-tilt-zoom-slam_amd", "synthetic.py"))
synthetic = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synthetic)
import bundle_adjustment as ref_ba  # noqa: E402  (REFERENCE module, via sys.path above)
import image_process as ref_ip  # noqa: E402
import transformation as ref_tf  # noqa: E402
import ptz_camera as ref_cam  # noqa: E402
import ptz_slam as ref_slam  # noqa: E402
from scipy.optimize import least_squares  # noqa: E402

assert ref_ba.__file__.startswith(REF), ref_ba.__file__
assert synthetic.__file__.startswith(REPO)


def out(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, os.path.getsize(path), "bytes")


# --------------------------------------------------------------------------------------------
# 1. projection KATs
# --------------------------------------------------------------------------------------------
def gen_projection(rng):
    n = 2000
    u, v = 640.0, 360.0
    f = rng.uniform(1900, 4300, n)
    cp = rng.uniform(40, 80, n)
    ct = rng.uniform(-15, 0, n)
    th = cp + rng.uniform(-20, 20, n)
    ph = ct + rng.uniform(-10, 10, n)
    # behind-camera subset (q2 < 0): ray > 90 deg away from the optical axis in pan
    nb = 400
    fb = rng.uniform(1900, 4300, nb)
    cpb = rng.uniform(50, 80, nb)
    ctb = rng.uniform(-15, 0, nb)
    thb = rng.uniform(-85, -30, nb)
    phb = rng.uniform(-25, 5, nb)
    F = np.concatenate([f, fb]); CP = np.concatenate([cp, cpb]); CT = np.concatenate([ct, ctb])
    TH = np.concatenate([th, thb]); PH = np.concatenate([ph, phb])
    xy = np.array([ref_tf.TransFunction.from_ray_to_image(u, v, a, b, c, d, e)
                   for a, b, c, d, e in zip(F, CP, CT, TH, PH)])
    # back-projection of random image points
    px = rng.uniform(0, 1280, n)
    py = rng.uniform(0, 720, n)
    ray = np.array([ref_tf.TransFunction.from_image_to_ray(u, v, a, b, c, d, e)
                    for a, b, c, d, e in zip(f, cp, ct, px, py)])
    # PTZCamera matrix form (signed q2), zero and non-zero displacement
    nc = 300
    disp = np.array([0.01, -0.02, 0.03, 1e-5, -2e-5, 3e-5])
    cam_rows = []
    for k in range(nc):
        d = None if k % 2 == 0 else disp
        cam = ref_cam.PTZCamera((u, v), np.zeros(3), np.eye(3), d)
        cam.set_ptz([cp[k], ct[k], f[k]])
        pr = cam.project_ray([th[k], ph[k]])
        bp = cam.back_project_to_ray(px[k], py[k])
        cam_rows.append([k % 2, cp[k], ct[k], f[k], th[k], ph[k], pr[0], pr[1], px[k], py[k], bp[0], bp[1]])
    out("kat_projection.npz", u=u, v=v, f=F, cam_pan=CP, cam_tilt=CT, theta=TH, phi=PH, xy=xy,
        n_front=n, bp_f=f, bp_pan=cp, bp_tilt=ct, bp_x=px, bp_y=py, bp_ray=ray,
        cam_rows=np.array(cam_rows), displacement=disp)


# --------------------------------------------------------------------------------------------
# synthetic detect/match monkeypatch for the reference front-end
# --------------------------------------------------------------------------------------------
class KP:
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (float(x), float(y))


class FrontEnd:
    """Stands in for cv2 SIFT + BF matching: 'images' are frame ids; matches are ground truth,
    optionally with injected inconsistent matches."""

    def __init__(self, scene, corrupt=0, seed=0):
        self.scene = scene
        self.corrupt = corrupt
        self.rng = np.random.default_rng(seed)
        self.raw = {}  # (i, j) -> (index1, index2) returned to the reference
        self.kps = {}  # frame -> keypoint objects handed out (to recover local indices)

    def detect(self, im, nfeatures, verbose=False):
        i = int(im)
        kps = [KP(x, y) for x, y in self.scene.kp_xy[i]]
        des = np.full((len(kps), 128), i, dtype=np.float32)
        des[:, 1] = np.arange(len(kps))
        self.kps[i] = kps
        return kps, des

    def match(self, kp1, des1, kp2, des2, pts_array=False, verbose=False):
        i = int(des1[0, 0]); j = int(des2[0, 0])
        r1 = self.scene.kp_ray[i]; r2 = self.scene.kp_ray[j]
        pos2 = {int(r): k for k, r in enumerate(r2)}
        idx1, idx2 = [], []
        for a, r in enumerate(r1):
            b = pos2.get(int(r))
            if b is not None:
                idx1.append(a); idx2.append(b)
        if self.corrupt and len(idx2) > 4:
            for _ in range(self.corrupt):
                p, q = self.rng.choice(len(idx2), 2, replace=False)
                idx2[p], idx2[q] = idx2[q], idx2[p]
        self.raw[(i, j)] = (list(idx1), list(idx2))
        pts1 = np.array([kp1[a].pt for a in idx1]).reshape(-1, 2)
        pts2 = np.array([kp2[b].pt for b in idx2]).reshape(-1, 2)
        return pts1, idx1, pts2, idx2


def pack_points(scene):
    off = np.concatenate([[0], np.cumsum([len(p) for p in scene.kp_xy])]).astype(np.int64)
    return np.concatenate(scene.kp_xy), off


def pack_raw(raw):
    keys = sorted(raw)
    pi = np.array([k[0] for k in keys], np.int64)
    pj = np.array([k[1] for k in keys], np.int64)
    cnt = np.array([len(raw[k][0]) for k in keys], np.int64)
    a = np.concatenate([np.asarray(raw[k][0], np.int64) for k in keys]) if keys else np.zeros(0, np.int64)
    b = np.concatenate([np.asarray(raw[k][1], np.int64) for k in keys]) if keys else np.zeros(0, np.int64)
    return pi, pj, cnt, a, b


def pack_lists(src, dst, lmk):
    n = len(src)
    mi, mj, k1, k2, lm = [], [], [], [], []
    for i in range(n):
        for j in range(n):
            for a, b, l in zip(src[i][j], dst[i][j], lmk[i][j]):
                mi.append(i); mj.append(j); k1.append(a); k2.append(b); lm.append(l)
    return [np.array(x, np.int64) for x in (mi, mj, k1, k2, lm)]


# --------------------------------------------------------------------------------------------
# 2-4. bundle_adjustment() end-to-end + residual vectors + tight optimum
# --------------------------------------------------------------------------------------------
def gen_ba(name, n_kf, n_rays, lo, hi, seed, tight=True):
    scene = synthetic.make_scene(n_kf, n_rays, lo, hi, seed=seed)
    fe = FrontEnd(scene)
    ref_ip.detect_compute_sift = fe.detect
    ref_ip.match_sift_features = fe.match
    ref_ba.draw_matches = lambda *a, **k: None
    captured = {}
    real_ls = ref_ba.least_squares

    def ls_capture(fun, x0, **kw):
        captured["x0"] = np.array(x0, copy=True)
        captured["args"] = kw["args"]
        t0 = time.time()
        res = real_ls(fun, x0, **kw)
        captured["time"] = time.time() - t0
        captured["res"] = res
        return res

    ref_ba.least_squares = ls_capture
    random.seed(seed)
    images = list(range(n_kf))
    center = np.array([0.0, -10.0, 5.0])
    rotation = np.eye(3)
    t0 = time.time()
    landmarks, keyframes = ref_ba.bundle_adjustment(images, list(range(100, 100 + n_kf)), "sift",
                                                    scene.init_ptz.copy(), center, rotation,
                                                    scene.u, scene.v, "/tmp", verbose=False)
    wall = time.time() - t0
    ref_ba.least_squares = real_ls
    res = captured["res"]
    (n_pose, n_landmark, n_residual, points, src, dst, lmk, u, v, ref_pose) = captured["args"]
    mi, mj, k1, k2, lm = pack_lists(src, dst, lmk)
    pts, off = pack_points(scene)
    pi, pj, cnt, ra, rb = pack_raw(fe.raw)
    # residual vectors at x0, x*, 3 perturbations
    rng = np.random.default_rng(seed + 1)
    xs = [captured["x0"], res.x]
    for _ in range(3):
        xs.append(res.x + rng.normal(0, 1, res.x.shape) * np.concatenate(
            [np.tile([0.05, 0.05, 5.0], n_pose - 1), np.full(2 * n_landmark, 0.05)]))
    rs = [ref_ba._compute_residual(x, *captured["args"]) for x in xs]
    kf_local = []
    for i, kf in enumerate(keyframes):
        pos = {id(o): k for k, o in enumerate(fe.kps[i])}
        kf_local.append(np.array([pos[id(o)] for o in kf.feature_pts], np.int64))
    kf_lmk = [np.asarray(kf.landmark_index, np.int64) for kf in keyframes]
    kf_pts = [np.array([p.pt for p in kf.feature_pts]).reshape(-1, 2) for kf in keyframes]
    kf_off = np.concatenate([[0], np.cumsum([len(a) for a in kf_lmk])]).astype(np.int64)
    data = dict(
        n_kf=n_kf, n_rays=n_rays, lo=lo, hi=hi, seed=seed, u=u, v=v,
        init_ptz=scene.init_ptz, gt_ptz=scene.gt_ptz, points=pts, points_off=off,
        raw_pi=pi, raw_pj=pj, raw_cnt=cnt, raw_a=ra, raw_b=rb,
        n_pose=n_pose, n_landmark=n_landmark, n_residual=n_residual,
        m_i=mi, m_j=mj, m_k1=k1, m_k2=k2, m_lm=lm, ref_pose=np.asarray(ref_pose, np.float64),
        x0=captured["x0"], x_ls=res.x, ls_cost=res.cost, ls_njev=res.njev, ls_nfev=res.nfev,
        ls_status=res.status, ls_time=captured["time"], ba_wall=wall,
        landmarks=landmarks, kf_ptz=np.array([[k.pan, k.tilt, k.f] for k in keyframes]),
        kf_lmk=np.concatenate(kf_lmk) if kf_lmk else np.zeros(0), kf_off=kf_off,
        kf_pts=np.concatenate(kf_pts) if kf_pts else np.zeros((0, 2)),
        kf_local=np.concatenate(kf_local) if kf_local else np.zeros(0, np.int64),
        xs=np.stack(xs), rs=np.stack(rs))
    print(f"{name}: N={n_pose} M={n_landmark} residuals={n_residual} njev={res.njev} "
          f"ls {captured['time']:.2f}s ({res.njev / captured['time']:.4f} it/s) status={res.status}")
    if tight:
        t0 = time.time()
        rt = least_squares(ref_ba._compute_residual, captured["x0"], x_scale="jac", ftol=1e-15,
                           xtol=1e-15, gtol=1e-15, method="trf", args=captured["args"])
        data.update(x_tight=rt.x, tight_cost=rt.cost, tight_njev=rt.njev, tight_status=rt.status,
                    tight_time=time.time() - t0)
        print(f"  tight: cost {rt.cost:.6f} njev {rt.njev} status {rt.status} {time.time() - t0:.1f}s")
    out(f"{name}.npz", **data)


# --------------------------------------------------------------------------------------------
# 6. matching-graph bookkeeping with caps (>200) and inconsistent matches
# --------------------------------------------------------------------------------------------
def gen_graph(seed):
    scene = synthetic.make_scene(6, 900, 50, 60, seed=seed)
    fe = FrontEnd(scene, corrupt=6, seed=seed)
    ref_ip.detect_compute_sift = fe.detect
    ref_ip.match_sift_features = fe.match
    n = 6
    mask = [[0] * n for _ in range(n)]
    ip = scene.init_ptz
    for i in range(n):
        for j in range(n):
            if synthetic.overlap_pan_angle(ip[i, 2], ip[i, 0], ip[j, 2], ip[j, 0], 1280) > 5:
                mask[i][j] = 1
    random.seed(seed)
    kps, des, points, src, dst, lmk, n_landmark = ref_ip.build_matching_graph(list(range(n)), mask, "sift")
    mi, mj, k1, k2, lm = pack_lists(src, dst, lmk)
    pi, pj, cnt, ra, rb = pack_raw(fe.raw)
    pts, off = pack_points(scene)
    print(f"graph: landmarks={n_landmark} matches={len(mi)} raw={int(cnt.sum())} max_raw={int(cnt.max())}")
    out("matching_graph.npz", seed=seed, mask=np.array(mask), raw_pi=pi, raw_pj=pj, raw_cnt=cnt, raw_a=ra,
        raw_b=rb, n_landmark=n_landmark, m_i=mi, m_j=mj, m_k1=k1, m_k2=k2, m_lm=lm, points=pts, points_off=off)


# --------------------------------------------------------------------------------------------
# 7. EKF update (ptz_slam.py:210-289) and compute_h_jacobian (:73-138)
# --------------------------------------------------------------------------------------------
def gen_ekf(R, seed):
    rng = np.random.default_rng(seed)
    u, v = 640.0, 360.0
    pan, tilt, f = 58.0, -8.0, 3000.0
    cam = ref_cam.PTZCamera((u, v), np.array([0.0, -10.0, 5.0]), np.eye(3))
    cam.set_ptz([pan, tilt, f])
    pts = np.stack([rng.uniform(20, 1260, R), rng.uniform(20, 700, R)], 1)
    rays = cam.back_project_to_rays(pts)
    rays = rays + rng.normal(0, 0.02, rays.shape)
    slam = ref_slam.PtzSlam()
    slam.cameras = [cam]
    slam.rays = rays.copy()
    cov = slam.angle_var * np.eye(3 + 2 * R)
    cov[2, 2] = slam.f_var
    B = rng.normal(0, 3e-3, (3 + 2 * R, 4))  # low-rank correlation so cov0 = base + B B^T is storable
    cov = cov + B @ B.T
    slam.state_cov = cov.copy()
    import copy
    pred = copy.deepcopy(cam)
    pred.set_ptz([pan + 0.05, tilt - 0.03, f + 5.0])
    slam.current_camera = pred
    # observations: true projections + noise, a sorted subset of rays (some dropped)
    keep = np.sort(rng.choice(R, int(R * 0.8), replace=False))
    true_cam = copy.deepcopy(cam)
    true_cam.set_ptz([pan + 0.08, tilt - 0.05, f + 8.0])
    obs = np.array([true_cam.project_ray(rays[k]) for k in keep]) + rng.normal(0, 0.3, (len(keep), 2))
    before = dict(pan=pred.pan, tilt=pred.tilt, f=pred.focal_length, rays=slam.rays.copy(), cov=slam.state_cov.copy())
    H = slam.compute_h_jacobian(pred.pan, pred.tilt, pred.focal_length, rays[keep[:20]])
    t0 = time.time()
    slam.ekf_update(obs, keep, 720, 1280)
    dt = time.time() - t0
    print(f"ekf R={R}: {dt:.3f}s")
    cov1 = slam.state_cov
    changed = np.argwhere(cov1 != before["cov"])
    pick = changed[np.random.default_rng(seed + 9).choice(len(changed), min(3000, len(changed)), replace=False)]
    out(f"ekf_R{R}.npz", u=u, v=v, pan0=before["pan"], tilt0=before["tilt"], f0=before["f"],
        rays0=before["rays"], cov_base_diag=np.diag(slam.angle_var * np.eye(3 + 2 * R)).copy(), f_var=slam.f_var,
        cov_B=B, obs=obs, obs_idx=keep, height=720, width=1280,
        pan1=slam.current_camera.pan, tilt1=slam.current_camera.tilt, f1=slam.current_camera.focal_length,
        velocity=slam.velocity, rays1=slam.rays, cov1_pose=cov1[:3, :3], cov1_diag=np.diag(cov1).copy(),
        cov1_sum=float(cov1.sum()), cov1_sumsq=float((cov1 * cov1).sum()), n_changed=len(changed),
        cov1_pick=pick, cov1_pick_val=cov1[pick[:, 0], pick[:, 1]], H=H, H_rays=rays[keep[:20]], time=dt)


# --------------------------------------------------------------------------------------------
# 5. config-2-scale optimum (oracle residual pinned by 2/4 above) + reference residual samples
# --------------------------------------------------------------------------------------------
def gen_config2():
    sys.path.insert(0, REPO)
    from oracle import ptz_oracle as orc
    p = synthetic.make_problem("config2", seed=0)
    n, m = p.n_pose, p.n_landmark
    x0_full = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    # reference residual at x0 on a 1000-sample subset, via the reference's own loop
    mi, mj, k1, k2 = (p.meta[k] for k in ("match_i", "match_j", "kp1", "kp2"))
    lm = p.landmark[0::2].astype(np.int64)
    # keypoints: per-frame arrays of the same scene (kp1/kp2 index into them)
    scene = synthetic.make_scene(*synthetic.CONFIGS["config2"][:4], seed=0)
    pts = scene.kp_xy
    src = [[[] for _ in range(n)] for _ in range(n)]
    dst = [[[] for _ in range(n)] for _ in range(n)]
    lmk = [[[] for _ in range(n)] for _ in range(n)]
    for a, b, c, d, l in zip(mi, mj, k1, k2, lm):
        src[a][b].append(int(c)); dst[a][b].append(int(d)); lmk[a][b].append(int(l))
    args = (n, m, 4 * len(mi), pts, src, dst, lmk, p.u, p.v, p.init_ptz[0])
    t0 = time.time()
    r_ref = ref_ba._compute_residual(x0_full[3:], *args)
    t_ref = time.time() - t0
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(len(r_ref), 1000, replace=False))
    frame = p.frame.astype(np.int64)
    landmark = p.landmark.astype(np.int64)

    def polish(x, loss):
        """Exact sparse Gauss-Newton (IRLS weights for huber) from scipy's trf solution to the
        stationary point sum rho'(r^2) J^T r = 0 of the same cost (scipy.sparse Cholesky-free solve)."""
        from scipy.sparse import diags
        from scipy.sparse.linalg import spsolve
        ref = p.init_ptz[0]
        for it in range(60):
            xf = np.concatenate([ref, x])
            r = orc.compute_residual_records(xf, n, p.u, p.v, frame, landmark, p.xy)
            J = orc.ba_jacobian(x, n, m, p.u, p.v, ref, frame, landmark)
            w = np.ones_like(r) if loss == "linear" else np.where(np.abs(r) <= 1.0, 1.0, 1.0 / np.maximum(np.abs(r), 1e-300))
            JW = J.T @ diags(w)
            g = JW @ r
            H = (JW @ J).tocsc()
            dx = spsolve(H, -g)
            x = x + dx
            if np.max(np.abs(dx)) < 1e-11:
                break
        return x, (it, float(np.max(np.abs(dx))))

    t0 = time.time()
    res = orc.solve_scipy(x0_full[3:], n, m, p.u, p.v, p.init_ptz[0], frame, landmark, p.xy, ftol=1e-10, xtol=1e-12,
                          gtol=1e-12, analytic=True)
    xt, its = polish(res.x, "linear")
    cost_t = orc.ba_cost(np.concatenate([p.init_ptz[0], xt]), n, p.u, p.v, frame, landmark, p.xy)
    print(f"config2 tight: scipy cost {res.cost:.8f} njev {res.njev}; polished cost {cost_t:.8f} in {its} GN steps "
          f"{time.time() - t0:.1f}s; ref residual eval {t_ref:.2f}s")
    # huber (scipy loss='huber', f_scale=1): its stationary point sum rho'(r^2) J^T r = 0, reached by IRLS
    # Gauss-Newton from the linear optimum (scipy trf+lsmr at tight tolerance needs > 10 min here)
    xh, its_h = polish(xt, "huber")
    cost_h = orc.ba_cost(np.concatenate([p.init_ptz[0], xh]), n, p.u, p.v, frame, landmark, p.xy, loss="huber")
    print(f"config2 tight huber: IRLS-GN cost {cost_h:.8f} in {its_h} steps")
    res = type("R", (), dict(x=xt, cost=cost_t))
    res_h = type("R", (), dict(x=xh, cost=cost_h))
    out("config2_optimum.npz", n_pose=n, n_landmark=m, n_records=len(p.frame),
        frame_sum=int(p.frame.sum()), landmark_sum=int(p.landmark.astype(np.int64).sum()),
        xy_sum=float(p.xy.sum()), x0=x0_full, r_ref_sample_idx=sample, r_ref_sample=r_ref[sample],
        r_ref_sumsq=float(np.sum(r_ref * r_ref)), x_tight=res.x, tight_cost=res.cost,
        x_tight_huber=res_h.x, tight_cost_huber=res_h.cost, ref_residual_time=t_ref)


# --------------------------------------------------------------------------------------------
# 5a. config-2 at the reference's own termination: scipy trf, x_scale='jac', ftol=1e-4, FD Jacobian
# --------------------------------------------------------------------------------------------
def gen_config2_ftol():
    """Where the reference's optimizer call (bundle_adjustment.py:200-202: least_squares(_compute_residual, x0,
    x_scale='jac', ftol=1e-4, method='trf'), '2-point' FD Jacobian with the pair structure as jac_sparsity) stops at
    config 2, on the pinned oracle residual (config2_optimum.npz pins it to the reference's own): x_ftol, njev,
    nfev, cost, status -- for the reference's linear loss and for loss='huber' (f_scale 1).  The GPU's ftol=1e-4
    solves are gated against it (tests/test_gpu_ba.py::test_config2_ftol_stop_matches_scipy_trf)."""
    sys.path.insert(0, REPO)
    from oracle import ptz_oracle as orc
    p = synthetic.make_problem("config2", seed=0)
    n, m = p.n_pose, p.n_landmark
    frame = p.frame.astype(np.int64)
    landmark = p.landmark.astype(np.int64)
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    arrays = dict(n_pose=n, n_landmark=m, n_records=len(p.frame), frame_sum=int(p.frame.sum()), x0=x0)
    for loss, key in (("linear", ""), ("huber", "_huber")):
        t0 = time.time()
        res = orc.solve_scipy(x0, n, m, p.u, p.v, p.init_ptz[0], frame, landmark, p.xy, ftol=1e-4, loss=loss,
                              f_scale=1.0)
        dt = time.time() - t0
        print(f"config2 ftol=1e-4 {loss}: cost {res.cost:.8f} njev {res.njev} nfev {res.nfev} status {res.status} "
              f"{dt:.1f}s")
        arrays.update({"x_ftol" + key: res.x, "cost_ftol" + key: res.cost, "njev" + key: res.njev,
                       "nfev" + key: res.nfev, "status" + key: res.status, "time" + key: dt})
    out("config2_ftol.npz", **arrays)


# --------------------------------------------------------------------------------------------
# 5b. config-3 (headline, 500 KF x 20k rays) tight optimum: the parity target of the bench's RMSE
# --------------------------------------------------------------------------------------------
def gen_config3():
    """Headline-size optimum of the pinned oracle: the reference residual
    (bundle_adjustment.py:25-106) with frame 0 as the gauge, minimised to a step of max |dx| < 1e-11 by
    orc.schur_tight_solve (landmarks eliminated per 2x2 block; J is never materialised at 29.2M x 41k).  The same
    solver reproduces config2_optimum.npz (scipy trf + sparse GN polish) to 1e-13 px.  Linear loss from x0, Huber
    (scipy's loss='huber', f_scale=1) from the linear optimum, as gen_config2.  A 1000-residual sample of the
    REFERENCE's own _compute_residual at x0 pins the records."""
    sys.path.insert(0, REPO)
    from oracle import ptz_oracle as orc
    t_all = time.time()
    p = synthetic.make_problem("config3", seed=0)
    n, m = p.n_pose, p.n_landmark
    frame = p.frame.astype(np.int64)
    landmark = p.landmark.astype(np.int64)
    print(f"config3: {n} KF, {m} landmarks, {len(frame)} records ({time.time() - t_all:.1f}s)")
    x0_full = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    mi, mj, k1, k2 = (p.meta[k] for k in ("match_i", "match_j", "kp1", "kp2"))
    scene = synthetic.make_scene(*synthetic.CONFIGS["config3"][:4], seed=0)
    pts = scene.kp_xy
    src = [[[] for _ in range(n)] for _ in range(n)]
    dst = [[[] for _ in range(n)] for _ in range(n)]
    lmk = [[[] for _ in range(n)] for _ in range(n)]
    for a_, b_, c_, d_, l_ in zip(mi.tolist(), mj.tolist(), k1.tolist(), k2.tolist(), landmark[0::2].tolist()):
        src[a_][b_].append(c_); dst[a_][b_].append(d_); lmk[a_][b_].append(l_)
    args = (n, m, 4 * len(mi), pts, src, dst, lmk, p.u, p.v, p.init_ptz[0])
    t0 = time.time()
    r_ref = ref_ba._compute_residual(x0_full[3:], *args)
    t_ref = time.time() - t0
    r_orc = orc.compute_residual_records(x0_full, n, p.u, p.v, frame, landmark, p.xy)
    print(f"config3 reference residual: {len(r_ref)} values in {t_ref:.1f}s, max |ref - oracle| "
          f"{np.abs(r_ref - r_orc).max():.3e}")
    del src, dst, lmk
    rng = np.random.default_rng(7)
    sample = np.sort(rng.choice(len(r_ref), 1000, replace=False))
    log = lambda s: print(s, flush=True)  # noqa: E731
    t0 = time.time()
    ptz_l, rays_l, info_l = orc.schur_tight_solve(p.init_ptz, p.init_rays, p.u, p.v, frame, landmark, p.xy,
                                                  loss="linear", log=log)
    t_l = time.time() - t0
    print(f"config3 linear: cost {info_l['cost']:.8f} in {info_l['iterations']} steps, {t_l:.0f}s")
    t0 = time.time()
    ptz_h, rays_h, info_h = orc.schur_tight_solve(ptz_l, rays_l, p.u, p.v, frame, landmark, p.xy, loss="huber",
                                                  f_scale=1.0, log=log)
    t_h = time.time() - t0
    print(f"config3 huber: cost {info_h['cost']:.8f} in {info_h['iterations']} steps, {t_h:.0f}s")
    # first-order optimality of both points (max |gradient| per parameter kind; x0's for scale)
    key, seg = np.unique(landmark * n + frame, return_inverse=True)
    grads = {}
    for name, (a_, b_, loss) in {"x0": (p.init_ptz, p.init_rays, "linear"), "linear": (ptz_l, rays_l, "linear"),
                                 "x0_huber": (p.init_ptz, p.init_rays, "huber"),
                                 "huber": (ptz_h, rays_h, "huber")}.items():
        *_, gp, gr, _c = orc._normal_blocks(a_, b_, p.u, p.v, frame, landmark, p.xy, seg, len(key), loss, 1.0)
        grads[name] = np.concatenate([np.abs(gp[1:]).max(0), np.abs(gr).max(0)])
        print(f"  |grad| {name}: {grads[name]}")
    out("config3_optimum.npz", n_pose=n, n_landmark=m, n_records=len(frame), frame_sum=int(frame.sum()),
        landmark_sum=int(landmark.sum()), xy_sum=float(p.xy.sum()), x0_sum=float(x0_full.sum()),
        r_ref_sample_idx=sample, r_ref_sample=r_ref[sample], r_ref_sumsq=float(np.sum(r_ref * r_ref)),
        ptz_tight=ptz_l, rays_tight=rays_l, tight_cost=info_l["cost"], iters=info_l["iterations"],
        last_step=info_l["last_step"], ptz_tight_huber=ptz_h, rays_tight_huber=rays_h,
        tight_cost_huber=info_h["cost"], iters_huber=info_h["iterations"], last_step_huber=info_h["last_step"],
        grad_x0=grads["x0"], grad_tight=grads["linear"], grad_x0_huber=grads["x0_huber"],
        grad_tight_huber=grads["huber"], ref_residual_time=t_ref, solve_time=[t_l, t_h])
    print(f"config3 total {time.time() - t_all:.0f}s")


# --------------------------------------------------------------------------------------------
# 8. relocalisation (relocalization.py): pose-only least_squares and relocalization_camera
# --------------------------------------------------------------------------------------------
def gen_reloc(seed):
    import relocalization as ref_rl  # REFERENCE module
    import scene_map as ref_sm
    import key_frame as ref_kf
    assert ref_rl.__file__.startswith(REF)
    u, v = 640.0, 360.0
    # (1) the refinement call of relocalization.py:186 on its own, reference residual (:22-40)
    rng = np.random.default_rng(seed)
    true = np.array([47.0, -9.0, 3100.0])
    px = np.stack([rng.uniform(40, 1240, 300), rng.uniform(40, 680, 300)], 1)
    rays = np.array([ref_tf.TransFunction.from_image_to_ray(u, v, true[2], true[0], true[1], x, y) for x, y in px])
    points = px + rng.normal(0, 0.5, px.shape)
    pose0 = true + np.array([0.8, -0.4, 60.0])
    r1 = least_squares(ref_rl._compute_residual, pose0, verbose=0, x_scale='jac', ftol=1e-4, method='trf',
                       args=(rays, points, u, v))
    rt = least_squares(ref_rl._compute_residual, pose0, x_scale='jac', ftol=1e-15, xtol=1e-15, gtol=1e-15,
                       method='trf', args=(rays, points, u, v))
    # (2) relocalization_camera end to end with the ray front-end monkeypatched in
    srays, cams, lost_init = synthetic.reloc_scene(seed)
    fe = synthetic.RayFrontEnd(srays, cams)
    ref_ip.detect_compute_sift = fe.detect
    ref_rl.match_sift_features = fe.match
    m = ref_sm.Map('sift')
    for k in range(4):
        pan, tilt, f = cams[k]
        m.keyframe_list.append(ref_kf.KeyFrame(k, k, np.zeros(3), np.eye(3), u, v, pan, tilt, f))
    reloc = ref_rl.relocalization_camera(m, 4, lost_init.copy())
    out("reloc.npz", u=u, v=v, rays=rays, points=points, pose0=pose0, x_ftol=r1.x, cost_ftol=r1.cost,
        njev_ftol=r1.njev, x_tight=rt.x, cost_tight=rt.cost, scene_seed=seed, scene_rays=srays, scene_cams=cams,
        lost_init=lost_init, reloc_pose=np.asarray(reloc, np.float64))

# --------------------------------------------------------------------------------------------
# 8f-2. incremental maps: Map.add_keyframe_with_ba (scene_map.py:53-117) and the sliding window of
# RandomForestMap.bundle_adjustment_processing (scene_map.py:198-244), whole sequences
# --------------------------------------------------------------------------------------------
def _map_state(step, kfs, rays, acc):
    for kf in kfs:
        pts = kf.feature_pts
        xy = np.array([p.pt for p in pts]).reshape(-1, 2) if isinstance(pts, list) else np.asarray(pts).reshape(-1, 2)
        acc["kf_step"].append(step)
        acc["kf_img"].append(int(kf.img))
        acc["kf_index"].append(int(kf.img_index))
        acc["kf_ptz"].append([kf.pan, kf.tilt, kf.f])
        acc["kf_nfeat"].append(len(xy))
        acc["feat_xy"].append(xy)
        acc["feat_lmk"].append(np.asarray(kf.landmark_index, np.int64).reshape(-1))
    acc["ray_n"].append(len(rays))
    acc["rays"].append(np.asarray(rays, np.float64).reshape(-1, 2))


def _pack_state(acc):
    return dict(kf_step=np.array(acc["kf_step"]), kf_img=np.array(acc["kf_img"]), kf_index=np.array(acc["kf_index"]),
                kf_ptz=np.array(acc["kf_ptz"]), kf_nfeat=np.array(acc["kf_nfeat"]),
                feat_xy=np.concatenate(acc["feat_xy"]), feat_lmk=np.concatenate(acc["feat_lmk"]),
                ray_n=np.array(acc["ray_n"]), rays=np.concatenate(acc["rays"]))


def gen_maps(seed):
    import scene_map as ref_sm
    import key_frame as ref_kf
    center, rot = np.array([0.0, -10.0, 5.0]), np.eye(3)
    ref_ba.draw_matches = lambda *a, **k: None
    # (1) growing map, every keyframe added with BA
    scene = synthetic.make_scene(6, 150, 54, 63, seed=seed)
    fe = FrontEnd(scene)
    calls = {"detect": 0, "match": 0}

    def det(*a, **k):
        calls["detect"] += 1
        return fe.detect(*a, **k)

    def mat(*a, **k):
        calls["match"] += 1
        return fe.match(*a, **k)
    ref_ip.detect_compute_sift, ref_ip.match_sift_features = det, mat
    random.seed(seed)
    ip = scene.init_ptz
    m = ref_sm.Map('sift')
    m.add_first_keyframe(ref_kf.KeyFrame(0, 100, center, rot, scene.u, scene.v, *ip[0]))
    acc = {k: [] for k in ("kf_step", "kf_img", "kf_index", "kf_ptz", "kf_nfeat", "feat_xy", "feat_lmk", "ray_n",
                           "rays")}
    t0 = time.time()
    for k in range(1, 6):
        m.add_keyframe_with_ba(ref_kf.KeyFrame(k, 100 + k, center, rot, scene.u, scene.v, *ip[k]), "/tmp")
        _map_state(k, m.keyframe_list, m.global_ray, acc)
    print(f"map: {time.time() - t0:.1f}s detect calls {calls['detect']} match calls {calls['match']}")
    out("map_incremental.npz", seed=seed, u=scene.u, v=scene.v, init_ptz=ip, ref_detect_calls=calls["detect"],
        ref_match_calls=calls["match"], **_pack_state(acc))
    # (2) sliding window of 10 over 12 keyframes
    scene = synthetic.make_scene(12, 160, 50, 66, seed=seed + 1)
    fe = FrontEnd(scene)
    ref_ip.detect_compute_sift, ref_ip.match_sift_features = fe.detect, fe.match
    random.seed(seed + 1)
    ip = scene.init_ptz
    rf = ref_sm.RandomForestMap()
    acc = {k: [] for k in acc}
    t0 = time.time()
    for k in range(12):
        rf.keyframe_list.append(ref_kf.KeyFrame(k, 200 + k, center, rot, scene.u, scene.v, *ip[k]))
        if len(rf.keyframe_list) > 1:
            rf.bundle_adjustment_processing()
        _map_state(k, rf.keyframe_list, np.zeros((0, 2)), acc)
    print(f"window: {time.time() - t0:.1f}s")
    out("map_window.npz", seed=seed + 1, u=scene.u, v=scene.v, init_ptz=ip, **_pack_state(acc))


# --------------------------------------------------------------------------------------------
# config 5: the streaming loop of demo_soccer.py:17-55 (PtzSlam.tracking / add_keyframe) on a synthetic
# 1080p stream, the front-end stand-in (synthetic.StreamFrontEnd) assigned to the reference's hooks
# --------------------------------------------------------------------------------------------
class _NumpyIndexCompat:
    """numpy as seen by the reference's ptz_slam module, with the one numpy-1.x behaviour it relies on:
    PtzSlam.remove_rays builds its covariance index list with np.append on a float array
    (ptz_slam.py:309-315) and passes it to np.delete, which numpy 1.11 (the README's pin) accepted and
    numpy 2 rejects.  Float index arrays are cast to int; everything else is numpy itself."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def delete(arr, obj, axis=None):
        o = np.asarray(obj)
        if o.dtype.kind == "f":
            o = o.astype(np.int64)
        return np.delete(arr, o, axis=axis)


def gen_stream(seed, n_frames):
    _sp = importlib.util.spec_from_file_location("demo_stream", os.path.join(REPO, "pan-tilt-zoom-slam_amd",
                                                                             "demo_stream.py"))
    demo_stream = importlib.util.module_from_spec(_sp)
    _sp.loader.exec_module(demo_stream)
    sc = synthetic.StreamScene(n_frames, seed=seed)
    fe = synthetic.StreamFrontEnd(sc).install(ref_ip)
    # ptz_slam binds the front-end names at import (`from image_process import *`, ptz_slam.py:17): rebind
    # them to image_process's own functions, which call the assigned hooks
    ref_slam.detect_compute_sift_array = ref_ip.detect_compute_sift_array
    ref_slam.matching_and_ransac = ref_ip.matching_and_ransac
    ref_ba.draw_matches = lambda *a, **k: None
    ref_slam.np = _NumpyIndexCompat()
    random.seed(seed)
    slam = ref_slam.PtzSlam()
    cam0 = ref_cam.PTZCamera((sc.u, sc.v), np.array([0.0, -16.0, 5.0]), np.eye(3))
    cam0.set_ptz(sc.cams[0].copy())
    cov_diag, cov_pose = [], []

    def on_frame(i, s):
        cov_diag.append(np.diag(s.state_cov).copy())
        cov_pose.append(s.state_cov[0:3, :].copy())

    t0 = time.time()
    rec = demo_stream.run_stream(slam, sc, n_frames, cam0, on_frame=on_frame)
    print(f"stream: {n_frames} frames in {time.time() - t0:.1f}s, keyframes {sum(rec['keyframe'])}, "
          f"rays {rec['n_rays'][-1]}")
    kfs = slam.keyframe_map.keyframe_list
    out("stream.npz", seed=seed, n_frames=n_frames, ptz=np.array(rec["ptz"]), velocity=np.array(rec["velocity"]),
        n_rays=np.array(rec["n_rays"]), n_kp=np.array(rec["n_kp"]), keyframe=np.array(rec["keyframe"]),
        lost=np.array(rec["lost"]), rays=np.asarray(slam.rays), cov_diag=np.concatenate(cov_diag),
        cov_diag_n=np.array([len(c) for c in cov_diag]), cov_pose=np.concatenate(cov_pose, axis=1),
        kf_index=np.array([k.img_index for k in kfs]), kf_ptz=np.array([[k.pan, k.tilt, k.f] for k in kfs]),
        global_ray=np.asarray(slam.keyframe_map.global_ray))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    rng = np.random.default_rng(1)
    todo = a.only.split(",") if a.only else ["proj", "ba", "graph", "ekf", "config2", "reloc", "maps", "stream"]
    if "proj" in todo:
        gen_projection(rng)
    if "ba" in todo:
        gen_ba("ba_4x60", 4, 60, 55, 61, seed=1)
        gen_ba("ba_6x120", 6, 120, 52, 62, seed=2)
        if not a.quick:
            gen_ba("ba_10x200", 10, 200, 50, 68, seed=1)
    if "graph" in todo:
        gen_graph(seed=3)
    if "ekf" in todo:
        gen_ekf(50, seed=4)
        gen_ekf(300, seed=5)
    if "reloc" in todo:
        gen_reloc(3)
    if "maps" in todo:
        gen_maps(21)
    if "config2" in todo:
        gen_config2()
    if "config2_ftol" in todo or "config2" in todo:
        gen_config2_ftol()
    if "config3" in todo:  # ~20 min; not in the default set
        gen_config3()
    if "stream" in todo:
        gen_stream(7, 30)


if __name__ == "__main__":
    main()
