"""
CPU ORACLE for the PTZ-SLAM bundle-adjustment / tracking hot path.

*** TEST INFRASTRUCTURE ONLY. ***  Only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` may import this module, and only as the checker / the
CPU baseline.  The product (`pan-tilt-zoom-slam_amd/`) never imports it and never falls
back to it.

What it is: a clean-room, vectorised NumPy (fp64) restatement of the reference's Python
hot path (all citations are into /root/reference/slam_system/):

  * `from_ray_to_image`      transformation.py:99-135   (literal atan closed form)
  * `from_image_to_ray`      transformation.py:137-175
  * `project_ray(s)`         ptz_camera.py:191-234      (matrix form, signed q2, displacement)
  * `back_project_to_ray(s)` ptz_camera.py:287-325
  * `overlap_pan_angle`      util.py:49-72
  * `get_overlap_index`      util.py:75-96
  * `build_landmark_index`   image_process.py:611-653   (first-seen landmark id rule)
  * `compute_residual`       bundle_adjustment.py:25-106 (pair order [dx_i,dy_i,dx_j,dy_j])
  * `init_x0`                bundle_adjustment.py:174-197 (last-writer-wins ray init)
  * `assemble_keyframes`     bundle_adjustment.py:216-248 (set() de-dup order)
  * `solve_scipy`            bundle_adjustment.py:200-202 (scipy trf, x_scale='jac', ftol=1e-4)
                             + `jac_sparsity` so it runs beyond toy sizes
  * `compute_h_jacobian`     ptz_slam.py:73-138          (central FD, vectorised)
  * `ekf_update`             ptz_slam.py:210-289          (incl. covariance write-back quirk)

Parity pinning: this restatement is checked against golden vectors produced by running the
reference itself in the build container (tests/golden/make_golden.py, fixtures
tests/golden/*.npz) — see tests/test_oracle_golden.py.
"""
import math

import numpy as np

D2R = math.pi / 180.0


# ----------------------------------------------------------------------------------------
# L1 camera model
# ----------------------------------------------------------------------------------------
def from_ray_to_image(u, v, f, c_p, c_t, p, t):
    """Vectorised restatement of TransFunction.from_ray_to_image (transformation.py:99-135).

    Keeps the reference's closed form literally (atan of a ratio, sqrt(tan^2+1)), which is
    what gives the `|q2|` semantics in y for rays behind the camera."""
    pan = np.radians(p)
    tilt = np.radians(t)
    cp = np.radians(c_p)
    ct = np.radians(c_t)
    tp = np.tan(pan)
    tt = np.tan(tilt)
    sec = np.sqrt(tp * tp + 1.0)
    num = tp * np.cos(cp) - np.sin(cp)
    den = tp * np.sin(cp) * np.cos(ct) + tt * sec * np.sin(ct) + np.cos(ct) * np.cos(cp)
    relative_pan = np.arctan(num / den)
    relative_tilt = np.arctan(-(tp * np.sin(ct) * np.sin(cp) - tt * sec * np.cos(ct)
                                + np.sin(ct) * np.cos(cp)) / np.sqrt(num * num + den * den))
    dx = f * np.tan(relative_pan)
    x = dx + u
    y = -np.sqrt(f * f + dx * dx) * np.tan(relative_tilt) + v
    return x, y


def _rot_tilt_pan(c_p, c_t):
    """R = R_tilt @ R_pan (ptz_camera.py:73-79) for arrays of angles in degrees -> [..., 3, 3]."""
    a = np.radians(np.asarray(c_p, dtype=np.float64))
    b = np.radians(np.asarray(c_t, dtype=np.float64))
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    z = np.zeros_like(ca)
    o = np.ones_like(ca)
    rt = np.stack([np.stack([o, z, z], -1), np.stack([z, cb, sb], -1), np.stack([z, -sb, cb], -1)], -2)
    rp = np.stack([np.stack([ca, z, -sa], -1), np.stack([z, o, z], -1), np.stack([sa, z, ca], -1)], -2)
    return rt @ rp


def from_image_to_ray(u, v, f, c_p, c_t, x, y):
    """Vectorised restatement of TransFunction.from_image_to_ray (transformation.py:137-175)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    theta_skim = np.arctan((x - u) / f)
    phi_skim = np.arctan((y - v) / (-f * np.sqrt(1.0 + ((x - u) / f) ** 2)))
    x3 = np.tan(theta_skim)
    y3 = -np.tan(phi_skim) * np.sqrt(np.tan(theta_skim) ** 2 + 1.0)
    r = _rot_tilt_pan(c_p, c_t)
    rinv = np.linalg.inv(r)
    vec = np.stack([x3, y3, np.ones_like(x3)], -1)
    out = np.einsum('...ij,...j->...i', rinv, vec)
    x3d, y3d, z3d = out[..., 0], out[..., 1], out[..., 2]
    theta = np.arctan(x3d / z3d)
    phi = np.arctan(-y3d / np.sqrt(x3d * x3d + z3d * z3d))
    return np.degrees(theta), np.degrees(phi)


def _displacement(f, disp):
    """PTZCamera.compute_dispalcement (ptz_camera.py:106-115)."""
    f = np.asarray(f, dtype=np.float64)
    w = np.zeros(6) if disp is None else np.asarray(disp, dtype=np.float64)
    return np.stack([w[0] + w[3] * f, w[1] + w[4] * f, w[2] + w[5] * f], -1)


def project_rays(u, v, f, pan, tilt, rays, displacement=None):
    """PTZCamera.project_ray over many rays (ptz_camera.py:191-210): matrix form, SIGNED q2.

    Returns [n, 2] image points (no visibility filtering)."""
    rays = np.asarray(rays, dtype=np.float64).reshape(-1, 2)
    th = np.radians(rays[:, 0])
    ph = np.radians(rays[:, 1])
    tth = np.tan(th)
    ray_p = np.stack([tth, -np.tan(ph) * np.sqrt(tth * tth + 1.0), np.ones_like(tth)], -1)
    r = _rot_tilt_pan(pan, tilt)
    d = _displacement(f, displacement)
    cam = ray_p @ r.T + d
    img = np.stack([f * cam[:, 0] + u * cam[:, 2], f * cam[:, 1] + v * cam[:, 2], cam[:, 2]], -1)
    return np.stack([img[:, 0] / img[:, 2], img[:, 1] / img[:, 2]], -1)


def project_rays_visible(u, v, f, pan, tilt, rays, height, width, displacement=None):
    """PTZCamera.project_rays with (height, width) (ptz_camera.py:212-234): strict 0<x<w, 0<y<h.
    Returns (points [k,2], index float [k])."""
    pts = project_rays(u, v, f, pan, tilt, rays, displacement)
    keep = (pts[:, 0] > 0) & (pts[:, 0] < width) & (pts[:, 1] > 0) & (pts[:, 1] < height)
    idx = np.flatnonzero(keep).astype(np.float64)
    return pts[keep], idx


def back_project_to_rays(u, v, f, pan, tilt, points, displacement=None):
    """PTZCamera.back_project_to_ray(s) (ptz_camera.py:287-325)."""
    points = np.asarray(points, dtype=np.float64).reshape(-1, 2)
    k = np.array([[f, 0, u], [0, f, v], [0, 0, 1.0]])
    kinv = np.linalg.inv(k)
    rinv = np.linalg.inv(_rot_tilt_pan(pan, tilt))
    d = _displacement(f, displacement)
    hom = np.concatenate([points, np.ones((len(points), 1))], 1)
    p = (hom @ kinv.T - d) @ rinv.T
    theta = np.arctan(p[:, 0] / p[:, 2])
    phi = np.arctan(-p[:, 1] / np.sqrt(p[:, 0] ** 2 + p[:, 2] ** 2))
    return np.stack([np.degrees(theta), np.degrees(phi)], -1)


# ----------------------------------------------------------------------------------------
# util
# ----------------------------------------------------------------------------------------
def overlap_pan_angle(fl_1, pan_1, fl_2, pan_2, im_width):
    """util.py:49-72 (vectorised; pan only, no wrap-around)."""
    w = im_width / 2.0
    d1 = np.degrees(np.arctan(w / np.asarray(fl_1, dtype=np.float64)))
    d2 = np.degrees(np.arctan(w / np.asarray(fl_2, dtype=np.float64)))
    a1 = np.maximum(pan_1 - d1, pan_2 - d2)
    a2 = np.minimum(pan_1 + d1, pan_2 + d2)
    return np.maximum(0.0, a2 - a1)


def get_overlap_index(index1, index2):
    """util.py:75-96: two-pointer merge of two (assumed sorted) arrays."""
    o1, o2 = [], []
    p1 = p2 = 0
    while p1 < len(index1) and p2 < len(index2):
        if index1[p1] == index2[p2]:
            o1.append(p1)
            o2.append(p2)
            p1 += 1
            p2 += 1
        elif index1[p1] < index2[p2]:
            p1 += 1
        else:
            p2 += 1
    return np.array(o1, dtype=np.int64), np.array(o2, dtype=np.int64)


# ----------------------------------------------------------------------------------------
# Matching-graph bookkeeping (image_process.py:611-653) — pure Python (bit-exact ids)
# ----------------------------------------------------------------------------------------
def build_landmark_index(n_frames, pair_list):
    """pair_list: ordered list of (i, j, src_idx list, dst_idx list) for i<j (already capped).
    Returns (src_pt_index, dst_pt_index, landmark_index) as N x N lists, n_landmark, n_warn."""
    maps = [dict() for _ in range(n_frames)]
    g = 0
    warn = 0
    for i, j, s, d in pair_list:
        for a, b in zip(s, d):
            ina = a in maps[i]
            inb = b in maps[j]
            if ina and inb:
                if maps[i][a] != maps[j][b]:
                    warn += 1
            elif ina:
                maps[j][b] = maps[i][a]
            elif inb:
                maps[i][a] = maps[j][b]
            else:
                maps[i][a] = g
                maps[j][b] = g
                g += 1
    src = [[[] for _ in range(n_frames)] for _ in range(n_frames)]
    dst = [[[] for _ in range(n_frames)] for _ in range(n_frames)]
    lmk = [[[] for _ in range(n_frames)] for _ in range(n_frames)]
    for i, j, s, d in pair_list:
        src[i][j] = list(s)
        dst[i][j] = list(d)
        lmk[i][j] = [maps[i][a] for a in s]
    return src, dst, lmk, g, warn


def flatten_matches(src_pt_index, dst_pt_index, landmark_index):
    """Flatten the N x N index lists in the reference's residual loop order
    (bundle_adjustment.py:67-73: i outer, j inner, matches in list order).
    Returns int64 arrays (i, j, kp1, kp2, landmark)."""
    n = len(src_pt_index)
    mi, mj, k1, k2, lm = [], [], [], [], []
    for i in range(n):
        for j in range(n):
            s = src_pt_index[i][j]
            if len(s) == 0:
                continue
            cnt = len(s)
            mi.append(np.full(cnt, i, np.int64))
            mj.append(np.full(cnt, j, np.int64))
            k1.append(np.asarray(s, np.int64))
            k2.append(np.asarray(dst_pt_index[i][j], np.int64))
            lm.append(np.asarray(landmark_index[i][j], np.int64))
    if not mi:
        e = np.zeros(0, np.int64)
        return e, e, e, e, e
    return tuple(np.concatenate(a) for a in (mi, mj, k1, k2, lm))


def pair_records(points, mi, mj, k1, k2, lm):
    """Pair-form observation records in residual order: record 2m = (i, kp1), 2m+1 = (j, kp2).
    Returns frame[int64 R], landmark[int64 R], xy[R, 2]."""
    n = len(mi)
    frame = np.empty(2 * n, np.int64)
    frame[0::2] = mi
    frame[1::2] = mj
    landmark = np.repeat(lm, 2)
    xy = np.empty((2 * n, 2))
    for f in np.unique(frame) if n else []:
        sel0 = np.flatnonzero(mi == f)
        sel1 = np.flatnonzero(mj == f)
        xy[2 * sel0] = points[f][k1[sel0]]
        xy[2 * sel1 + 1] = points[f][k2[sel1]]
    return frame, landmark, xy


# ----------------------------------------------------------------------------------------
# BA residual / init / assembly / solve
# ----------------------------------------------------------------------------------------
def compute_residual_records(x_full, n_pose, u, v, frame, landmark, xy):
    """Residual of pair-form records: [proj(frame, landmark) - xy] flattened, fp64."""
    ptz = x_full[:3 * n_pose].reshape(-1, 3)
    rays = x_full[3 * n_pose:].reshape(-1, 2)
    px, py = from_ray_to_image(u, v, ptz[frame, 2], ptz[frame, 0], ptz[frame, 1],
                               rays[landmark, 0], rays[landmark, 1])
    return np.stack([px - xy[:, 0], py - xy[:, 1]], -1).reshape(-1)


def compute_residual(x, n_pose, n_landmark, n_residual, keypoints, src_pt_index, dst_pt_index,
                     landmark_index, u, v, reference_pose):
    """Same signature/semantics as bundle_adjustment._compute_residual (bundle_adjustment.py:25-106)."""
    assert x.shape[0] == (n_pose - 1) * 3 + n_landmark * 2
    x0 = np.concatenate([np.asarray(reference_pose, np.float64), x])
    mi, mj, k1, k2, lm = flatten_matches(src_pt_index, dst_pt_index, landmark_index)
    frame, landmark, xy = pair_records(keypoints, mi, mj, k1, k2, lm)
    r = compute_residual_records(x0, n_pose, u, v, frame, landmark, xy)
    assert r.shape[0] == n_residual
    return r


def init_x0(initial_ptzs, n_landmark, points, mi, mj, k1, lm, u, v):
    """bundle_adjustment.py:174-194: poses from initial_ptzs, rays from from_image_to_ray of the
    src observation in frame i; the LAST match (in loop order) referencing a landmark wins."""
    n = len(initial_ptzs)
    x0 = np.zeros(3 * n + 2 * n_landmark)
    x0[:3 * n] = np.asarray(initial_ptzs, np.float64).reshape(-1)
    if len(lm):
        rev = len(lm) - 1 - np.unique(lm[::-1], return_index=True)[1]
        last = np.sort(rev)
        ii = mi[last]
        pts = np.stack([points[i][k] for i, k in zip(ii, k1[last])]) if len(last) else np.zeros((0, 2))
        ptz = np.asarray(initial_ptzs, np.float64)[ii]
        th, ph = from_image_to_ray(u, v, ptz[:, 2], ptz[:, 0], ptz[:, 1], pts[:, 0], pts[:, 1])
        lid = lm[last]
        x0[3 * n + 2 * lid] = th
        x0[3 * n + 2 * lid + 1] = ph
    return x0


def assemble_keyframe_pairs(n_frames, src_pt_index, dst_pt_index, landmark_index):
    """bundle_adjustment.py:221-245: per keyframe, (local, global) pairs from src and dst roles,
    de-duplicated through a Python set (its iteration order is the keyframe's feature order).
    Returns list of (local_index list, global_index int32 array)."""
    out = []
    for i in range(n_frames):
        pairs = []
        for j in range(n_frames):
            if len(src_pt_index[i][j]) == 0:
                continue
            for a, l in zip(src_pt_index[i][j], landmark_index[i][j]):
                pairs.append((int(a), int(l)))
        for j in range(n_frames):
            if len(dst_pt_index[j][i]) == 0:
                continue
            for b, l in zip(dst_pt_index[j][i], landmark_index[j][i]):
                pairs.append((int(b), int(l)))
        pairs = set(pairs)
        loc = [p[0] for p in pairs]
        glb = [p[1] for p in pairs]
        out.append((loc, np.array(glb, dtype=np.int32)))
    return out


def ba_jacobian_sparsity(n_pose, n_landmark, frame, landmark):
    """Sparsity of d r / d x (frame 0 fixed) for pair-form records (2 rows each)."""
    from scipy.sparse import coo_matrix
    R = len(frame)
    rows, cols = [], []
    rr = np.arange(R)
    for k in range(2):
        row = 2 * rr + k
        m = frame > 0
        for c in range(3):
            rows.append(row[m])
            cols.append(3 * (frame[m] - 1) + c)
        for c in range(2):
            rows.append(row)
            cols.append(3 * (n_pose - 1) + 2 * landmark + c)
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    return coo_matrix((np.ones(len(rows), np.int8), (rows, cols)),
                      shape=(2 * R, 3 * (n_pose - 1) + 2 * n_landmark)).tocsr()


def ba_jacobian(x, n_pose, n_landmark, u, v, ref_pose, frame, landmark):
    """Analytic sparse Jacobian of the pair-form residual, fp64."""
    from scipy.sparse import coo_matrix
    x0 = np.concatenate([np.asarray(ref_pose, np.float64), x])
    ptz = x0[:3 * n_pose].reshape(-1, 3)
    rays = x0[3 * n_pose:].reshape(-1, 2)
    J = record_jacobian(u, v, ptz[frame], rays[landmark])  # [R, 2, 5]
    R = len(frame)
    rows, cols, vals = [], [], []
    rr = np.arange(R)
    m = frame > 0
    for k in range(2):
        for c in range(3):
            rows.append(2 * rr[m] + k)
            cols.append(3 * (frame[m] - 1) + c)
            vals.append(J[m, k, c])
        for c in range(2):
            rows.append(2 * rr + k)
            cols.append(3 * (n_pose - 1) + 2 * landmark + c)
            vals.append(J[:, k, 3 + c])
    return coo_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(2 * R, 3 * (n_pose - 1) + 2 * n_landmark)).tocsr()


def record_jacobian(u, v, ptz, rays):
    """d(x,y)/d(pan, tilt, f, theta, phi) per record (|q2| in y). [R,2,5]."""
    a = np.radians(ptz[:, 0]); b = np.radians(ptz[:, 1]); f = ptz[:, 2]
    th = np.radians(rays[:, 0]); ph = np.radians(rays[:, 1])
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    tth, sth = np.tan(th), 1.0 / np.cos(th)
    tph, sph = np.tan(ph), 1.0 / np.cos(ph)
    p0 = tth
    p1 = -tph * sth
    w0 = ca * p0 - sa
    w2 = sa * p0 + ca
    q0 = w0
    q1 = cb * p1 + sb * w2
    q2 = -sb * p1 + cb * w2
    aq2 = np.abs(q2)
    sg = np.sign(q2)
    # d(x,y)/dq
    dx = np.stack([f / q2, np.zeros_like(f), -f * q0 / (q2 * q2)], -1)
    dy = np.stack([np.zeros_like(f), f / aq2, -f * q1 * sg / (q2 * q2)], -1)
    dq_pan = np.stack([-w2, sb * w0, cb * w0], -1) * D2R
    dq_tilt = np.stack([np.zeros_like(f), q2, -q1], -1) * D2R
    d0 = sth * sth
    d1 = -tph * sth * tth
    dq_th = np.stack([ca * d0, cb * d1 + sb * sa * d0, -sb * d1 + cb * sa * d0], -1) * D2R
    e1 = -sph * sph * sth
    dq_ph = np.stack([np.zeros_like(f), cb * e1, -sb * e1], -1) * D2R
    J = np.zeros((len(f), 2, 5))
    for c, dq in enumerate([dq_pan, dq_tilt]):
        J[:, 0, c] = np.sum(dx * dq, -1)
        J[:, 1, c] = np.sum(dy * dq, -1)
    J[:, 0, 2] = q0 / q2
    J[:, 1, 2] = q1 / aq2
    for c, dq in enumerate([dq_th, dq_ph]):
        J[:, 0, 3 + c] = np.sum(dx * dq, -1)
        J[:, 1, 3 + c] = np.sum(dy * dq, -1)
    return J


def solve_scipy(x0_free, n_pose, n_landmark, u, v, ref_pose, frame, landmark, xy,
                ftol=1e-4, xtol=1e-8, gtol=1e-8, analytic=False, loss='linear', f_scale=1.0,
                max_nfev=None, verbose=0):
    """bundle_adjustment.py:200-202 option set (method='trf', x_scale='jac', ftol=1e-4), with a
    `jac_sparsity` (FD, as the reference) or an analytic sparse Jacobian (tight goldens)."""
    from scipy.optimize import least_squares
    ref_pose = np.asarray(ref_pose, np.float64)

    def fun(x):
        x_full = np.concatenate([ref_pose, x])
        return compute_residual_records(x_full, n_pose, u, v, frame, landmark, xy)

    kw = dict(x_scale='jac', ftol=ftol, xtol=xtol, gtol=gtol, method='trf', verbose=verbose,
              loss=loss, f_scale=f_scale)
    if max_nfev is not None:
        kw['max_nfev'] = max_nfev
    if analytic:
        if len(x0_free) < 2000:  # scipy's 'exact' trust-region solver needs a dense Jacobian
            kw['jac'] = lambda x: ba_jacobian(x, n_pose, n_landmark, u, v, ref_pose, frame, landmark).toarray()
            kw['tr_solver'] = 'exact'
        else:
            kw['jac'] = lambda x: ba_jacobian(x, n_pose, n_landmark, u, v, ref_pose, frame, landmark)
            kw['tr_solver'] = 'lsmr'
    else:
        kw['jac_sparsity'] = ba_jacobian_sparsity(n_pose, n_landmark, frame, landmark)
    return least_squares(fun, x0_free, **kw)


def _loss_weights(r, loss, f_scale):
    """scipy least_squares convention (cost = 0.5 f^2 sum rho((r/f)^2) over SCALAR residuals): per residual
    0.5 f^2 rho(z), the gradient weight rho'(z) (d cost / d r = rho' r) and the curvature weight rho' + 2 rho'' z
    (d^2 cost / d r^2).  huber: rho = z inside the unit, 2 sqrt(z) - 1 beyond, rho' = 1 / sqrt(z) there and the
    curvature is 0 (the cost is linear in |r|); it is floored at 0.1 rho' so every 2x2 landmark block stays
    well conditioned -- the floor changes the convergence rate of the Newton iteration, not its fixed point (at 1.0
    this is IRLS; at 0.1 config 2 converges in 11 instead of ~45 steps from the linear-loss optimum)."""
    z = (r / f_scale) ** 2
    if loss == 'huber':
        rho = np.where(z <= 1.0, z, 2.0 * np.sqrt(z) - 1.0)
        w1 = np.where(z <= 1.0, 1.0, 1.0 / np.sqrt(np.maximum(z, 1.0)))
        w2 = np.where(z <= 1.0, 1.0, 0.3 * w1)
        return 0.5 * f_scale ** 2 * rho, w1, w2
    one = np.ones_like(r)
    return 0.5 * r * r, one, one


def ba_cost_chunked(ptz, rays, u, v, frame, landmark, xy, loss='linear', f_scale=1.0, chunk=2_000_000):
    """ba_cost with bounded host memory (headline-size record arrays)."""
    c = 0.0
    for a in range(0, len(frame), chunk):
        b = min(len(frame), a + chunk)
        fr, lm = frame[a:b], landmark[a:b]
        px, py = from_ray_to_image(u, v, ptz[fr, 2], ptz[fr, 0], ptz[fr, 1], rays[lm, 0], rays[lm, 1])
        r = np.stack([px - xy[a:b, 0], py - xy[a:b, 1]], -1)
        c += float(np.sum(_loss_weights(r, loss, f_scale)[0]))
    return c


def _normal_blocks(ptz, rays, u, v, frame, landmark, xy, seg, n_seg, loss, f_scale, chunk=2_000_000):
    """Gauss-Newton blocks of the (robust-weighted) pair-form cost, accumulated per record without forming J:
    U [n,3,3] (pose-pose, per frame), V [m,2,2] (ray-ray, per landmark), W [n_seg,3,2] (pose-ray, per unique
    (frame, landmark) segment), gradients g_pose [n,3], g_ray [m,2], cost.  Per record the 2x5 analytic Jacobian
    (record_jacobian) of the residual of bundle_adjustment.py:67-99."""
    n, m = len(ptz), len(rays)
    U = np.zeros((n, 9))
    V = np.zeros((m, 4))
    W = np.zeros((n_seg, 6))
    gp = np.zeros((n, 3))
    gr = np.zeros((m, 2))
    cost = 0.0
    for a in range(0, len(frame), chunk):
        b = min(len(frame), a + chunk)
        fr, lm, sg = frame[a:b], landmark[a:b], seg[a:b]
        px, py = from_ray_to_image(u, v, ptz[fr, 2], ptz[fr, 0], ptz[fr, 1], rays[lm, 0], rays[lm, 1])
        r = np.stack([px - xy[a:b, 0], py - xy[a:b, 1]], -1)
        rho, w1, w2 = _loss_weights(r, loss, f_scale)
        cost += float(np.sum(rho))
        J = record_jacobian(u, v, ptz[fr], rays[lm])
        Jw = J * w2[:, :, None]  # curvature-weighted rows (Hessian blocks)
        r = r * w1  # gradient: J^T (rho' r)
        for i in range(3):
            for j in range(3):
                U[:, 3 * i + j] += np.bincount(fr, np.einsum("rk,rk->r", Jw[:, :, i], J[:, :, j]), n)
            for j in range(2):
                W[:, 2 * i + j] += np.bincount(sg, np.einsum("rk,rk->r", Jw[:, :, i], J[:, :, 3 + j]), n_seg)
            gp[:, i] += np.bincount(fr, np.einsum("rk,rk->r", J[:, :, i], r), n)
        for i in range(2):
            for j in range(2):
                V[:, 2 * i + j] += np.bincount(lm, np.einsum("rk,rk->r", Jw[:, :, 3 + i], J[:, :, 3 + j]), m)
            gr[:, i] += np.bincount(lm, np.einsum("rk,rk->r", J[:, :, 3 + i], r), m)
    return U.reshape(n, 3, 3), V.reshape(m, 2, 2), W.reshape(n_seg, 3, 2), gp, gr, cost


def schur_tight_solve(ptz0, rays0, u, v, frame, landmark, xy, loss='linear', f_scale=1.0, n_fixed=1,
                      max_iter=100, tol=1e-11, log=None):
    """Tight optimum of the reference BA cost (bundle_adjustment.py:25-106 residual, :200-202 least squares with
    frame 0 as the fixed gauge, :197) at sizes where J cannot be materialised (headline: 29.2M x 41k): Levenberg-
    Marquardt with Marquardt scaling, then undamped Gauss-Newton (for huber with the loss's own curvature weights,
    _loss_weights) to a step of max |dx| < tol.  The landmarks are eliminated per 2x2 block (S = U - sum_l W_l V_l^-1 W_l^T as a sparse
    product, dense Cholesky of the reduced pose system).  The stationary point is the same one scipy's trf
    approaches; this is the parity target SURVEY §8c-4/5 prescribes (tight optimum of the reference residual).
    Returns (ptz [n,3], rays [m,2], info dict)."""
    import scipy.linalg as sla
    import scipy.sparse as sp
    ptz = np.array(ptz0, np.float64).copy()
    rays = np.array(rays0, np.float64).copy()
    n, m = len(ptz), len(rays)
    frame = np.asarray(frame, np.int64)
    landmark = np.asarray(landmark, np.int64)
    key, seg = np.unique(landmark * n + frame, return_inverse=True)
    seg = seg.astype(np.int64)
    n_seg = len(key)
    seg_lm, seg_fr = key // n, key % n
    rows = (3 * seg_fr[:, None, None] + np.arange(3)[None, :, None]).repeat(2, 2).reshape(-1)
    cols = (2 * seg_lm[:, None, None] + np.arange(2)[None, None, :]).repeat(3, 1).reshape(-1)
    free = np.arange(3 * n_fixed, 3 * n)
    lam, nu = None, 2.0
    hist = []
    it = 0
    undamped = False
    x_step = np.inf
    while it < max_iter:
        U, V, W, gp, gr, cost = _normal_blocks(ptz, rays, u, v, frame, landmark, xy, seg, n_seg, loss, f_scale)
        Wm = sp.csr_matrix((W.reshape(-1), (rows, cols)), shape=(3 * n, 2 * m))
        dU = np.einsum("nii->ni", U).reshape(-1)
        dV = np.einsum("mii->mi", V).reshape(-1)
        if lam is None:
            lam = 1e-3
        while True:
            lv = 0.0 if undamped else lam
            a_ = V[:, 0, 0] + lv * dV[0::2]
            b_ = V[:, 0, 1]
            c_ = V[:, 1, 1] + lv * dV[1::2]
            det = a_ * c_ - b_ * b_
            Vi = np.stack([c_ / det, -b_ / det, -b_ / det, a_ / det], -1).reshape(m, 2, 2)
            bi = np.repeat(np.arange(m), 4) * 2 + np.tile([0, 0, 1, 1], m)
            bj = np.repeat(np.arange(m), 4) * 2 + np.tile([0, 1, 0, 1], m)
            Vsp = sp.csr_matrix((Vi.reshape(-1), (bi, bj)), shape=(2 * m, 2 * m))
            Y = (Wm @ Vsp).tocsr()
            S = sp.block_diag(list(U), format="csr").toarray() - (Y @ Wm.T).toarray()
            S[np.diag_indices(3 * n)] += lv * dU
            rhs = -gp.reshape(-1) + Y @ gr.reshape(-1)
            Sf = S[np.ix_(free, free)]
            dp = np.zeros(3 * n)
            dp[free] = sla.cho_solve(sla.cho_factor(Sf, lower=True), rhs[free])
            dr = -np.einsum("mij,mj->mi", Vi, gr + (Wm.T @ dp).reshape(m, 2))
            ptz_t = ptz + dp.reshape(n, 3)
            rays_t = rays + dr
            cost_t = ba_cost_chunked(ptz_t, rays_t, u, v, frame, landmark, xy, loss, f_scale)
            x_step = max(np.abs(dp).max(), np.abs(dr).max())
            if cost_t <= cost or undamped:
                break
            lam *= nu
            nu *= 2.0
        it += 1
        hist.append((it, cost, cost_t, 0.0 if undamped else lam, x_step))
        if log:
            log(f"  it {it}: cost {cost:.10f} -> {cost_t:.10f} lambda {0.0 if undamped else lam:.3g} max|dx| {x_step:.3e}")
        ptz, rays = ptz_t, rays_t
        if undamped:
            if x_step < tol:
                break
        else:
            lam = max(lam / 3.0, 1e-12)
            nu = 2.0
            if x_step < 1e-6:
                undamped = True
    cost = ba_cost_chunked(ptz, rays, u, v, frame, landmark, xy, loss, f_scale)
    return ptz, rays, dict(cost=cost, iterations=it, last_step=float(x_step), history=np.array(hist),
                           n_segments=n_seg)


def ba_cost(x_full, n_pose, u, v, frame, landmark, xy, loss='linear', f_scale=1.0):
    """scipy cost convention: 0.5 * sum rho(r_i^2) over scalar residuals."""
    r = compute_residual_records(x_full, n_pose, u, v, frame, landmark, xy)
    z = (r / f_scale) ** 2
    if loss == 'huber':
        rho = np.where(z <= 1.0, z, 2.0 * np.sqrt(z) - 1.0)
        return 0.5 * f_scale ** 2 * float(np.sum(rho))
    return 0.5 * float(np.sum(r * r))


# ----------------------------------------------------------------------------------------
# EKF tracking (ptz_slam.py:73-289)
# ----------------------------------------------------------------------------------------
def compute_h_jacobian(u, v, pan, tilt, f, rays, displacement=None):
    """ptz_slam.py:73-138: central FD, d_angle = 0.001 deg, d_f = 0.1 px; H [2R, 3+2R]."""
    rays = np.asarray(rays, np.float64).reshape(-1, 2)
    n = len(rays)
    da, dfl = 0.001, 0.1
    H = np.zeros((2 * n, 3 + 2 * n))

    def P(pp, tt, ff, rr):
        return project_rays(u, v, ff, pp, tt, rr, displacement)

    cols = [
        (P(pan + da, tilt, f, rays) - P(pan - da, tilt, f, rays)) / (2 * da),
        (P(pan, tilt + da, f, rays) - P(pan, tilt - da, f, rays)) / (2 * da),
        (P(pan, tilt, f + dfl, rays) - P(pan, tilt, f - dfl, rays)) / (2 * dfl),
    ]
    for c in range(3):
        H[0::2, c] = cols[c][:, 0]
        H[1::2, c] = cols[c][:, 1]
    dth = np.array([da, 0.0])
    dph = np.array([0.0, da])
    jt = (P(pan, tilt, f, rays + dth) - P(pan, tilt, f, rays - dth)) / (2 * da)
    jp = (P(pan, tilt, f, rays + dph) - P(pan, tilt, f, rays - dph)) / (2 * da)
    idx = np.arange(n)
    H[2 * idx, 3 + 2 * idx] = jt[:, 0]
    H[2 * idx, 4 + 2 * idx] = jp[:, 0]
    H[2 * idx + 1, 3 + 2 * idx] = jt[:, 1]
    H[2 * idx + 1, 4 + 2 * idx] = jp[:, 1]
    return H


def ekf_update(state, observed_keypoints, observed_keypoint_index, height, width, observe_var=0.1):
    """ptz_slam.py:210-289 on a plain state dict: u, v, pan, tilt, f, displacement, rays [R,2],
    state_cov [3+2R]^2. Returns a new state dict (and velocity)."""
    s = {k: (np.array(v_, copy=True) if isinstance(v_, np.ndarray) else v_) for k, v_ in state.items()}
    u, v = s['u'], s['v']
    pred_pts, pred_idx = project_rays_visible(u, v, s['f'], s['pan'], s['tilt'], s['rays'], height, width,
                                              s.get('displacement'))
    o1, o2 = get_overlap_index(observed_keypoint_index, pred_idx)
    y = (np.asarray(observed_keypoints)[o1] - pred_pts[o2]).reshape(-1)
    matched = np.asarray(observed_keypoint_index)[o1].astype(np.int64)
    nr = len(matched)
    pr = np.concatenate([[0, 1, 2], np.stack([2 * matched + 3, 2 * matched + 4], -1).reshape(-1)]).astype(np.int64)
    P = s['state_cov'][np.ix_(pr, pr)]
    H = compute_h_jacobian(u, v, s['pan'], s['tilt'], s['f'], s['rays'][matched], s.get('displacement'))
    Sk = H @ P @ H.T + observe_var * np.eye(2 * nr)
    K = P @ H.T @ np.linalg.inv(Sk)
    ky = K @ y
    s['pan'] = s['pan'] + ky[0]
    s['tilt'] = s['tilt'] + ky[1]
    s['f'] = s['f'] + ky[2]
    s['velocity'] = ky[0:3].copy()
    s['rays'][matched] += ky[3:].reshape(-1, 2)
    Pu = (np.eye(3 + 2 * nr) - K @ H) @ P
    cov = s['state_cov']
    cov[0:3, 0:3] = Pu[0:3, 0:3]
    rows = 3 + 2 * matched
    cov[np.ix_(rows, rows)] = Pu[3::2, 3::2]
    cov[np.ix_(rows + 1, rows + 1)] = Pu[4::2, 4::2]
    return s


# --------------------------------------------------------------------------------------------
# relocalisation (relocalization.py)
# --------------------------------------------------------------------------------------------
def reloc_residual(pose, rays, points, u, v):
    """relocalization.py:22-40: [x_i - px_i, y_i - py_i] interleaved, from_ray_to_image projection."""
    rays = np.asarray(rays, np.float64).reshape(-1, 2)
    points = np.asarray(points, np.float64).reshape(-1, 2)
    n = len(rays)
    x, y = from_ray_to_image(u, v, np.full(n, pose[2]), np.full(n, pose[0]), np.full(n, pose[1]), rays[:, 0],
                             rays[:, 1])
    return np.stack([x - points[:, 0], y - points[:, 1]], 1).reshape(-1)


def refine_pose(pose0, rays, points, u, v, ftol=1e-4, xtol=1e-8, gtol=1e-8):
    """relocalization.py:186: least_squares(_compute_residual, pose, x_scale='jac', ftol=1e-4, 'trf')."""
    from scipy.optimize import least_squares
    res = least_squares(reloc_residual, np.asarray(pose0, np.float64), x_scale='jac', ftol=ftol, xtol=xtol,
                        gtol=gtol, method='trf', args=(rays, points, u, v))
    return res.x, res.cost


# --------------------------------------------------------------------------------------------
# feature front-end (image_process.py:178-234, 418-441): the GPU matcher / RANSAC's restatement
# --------------------------------------------------------------------------------------------
def knn2(des1, des2):
    """cv.BFMatcher().knnMatch(des1, des2, k=2) (image_process.py:191), L2: for each query the two nearest
    train rows, ties to the lower index.  Distances summed in fp64 (exact for SIFT's integer descriptors)."""
    a = np.asarray(des1, np.float64)
    b = np.asarray(des2, np.float64)
    d2 = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
    order = np.lexsort((np.broadcast_to(np.arange(len(b)), d2.shape), d2), axis=1)[:, :2]
    return order.astype(np.int32), np.sqrt(np.take_along_axis(d2, order, 1))


_M64 = (1 << 64) - 1


def _mix64(z):
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _ransac_draw(seed, h, k, attempt, n):
    z = _mix64((seed * 0x9E3779B97F4A7C15 + (h << 20) + (attempt << 4) + k + 1) & _M64)
    return z % n


def _ransac_sample(seed, h, n):
    s = []
    for k in range(4):
        att = 0
        while True:
            v = _ransac_draw(seed, h, k, att, n)
            att += 1
            if v not in s or att >= 64:
                break
        s.append(v)
    return s


def _solve8(M):
    """Gaussian elimination with partial pivoting on the 8x9 augmented system (the GPU's solve8)."""
    M = np.array(M, dtype=np.float64)
    for c in range(8):
        p = c + int(np.argmax(np.abs(M[c:, c])))
        if not np.abs(M[p, c]) > 1e-12:
            return None
        if p != c:
            M[[c, p]] = M[[p, c]]
        inv = 1.0 / M[c, c]
        for r in range(c + 1, 8):
            f = M[r, c] * inv
            M[r, c:] -= f * M[c, c:]
    x = np.zeros(8)
    for c in range(7, -1, -1):
        x[c] = (M[c, 8] - M[c, c + 1:8] @ x[c + 1:]) / M[c, c]
    return x


def _dlt_rows(x, y, u, v):
    return ([x, y, 1, 0, 0, 0, -u * x, -u * y, u], [0, 0, 0, x, y, 1, -v * x, -v * y, v])


def homography_ransac(p1, p2, threshold, n_hyp=2000, seed=0):
    """Restatement of ptz_homography_ransac (the cv.findHomography RANSAC call of image_process.py:433):
    counter-keyed 4-point samples, Hartley-normalised DLT, most inliers (then lowest index), linear
    least-squares refit on the inliers, final mask.  Returns (mask, H, count)."""
    p1 = np.asarray(p1, np.float64).reshape(-1, 2)
    p2 = np.asarray(p2, np.float64).reshape(-1, 2)
    n = len(p1)
    c1, c2 = p1.mean(0), p2.mean(0)
    s1 = np.sqrt(2.0) * n / np.sqrt(((p1 - c1) ** 2).sum(1)).sum()
    s2 = np.sqrt(2.0) * n / np.sqrt(((p2 - c2) ** 2).sum(1)).sum()
    q1, q2 = s1 * (p1 - c1), s2 * (p2 - c2)
    T1 = np.array([[s1, 0, -s1 * c1[0]], [0, s1, -s1 * c1[1]], [0, 0, 1]])
    T2i = np.array([[1 / s2, 0, c2[0]], [0, 1 / s2, c2[1]], [0, 0, 1]])

    def denorm(h):
        return T2i @ np.append(h, 1.0).reshape(3, 3) @ T1

    def err2(H):
        w = H[2, 0] * p1[:, 0] + H[2, 1] * p1[:, 1] + H[2, 2]
        px = (H[0, 0] * p1[:, 0] + H[0, 1] * p1[:, 1] + H[0, 2]) / w
        py = (H[1, 0] * p1[:, 0] + H[1, 1] * p1[:, 1] + H[1, 2]) / w
        return (px - p2[:, 0]) ** 2 + (py - p2[:, 1]) ** 2

    thr2 = threshold * threshold
    best, best_h, best_H = -1, -1, None
    for h in range(n_hyp):
        s = _ransac_sample(seed, h, n)
        rows = []
        for k in s:
            rows.extend(_dlt_rows(q1[k, 0], q1[k, 1], q2[k, 0], q2[k, 1]))
        x = _solve8(rows)
        if x is None:
            continue
        H = denorm(x)
        c = int((err2(H) < thr2).sum())
        if c > best:
            best, best_h, best_H = c, h, H
    if best_H is None:
        return np.zeros(n, bool), np.zeros((3, 3)), 0
    inl = err2(best_H) < thr2
    A = np.array([r for i in np.flatnonzero(inl) for r in _dlt_rows(q1[i, 0], q1[i, 1], q2[i, 0], q2[i, 1])])
    G = A.T @ A
    x = _solve8(np.concatenate([G[:8, :8], G[:8, 8:9]], 1))
    H = denorm(x) if x is not None else best_H
    mask = err2(H) < thr2
    return mask, H / H[2, 2], int(mask.sum())


# ---------------------------------------------------------------------------------------------
# pyramidal Lucas-Kanade (cv.calcOpticalFlowPyrLK(img, next_img, points, None, winSize=(31, 31)),
# optical_flow_matching, image_process.py:393-415).  OpenCV is not installed here, so this restates the
# algorithm ptz_lk_track implements (include/ptzba.h): parity of the GPU path is pinned to THIS restatement
# and to the known motion of synthetic images; agreement with cv2's own numbers is unpinned.
# ---------------------------------------------------------------------------------------------
def pyr_down(img):
    """cv.pyrDown: 5x5 binomial [1 4 6 4 1]^2 / 256 over a reflect-101 border, every second pixel."""
    h, w = img.shape
    P = np.pad(np.asarray(img, np.float64), 2, mode="reflect")
    k = np.array([1.0, 4.0, 6.0, 4.0, 1.0])
    dh, dw = (h + 1) // 2, (w + 1) // 2
    rows = sum(k[i] * P[i:i + 2 * dh:2, :] for i in range(5))
    return sum(k[j] * rows[:, j:j + 2 * dw:2] for j in range(5)) / 256.0


def scharr(img):
    """Scharr derivatives / 32 over a reflect-101 border: (gx, gy)."""
    P = np.pad(np.asarray(img, np.float64), 1, mode="reflect")
    h, w = img.shape
    S = lambda dy, dx: P[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
    gx = (3 * (S(-1, 1) - S(-1, -1)) + 10 * (S(0, 1) - S(0, -1)) + 3 * (S(1, 1) - S(1, -1))) / 32.0
    gy = (3 * (S(1, -1) - S(-1, -1)) + 10 * (S(1, 0) - S(-1, 0)) + 3 * (S(1, 1) - S(-1, 1))) / 32.0
    return gx, gy


def bilinear(img, x, y):
    """Bilinear sample with the coordinates clamped to the image (ptz_lk_track's sampler)."""
    h, w = img.shape
    x = np.clip(x, 0.0, w - 1.0)
    y = np.clip(y, 0.0, h - 1.0)
    x0 = np.minimum(x.astype(np.int64), max(w - 2, 0))
    y0 = np.minimum(y.astype(np.int64), max(h - 2, 0))
    x1 = np.minimum(x0 + 1, w - 1)
    y1 = np.minimum(y0 + 1, h - 1)
    ax, ay = x - x0, y - y0
    return (1 - ay) * ((1 - ax) * img[y0, x0] + ax * img[y0, x1]) + ay * ((1 - ax) * img[y1, x0] + ax * img[y1, x1])


def corner_min_eig(img):
    """cv.cornerMinEigenVal(img, blockSize=3, ksize=3) as goodFeaturesToTrack uses it (detect_harris_corner_grid,
    image_process.py:352-390; OpenCV's published algorithm, cv2 itself is not importable here): 3x3 Sobel sums
    scaled by 1/(4*3*255), products summed over a 3x3 block with reflect-101 borders (of the source for the
    derivatives, of the product image for the block), smaller eigenvalue (a+c) - sqrt((a-c)^2 + b^2) with
    a, c = half the summed squares.  float32, every operation rounded separately in the kernel's order.
    Returns (eig [h, w] float32, 3x3 local maxima with eig > 0 off the one-pixel border [h, w] bool)."""
    im = np.asarray(img, np.int32)
    h, w = im.shape

    def r101(i, n):
        i = np.abs(i)
        return np.where(i >= n, 2 * n - 2 - i, i) if n > 1 else np.zeros_like(i)
    ys, xs = np.arange(h), np.arange(w)
    scale = np.float32(1.0 / (4.0 * 3.0 * 255.0))
    # derivatives at every pixel (reflected source)
    xm, xp = r101(xs - 1, w), r101(xs + 1, w)
    ym, yp = r101(ys - 1, h), r101(ys + 1, h)
    gx = np.zeros((h, w), np.int64)
    gy = np.zeros((h, w), np.int64)
    for j, wj in ((-1, 1), (0, 2), (1, 1)):
        yy = r101(ys + j, h)
        xx = r101(xs + j, w)
        gx += wj * (im[yy][:, xp] - im[yy][:, xm])
        gy += wj * (im[yp][:, xx] - im[ym][:, xx])
    dx = gx.astype(np.float32) * scale
    dy = gy.astype(np.float32) * scale
    pa, pb, pc = dx * dx, dx * dy, dy * dy
    sa = np.zeros((h, w), np.float32)
    sb = np.zeros((h, w), np.float32)
    sc = np.zeros((h, w), np.float32)
    for by in (-1, 0, 1):
        cy = r101(ys + by, h)
        for bx in (-1, 0, 1):
            cx = r101(xs + bx, w)
            sa = sa + pa[cy][:, cx]
            sb = sb + pb[cy][:, cx]
            sc = sc + pc[cy][:, cx]
    a = sa * np.float32(0.5)
    c = sc * np.float32(0.5)
    d = (a - c) * (a - c) + sb * sb
    eig = (a + c) - np.sqrt(d)
    loc = np.zeros((h, w), bool)
    if h >= 3 and w >= 3:
        core = eig[1:-1, 1:-1]
        mx = np.full(core.shape, -np.inf, np.float32)
        for oy in (-1, 0, 1):
            for ox in (-1, 0, 1):
                mx = np.maximum(mx, eig[1 + oy:h - 1 + oy, 1 + ox:w - 1 + ox])
        loc[1:-1, 1:-1] = (core > 0) & (core >= mx)
    return eig.astype(np.float32), loc


def lk_track(img0, img1, pts, win=31, levels=4, max_iter=30, eps=0.01, min_eig=1e-4):
    """Restatement of ptz_lk_track: returns (next points [n, 2], status [n] uint8, err [n])."""
    pts = np.asarray(pts, np.float64).reshape(-1, 2)
    n = len(pts)
    I = [np.asarray(img0, np.float64)]
    J = [np.asarray(img1, np.float64)]
    for _ in range(1, levels):
        I.append(pyr_down(I[-1]))
        J.append(pyr_down(J[-1]))
    half = win // 2
    oy, ox = np.divmod(np.arange(win * win), win)
    ox = (ox - half).astype(np.float64)[None, :]
    oy = (oy - half).astype(np.float64)[None, :]
    g = np.zeros((n, 2))
    d = np.zeros((n, 2))
    ok = np.ones(n, bool)
    area = win * win
    for L in range(levels - 1, -1, -1):
        c = pts / (1 << L)
        X, Y = c[:, :1] + ox, c[:, 1:] + oy
        gxL, gyL = scharr(I[L])
        Iv, Ix, Iy = bilinear(I[L], X, Y), bilinear(gxL, X, Y), bilinear(gyL, X, Y)
        a, b, cc = (Ix * Ix).sum(1), (Ix * Iy).sum(1), (Iy * Iy).sum(1)
        det = a * cc - b * b
        mineig = 0.5 * (a + cc - np.sqrt(np.maximum((a - cc) ** 2 + 4 * b * b, 0.0))) / area
        ok &= (mineig >= min_eig) & (det > 0)
        d[:] = 0.0
        act = ok.copy()
        for _ in range(max_iter):
            if not act.any():
                break
            e = Iv - bilinear(J[L], X + (g[:, :1] + d[:, :1]), Y + (g[:, 1:] + d[:, 1:]))
            b0, b1 = (e * Ix).sum(1), (e * Iy).sum(1)
            with np.errstate(divide="ignore", invalid="ignore"):
                ddx = (cc * b0 - b * b1) / det
                ddy = (a * b1 - b * b0) / det
            d[act, 0] += ddx[act]
            d[act, 1] += ddy[act]
            act &= ~(ddx * ddx + ddy * ddy < eps * eps)
        if L > 0:
            g = np.where(ok[:, None], 2.0 * (g + d), g)
    nxt = pts + g + d
    h, w = I[0].shape
    err = np.abs(bilinear(I[0], pts[:, :1] + ox, pts[:, 1:] + oy) -
                 bilinear(J[0], nxt[:, :1] + ox, nxt[:, 1:] + oy)).sum(1) / area
    inside = (nxt[:, 0] >= 0) & (nxt[:, 1] >= 0) & (nxt[:, 0] <= w - 1) & (nxt[:, 1] <= h - 1)
    return nxt, (ok & inside).astype(np.uint8), np.where(ok, err, np.inf)


# ---------------------------------------------------------------------------------------------
# SIFT detection + description (cv.xfeatures2d.SIFT_create(nfeatures).detectAndCompute, detect_compute_sift,
# image_process.py:56-79).  OpenCV is not installed here: this restates Lowe's algorithm with OpenCV's
# defaults (3 layers per octave, contrast 0.04, edge 10, sigma 1.6, input blur 0.5, image doubled first) as
# ptz_sift implements it (include/ptzba.h); parity of the GPU path is pinned to THIS restatement and to
# repeatability under known homographies -- agreement with cv2's keypoints is unpinned.  Deliberate
# differences from OpenCV: exact atan2 instead of fastAtan2, keypoints ordered by (-response, y, x, angle)
# before the nfeatures cut.  The Gaussian pyramid is float32 with the GPU's operation order (bit-exact).
# ---------------------------------------------------------------------------------------------
SIFT_LAYERS, SIFT_CONTRAST, SIFT_EDGE, SIFT_SIGMA, SIFT_INIT_SIGMA = 3, 0.04, 10.0, 1.6, 0.5
SIFT_BORDER, SIFT_MAX_INTERP, SIFT_ORI_BINS, SIFT_ORI_PEAK = 5, 5, 36, 0.8
SIFT_D, SIFT_N = 4, 8


def sift_gauss_kernel(sigma):
    """Separable Gaussian weights (float32) as the host passes them to the GPU: size round(8 sigma + 1) | 1."""
    k = int(round(sigma * 8 + 1)) | 1
    r = k // 2
    w = [math.exp(-float(i - r) * float(i - r) / (2.0 * sigma * sigma)) for i in range(k)]  # libm exp, as the host
    s = 0.0
    for v in w:
        s += v
    return np.array([v / s for v in w], np.float64).astype(np.float32)


def _refl101(i, n):
    if n == 1:
        return np.zeros_like(i)
    p = 2 * n - 2
    i = np.abs(i) % p
    return np.where(i >= n, p - i, i)


def sift_blur(img, sigma):
    """Row then column pass, reflect-101 border, float32 accumulation k = 0..K-1 (mul, then add)."""
    w = sift_gauss_kernel(sigma)
    r = len(w) // 2
    h, wd = img.shape
    img = img.astype(np.float32)
    xs = np.arange(wd)
    acc = np.zeros_like(img)
    for k in range(len(w)):
        acc = acc + w[k] * img[:, _refl101(xs + k - r, wd)]
    ys = np.arange(h)
    out = np.zeros_like(acc)
    for k in range(len(w)):
        out = out + w[k] * acc[_refl101(ys + k - r, h), :]
    return out


def sift_upscale(img):
    """2x bilinear (OpenCV INTER_LINEAR centres: src = dst / 2 - 0.25), float32, clamped at the border."""
    h, w = img.shape
    img = img.astype(np.float32)

    def coords(n_src, n_dst):
        s = np.arange(n_dst, dtype=np.float32) * np.float32(0.5) - np.float32(0.25)
        i0 = np.floor(s).astype(np.int64)
        a = (s - i0).astype(np.float32)
        lo = i0 < 0
        a[lo] = 0
        i0[lo] = 0
        hi = i0 >= n_src - 1
        a[hi] = 0
        i0[hi] = n_src - 1
        return i0, np.minimum(i0 + 1, n_src - 1), a
    x0, x1, ax = coords(w, 2 * w)
    y0, y1, ay = coords(h, 2 * h)
    one = np.float32(1)
    top = (one - ax)[None, :] * img[y0][:, x0] + ax[None, :] * img[y0][:, x1]
    bot = (one - ax)[None, :] * img[y1][:, x0] + ax[None, :] * img[y1][:, x1]
    return (one - ay)[:, None] * top + ay[:, None] * bot


def sift_pyramid(img_u8):
    """Gaussian pyramid [octave][S + 3] and DoG pyramid [octave][S + 2] (float32)."""
    S = SIFT_LAYERS
    base = sift_upscale(np.asarray(img_u8, np.float32))
    base = sift_blur(base, np.sqrt(max(SIFT_SIGMA ** 2 - (2 * SIFT_INIT_SIGMA) ** 2, 0.01)))
    n_oct = int(round(np.log2(min(base.shape)) - 2))
    k = 2.0 ** (1.0 / S)
    sig = [SIFT_SIGMA]
    for i in range(1, S + 3):
        prev = (k ** (i - 1)) * SIFT_SIGMA
        sig.append(np.sqrt((prev * k) ** 2 - prev ** 2))
    gp, dp = [], []
    for o in range(n_oct):
        lv = [base if o == 0 else gp[o - 1][S][::2, ::2][:gp[o - 1][S].shape[0] // 2, :gp[o - 1][S].shape[1] // 2]]
        for i in range(1, S + 3):
            lv.append(sift_blur(lv[-1], sig[i]))
        gp.append(lv)
        dp.append([lv[i + 1] - lv[i] for i in range(S + 2)])
    return gp, dp


def _sift_refine(D, o, l, r, c):
    """adjustLocalExtrema in fp64; returns (l, r, c, xi, xr, xc, contr) or None."""
    S = SIFT_LAYERS
    sc = 1.0 / 255.0
    ds, s2, cs = sc * 0.5, sc, sc * 0.25
    rows, cols = D[0].shape
    for it in range(SIFT_MAX_INTERP):
        P, C, N = D[l - 1].astype(np.float64), D[l].astype(np.float64), D[l + 1].astype(np.float64)
        dD = np.array([(C[r, c + 1] - C[r, c - 1]) * ds, (C[r + 1, c] - C[r - 1, c]) * ds, (N[r, c] - P[r, c]) * ds])
        v2 = C[r, c] * 2
        dxx = (C[r, c + 1] + C[r, c - 1] - v2) * s2
        dyy = (C[r + 1, c] + C[r - 1, c] - v2) * s2
        dss = (N[r, c] + P[r, c] - v2) * s2
        dxy = (C[r + 1, c + 1] - C[r + 1, c - 1] - C[r - 1, c + 1] + C[r - 1, c - 1]) * cs
        dxs = (N[r, c + 1] - N[r, c - 1] - P[r, c + 1] + P[r, c - 1]) * cs
        dys = (N[r + 1, c] - N[r - 1, c] - P[r + 1, c] + P[r - 1, c]) * cs
        X = _solve3_sym(dxx, dxy, dxs, dyy, dys, dss, dD)
        if X is None:
            return None
        xc, xr, xi = -X[0], -X[1], -X[2]
        if abs(xi) < 0.5 and abs(xr) < 0.5 and abs(xc) < 0.5:
            break
        if abs(xi) > 1e6 or abs(xr) > 1e6 or abs(xc) > 1e6:
            return None
        c += int(round(xc))
        r += int(round(xr))
        l += int(round(xi))
        if l < 1 or l > S or c < SIFT_BORDER or c >= cols - SIFT_BORDER or r < SIFT_BORDER or r >= rows - SIFT_BORDER:
            return None
    else:
        return None
    P, C, N = D[l - 1].astype(np.float64), D[l].astype(np.float64), D[l + 1].astype(np.float64)
    dD = np.array([(C[r, c + 1] - C[r, c - 1]) * ds, (C[r + 1, c] - C[r - 1, c]) * ds, (N[r, c] - P[r, c]) * ds])
    t = dD[0] * xc + dD[1] * xr + dD[2] * xi
    contr = C[r, c] * sc + t * 0.5
    if abs(contr) * S < SIFT_CONTRAST:
        return None
    v2 = C[r, c] * 2
    dxx = (C[r, c + 1] + C[r, c - 1] - v2) * s2
    dyy = (C[r + 1, c] + C[r - 1, c] - v2) * s2
    dxy = (C[r + 1, c + 1] - C[r + 1, c - 1] - C[r - 1, c + 1] + C[r - 1, c - 1]) * cs
    tr, det = dxx + dyy, dxx * dyy - dxy * dxy
    if det <= 0 or tr * tr * SIFT_EDGE >= (SIFT_EDGE + 1) ** 2 * det:
        return None
    return l, r, c, xi, xr, xc, contr


def _solve3_sym(a, b, c, d, e, f, y):
    """[[a b c] [b d e] [c e f]] x = y by the explicit adjugate (the GPU's formula, fp64)."""
    A0, A1, A2 = d * f - e * e, c * e - b * f, b * e - c * d
    det = a * A0 + b * A1 + c * A2
    if det == 0:
        return None
    B1, B2, C2 = a * f - c * c, b * c - a * e, a * d - b * b
    inv = 1.0 / det
    return np.array([(A0 * y[0] + A1 * y[1] + A2 * y[2]) * inv, (A1 * y[0] + B1 * y[1] + B2 * y[2]) * inv,
                     (A2 * y[0] + B2 * y[1] + C2 * y[2]) * inv])


def _grad(img, r, c):
    return img[r, c + 1] - img[r, c - 1], img[r - 1, c] - img[r + 1, c]


def sift_detect(img_u8):
    """All keypoints: list of dicts (x, y, size, angle, response, octave o, layer l, r, c) in image coords."""
    S = SIFT_LAYERS
    gp, dp = sift_pyramid(img_u8)
    thr = np.floor(0.5 * SIFT_CONTRAST / S * 255)
    kps = []
    for o, D in enumerate(dp):
        rows, cols = D[0].shape
        if rows <= 2 * SIFT_BORDER or cols <= 2 * SIFT_BORDER:
            continue
        for l in range(1, S + 1):
            C = D[l]
            b = SIFT_BORDER
            v = C[b:rows - b, b:cols - b]
            nb = []
            for dl in (-1, 0, 1):
                for dy in (-1, 0, 1):
                    for dx in (-1, 0, 1):
                        if dl == 0 and dy == 0 and dx == 0:
                            continue
                        nb.append(D[l + dl][b + dy:rows - b + dy, b + dx:cols - b + dx])
            nb = np.stack(nb)
            ismax = (v > 0) & np.all(v[None] >= nb, axis=0)
            ismin = (v < 0) & np.all(v[None] <= nb, axis=0)
            cand = (np.abs(v) > thr) & (ismax | ismin)
            for r, c in zip(*np.nonzero(cand)):
                res = _sift_refine(D, o, l, int(r) + b, int(c) + b)
                if res is None:
                    continue
                L, R, Cc, xi, xr, xc, contr = res
                scale = 2.0 ** (o - 1)  # octave 0 is the doubled image
                size = SIFT_SIGMA * 2.0 ** ((L + xi) / S) * 2.0 ** o * 2 * 0.5
                x, y = (Cc + xc) * scale, (R + xr) * scale
                scl_oct = SIFT_SIGMA * 2.0 ** ((L + xi) / S)
                for ang in _sift_orientations(gp[o][L], R, Cc, scl_oct):
                    kps.append(dict(x=np.float32(x), y=np.float32(y), size=np.float32(size), angle=np.float32(ang),
                                    response=np.float32(abs(contr)), o=o, l=L, r=R, c=Cc,
                                    scl=float(np.float32(scl_oct))))
    return kps, gp


def _sift_orientations(img, r, c, scl):
    n = SIFT_ORI_BINS
    rad = int(round(3 * 1.5 * scl))
    sig = 1.5 * scl
    rows, cols = img.shape
    hist = np.zeros(n, np.float32)
    es = np.float32(-1.0 / (2.0 * sig * sig))
    for i in range(-rad, rad + 1):
        y = r + i
        if y <= 0 or y >= rows - 1:
            continue
        for j in range(-rad, rad + 1):
            x = c + j
            if x <= 0 or x >= cols - 1:
                continue
            dx, dy = _grad(img, y, x)
            w = np.float32(np.exp(np.float32(i * i + j * j) * es))
            ori = np.float32(np.degrees(np.arctan2(np.float64(dy), np.float64(dx))))
            if ori < 0:
                ori = np.float32(ori + 360)
            mag = np.float32(np.sqrt(np.float32(dx * dx + dy * dy)))
            bn = int(np.rint(np.float32(n / 360.0) * ori))
            bn = bn - n if bn >= n else (bn + n if bn < 0 else bn)
            hist[bn] = np.float32(hist[bn] + np.float32(w * mag))
    sm = np.zeros(n, np.float32)
    for i in range(n):
        sm[i] = (np.float32(hist[(i - 2) % n] + hist[(i + 2) % n]) * np.float32(1 / 16.) +
                 np.float32(hist[(i - 1) % n] + hist[(i + 1) % n]) * np.float32(4 / 16.) + hist[i] * np.float32(6 / 16.))
    omax = sm.max()
    out = []
    for j in range(n):
        lft, rgt = sm[(j - 1) % n], sm[(j + 1) % n]
        if sm[j] > lft and sm[j] > rgt and sm[j] >= omax * np.float32(SIFT_ORI_PEAK):
            bn = j + 0.5 * (lft - rgt) / (lft - 2 * sm[j] + rgt)
            bn = bn + n if bn < 0 else (bn - n if bn >= n else bn)
            ang = 360.0 - (360.0 / n) * bn
            out.append(0.0 if abs(ang - 360.0) < 1.2e-7 else ang)
    return out


def sift_descriptor(img, x, y, angle, scl):
    """calcSIFTDescriptor at octave coordinates (x, y), orientation `angle` (deg), scale scl: 128 values
    (integers 0..255 as float32)."""
    d, n = SIFT_D, SIFT_N
    ori = 360.0 - angle
    if abs(ori - 360.0) < 1.2e-7:
        ori = 0.0
    cos_t, sin_t = np.cos(np.radians(ori)), np.sin(np.radians(ori))
    hist_w = 3.0 * scl
    rad = int(round(hist_w * np.sqrt(2.0) * (d + 1) * 0.5))
    rows, cols = img.shape
    rad = min(rad, int(np.sqrt(float(rows) ** 2 + float(cols) ** 2)))
    cos_t /= hist_w
    sin_t /= hist_w
    px, py = int(round(x)), int(round(y))
    hist = np.zeros((d + 2, d + 2, n + 2), np.float64)
    es = -1.0 / (d * d * 0.5)
    bpr = n / 360.0
    for i in range(-rad, rad + 1):
        for j in range(-rad, rad + 1):
            c_rot = j * cos_t - i * sin_t
            r_rot = j * sin_t + i * cos_t
            rbin = r_rot + d / 2 - 0.5
            cbin = c_rot + d / 2 - 0.5
            r, c = py + i, px + j
            if not (-1 < rbin < d and -1 < cbin < d and 0 < r < rows - 1 and 0 < c < cols - 1):
                continue
            dx, dy = float(img[r, c + 1] - img[r, c - 1]), float(img[r - 1, c] - img[r + 1, c])
            w = np.exp((c_rot * c_rot + r_rot * r_rot) * es)
            o = np.degrees(np.arctan2(dy, dx))
            o = o + 360 if o < 0 else o
            mag = np.sqrt(dx * dx + dy * dy) * w
            obin = (o - ori) * bpr
            r0, c0, o0 = int(np.floor(rbin)), int(np.floor(cbin)), int(np.floor(obin))
            rb, cb, ob = rbin - r0, cbin - c0, obin - o0
            o0 = o0 + n if o0 < 0 else (o0 - n if o0 >= n else o0)
            for dr, wr in ((0, 1 - rb), (1, rb)):
                for dc, wc in ((0, 1 - cb), (1, cb)):
                    for do, wo in ((0, 1 - ob), (1, ob)):
                        hist[r0 + 1 + dr, c0 + 1 + dc, o0 + do] += mag * wr * wc * wo
    hist[:, :, 0] += hist[:, :, n]
    hist[:, :, 1] += hist[:, :, n + 1]
    v = hist[1:d + 1, 1:d + 1, :n].reshape(-1)
    thr = np.sqrt((v * v).sum()) * 0.2
    v = np.minimum(v, thr)
    nrm = 512.0 / max(np.sqrt((v * v).sum()), 1.2e-7)
    return np.clip(np.rint(v * nrm), 0, 255).astype(np.float32)


def sift_detect_compute(img_u8, nfeatures=0):
    """detectAndCompute: (keypoints [n, 4] = x, y, size, angle (image coords), response [n], descriptors [n, 128])
    ordered by (-response, y, x, angle), cut to nfeatures (> 0)."""
    kps, gp = sift_detect(img_u8)
    kps.sort(key=lambda k: (-float(k["response"]), float(k["y"]), float(k["x"]), float(k["angle"])))
    if nfeatures > 0:
        kps = kps[:nfeatures]
    kp = np.array([[k["x"], k["y"], k["size"], k["angle"]] for k in kps], np.float32).reshape(-1, 4)
    resp = np.array([k["response"] for k in kps], np.float32)
    des = np.zeros((len(kps), 128), np.float32)
    for i, k in enumerate(kps):
        s = 2.0 ** (k["o"] - 1)
        des[i] = sift_descriptor(gp[k["o"]][k["l"]], k["x"] / s, k["y"] / s, k["angle"], k["scl"])
    return kp, resp, des


def hamming_cross(des1, des2):
    """cv.BFMatcher(cv.NORM_HAMMING, crossCheck=True).match restated (image_process.py:249-250): mutual
    nearest neighbours by bit distance, ties to the lower index, in query order -> (query, train, distance)."""
    a = np.unpackbits(np.asarray(des1, np.uint8), axis=1).astype(np.int32)
    b = np.unpackbits(np.asarray(des2, np.uint8), axis=1).astype(np.int32)
    D = a @ (1 - b).T + (1 - a) @ b.T
    i12 = np.argmin(D, axis=1)
    i21 = np.argmin(D, axis=0)
    q = np.flatnonzero(i21[i12] == np.arange(len(a)))
    return q, i12[q], D[q, i12[q]]


# ----------------------------------------------------------------------------------------
# ORB / LATCH detection + description (image_process.py:105-155 -> cv.ORB_create(nfeatures), LATCH_create(64)),
# restated step for step as csrc/orb.hip implements OpenCV's published pipeline.  OpenCV's learned sampling
# tables are not available: both sides use the generated tables below, so descriptors are checked against
# this restatement only (parity unpinned against cv2).  Integer stages are exact; the float stages repeat the
# kernel's fp32 operation order.
# ----------------------------------------------------------------------------------------
ORB_LEVELS, ORB_EDGE, ORB_HALF, ORB_FAST_T = 8, 31, 15, 20
LATCH_HALF_SSD = 3
LATCH_BORDER = 48 // 2 + LATCH_HALF_SSD


def orb_tables():
    """(pattern [256, 4] int: x0, y0, x1, y1;  latch triplets [512, 6] int) -- csrc/orb.hip orb_tables."""
    pat = []
    k = 0
    base = (0x0B5EED * 0x9E3779B97F4A7C15) & _M64
    for _ in range(256 * 4):
        s = 0
        for _r in range(4):
            s += _mix64((base + k) & _M64) % 11 - 5
            k += 1
        pat.append(max(-13, min(13, s)))
    trip = []
    c = 0
    base = (0x1A7C4 * 0x9E3779B97F4A7C15) & _M64
    for _ in range(512 * 3):
        while True:
            x = _mix64((base + c) & _M64) % 39 - 19
            c += 1
            y = _mix64((base + c) & _M64) % 39 - 19
            c += 1
            if x * x + y * y <= 19 * 19:
                break
        trip += [x, y]
    return np.array(pat, np.int64).reshape(256, 4), np.array(trip, np.int64).reshape(512, 6)


def orb_umax():
    umax = [0] * (ORB_HALF + 2)
    vmax = int(math.floor(ORB_HALF * float(np.sqrt(np.float32(2))) / 2 + 1))
    vmin = int(math.ceil(ORB_HALF * float(np.sqrt(np.float32(2))) / 2))
    for v in range(vmax + 1):
        umax[v] = int(np.rint(math.sqrt(float(ORB_HALF * ORB_HALF - v * v))))
    v0 = 0
    for v in range(ORB_HALF, vmin - 1, -1):
        while umax[v0] == umax[v0 + 1]:
            v0 += 1
        umax[v] = v0
        v0 += 1
    return umax


def orb_scale(level):
    return np.float32(1.2 ** level)


def orb_level_counts(nfeatures):
    factor = 1.0 / 1.2
    nd = nfeatures * (1 - factor) / (1 - factor ** ORB_LEVELS)
    n, s = [], 0
    for _ in range(ORB_LEVELS - 1):
        n.append(int(np.rint(nd)))
        s += n[-1]
        nd *= factor
    n.append(max(nfeatures - s, 0))
    return n


def orb_resize(src, dw, dh):
    """8-bit bilinear resize, pixel-centre geometry, 11-bit weights (csrc/orb.hip k_orb_resize)."""
    sh, sw = src.shape

    def axis(n_dst, n_src):
        f = (np.arange(n_dst, dtype=np.float64) + 0.5) * (float(n_src) / float(n_dst)) - 0.5
        i0 = np.floor(f).astype(np.int64)
        a = np.rint((f - i0) * 2048.0).astype(np.int64)
        a = np.where(i0 < 0, 0, a)
        i0 = np.maximum(i0, 0)
        a = np.where(i0 >= n_src - 1, 0, a)
        i0 = np.minimum(i0, n_src - 1)
        return i0, np.minimum(i0 + 1, n_src - 1), a

    x0, x1, ax = axis(dw, sw)
    y0, y1, ay = axis(dh, sh)
    s = src.astype(np.int64)
    t = s[y0][:, x0] * (2048 - ax) + s[y0][:, x1] * ax
    b = s[y1][:, x0] * (2048 - ax) + s[y1][:, x1] * ax
    return ((t * (2048 - ay)[:, None] + b * ay[:, None] + (1 << 21)) >> 22).astype(np.uint8)


def orb_gauss_taps(n, sigma):
    w = [math.exp(-(i - (n - 1) * 0.5) ** 2 / (2 * sigma * sigma)) for i in range(n)]
    s = 0.0
    for v in w:
        s += v
    return np.array([v / s for v in w], np.float64).astype(np.float32)


def orb_blur(img, n, sigma):
    """Separable Gaussian, reflect-101, fp32 mul-then-add per tap, columns rounded half to even to 8 bits."""
    c = orb_gauss_taps(n, sigma)
    r = n // 2
    h, w = img.shape
    f = img.astype(np.float32)
    xs, ys = np.arange(w), np.arange(h)
    acc = np.zeros_like(f)
    for i in range(n):
        acc = acc + c[i] * f[:, _refl101(xs + i - r, w)]
    out = np.zeros_like(f)
    for i in range(n):
        out = out + c[i] * acc[_refl101(ys + i - r, h), :]
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


_FAST_DX = [0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1]
_FAST_DY = [3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3]


def fast_score(img, thr=ORB_FAST_T):
    """FAST-9 score image (0 = no corner): max over 9-arcs of the arc minimum of p - I (darker) or I - p
    (brighter), minus one, kept when >= thr; zero within 3 px of the border."""
    h, w = img.shape
    s = np.zeros((h, w), np.int64)
    if h < 7 or w < 7:
        return s
    im = img.astype(np.int64)
    p = im[3:h - 3, 3:w - 3]
    d = np.stack([p - im[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in zip(_FAST_DX, _FAST_DY)])
    a = np.full(p.shape, -1000, np.int64)
    b = np.full(p.shape, -1000, np.int64)
    for k in range(16):
        arc = d[[(k + m) % 16 for m in range(9)]]
        a = np.maximum(a, arc.min(0))
        b = np.maximum(b, -arc.max(0))
    t = np.maximum(a, b) - 1
    s[3:h - 3, 3:w - 3] = np.where(t >= thr, t, 0)
    return s


def fast_nms_points(score, edge=ORB_EDGE):
    """(x, y, score) of strict 3x3 maxima at least `edge` px inside the image."""
    h, w = score.shape
    if h <= 2 * edge or w <= 2 * edge:
        return np.zeros((0, 3), np.int64)
    c = score[edge:h - edge, edge:w - edge]
    keep = c > 0
    for j in (-1, 0, 1):
        for i in (-1, 0, 1):
            if i or j:
                keep &= c > score[edge + j:h - edge + j, edge + i:w - edge + i]
    ys, xs = np.nonzero(keep)
    return np.stack([xs + edge, ys + edge, c[ys, xs]], 1).astype(np.int64)


def orb_harris(img, xs, ys):
    """OpenCV HarrisResponses (block 7, k 0.04) at integer points: integer Sobel sums, fp32 response."""
    im = img.astype(np.int64)
    a = np.zeros(len(xs), np.int64)
    b = np.zeros(len(xs), np.int64)
    c = np.zeros(len(xs), np.int64)
    for v in range(-3, 4):
        for u in range(-3, 4):
            y, x = ys + v, xs + u
            ix = (im[y, x + 1] - im[y, x - 1]) * 2 + (im[y - 1, x + 1] - im[y - 1, x - 1]) + (im[y + 1, x + 1] - im[y + 1, x - 1])
            iy = (im[y + 1, x] - im[y - 1, x]) * 2 + (im[y + 1, x - 1] - im[y - 1, x - 1]) + (im[y + 1, x + 1] - im[y - 1, x + 1])
            a += ix * ix
            b += iy * iy
            c += ix * iy
    f32 = np.float32
    sc = f32(1.0) / (f32(28) * f32(255.0))
    s4 = sc * sc * sc * sc
    fa, fb, fc = a.astype(f32), b.astype(f32), c.astype(f32)
    k = f32(0.04)
    return ((fa * fb - fc * fc - k * (fa + fb) * (fa + fb)) * s4).astype(f32)


def _retain_best(rows, m, key):
    """KeyPointsFilter::retainBest: order (value desc, y, x), keep m plus every point tied with the m-th."""
    rows = sorted(rows, key=lambda r: (-key(r), r[1], r[0]))
    if len(rows) <= m:
        return rows
    if m <= 0:
        return []
    cut = key(rows[m - 1])
    e = m
    while e < len(rows) and key(rows[e]) >= cut:
        e += 1
    return rows[:e]


def orb_angle(img, x, y, umax):
    m01 = m10 = 0
    for v in range(-ORB_HALF, ORB_HALF + 1):
        d = umax[abs(v)]
        row = img[y + v, x - d:x + d + 1].astype(np.int64)
        u = np.arange(-d, d + 1)
        m10 += int((u * row).sum())
        m01 += int(v * row.sum())
    ang = math.atan2(float(m01), float(m10)) * (180.0 / 3.14159265358979323846)
    if ang < 0:
        ang += 360.0
    return ang


def orb_detect_compute(img, nfeatures=500, descriptor="orb"):
    """GPU ptz_orb restated: returns (kp [n, 6] float32 = x, y, size, angle, response, octave; descriptors
    [n, 32] (orb) or [n, 64] (latch) uint8), every tie at the per-level cuts kept, order (level, response
    desc, y, x)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    pat, trip = orb_tables()
    umax = orb_umax()
    per = orb_level_counts(nfeatures)
    levels = [img]
    for l in range(1, ORB_LEVELS):
        sc = orb_scale(l)
        lw = int(np.rint(np.float32(W) / sc))
        lh = int(np.rint(np.float32(H) / sc))
        levels.append(orb_resize(levels[-1], lw, lh))
    fin = []
    for l, im in enumerate(levels):
        pts = fast_nms_points(fast_score(im))
        rows = [(int(x), int(y), float(s)) for x, y, s in pts]
        rows = _retain_best(rows, 2 * per[l], key=lambda r: r[2])
        if not rows:
            continue
        xs = np.array([r[0] for r in rows])
        ys = np.array([r[1] for r in rows])
        hr = orb_harris(im, xs, ys)
        rows = [(r[0], r[1], float(v)) for r, v in zip(rows, hr)]
        rows = _retain_best(rows, per[l], key=lambda r: r[2])
        fin += [(x, y, l, r) for x, y, r in rows]
    if descriptor == "latch":
        keep = []
        for x, y, l, r in fin:
            sc = orb_scale(l)
            X, Y = np.float32(x) * sc, np.float32(y) * sc
            if X >= LATCH_BORDER and Y >= LATCH_BORDER and X < W - LATCH_BORDER and Y < H - LATCH_BORDER:
                keep.append((x, y, l, r))
        fin = keep
        lblur = orb_blur(img, 13, 2.0).astype(np.int64)
    else:
        blurs = [orb_blur(im, 7, 2.0).astype(np.int64) for im in levels]
    nb = 64 if descriptor == "latch" else 32
    kp = np.zeros((len(fin), 6), np.float32)
    des = np.zeros((len(fin), nb), np.uint8)
    for i, (x, y, l, r) in enumerate(fin):
        ang = orb_angle(levels[l], x, y, umax)
        rad = ang * (3.14159265358979323846 / 180.0)
        ca, sa = math.cos(rad), math.sin(rad)

        def rot(p, q):
            return int(np.rint(p * ca - q * sa)), int(np.rint(p * sa + q * ca))

        bits = []
        if descriptor == "latch":
            sc = orb_scale(l)
            cx, cy = int(np.rint(np.float32(x) * sc)), int(np.rint(np.float32(y) * sc))
            for t in trip:
                ax, ay = rot(t[0], t[1])
                bx, by = rot(t[2], t[3])
                ex, ey = rot(t[4], t[5])
                A = lblur[cy + ay - 3:cy + ay + 4, cx + ax - 3:cx + ax + 4]
                B = lblur[cy + by - 3:cy + by + 4, cx + bx - 3:cx + bx + 4]
                E = lblur[cy + ey - 3:cy + ey + 4, cx + ex - 3:cx + ex + 4]
                bits.append(int(((A - B) ** 2).sum()) < int(((A - E) ** 2).sum()))
        else:
            bl = blurs[l]
            for p in pat:
                x0, y0 = rot(p[0], p[1])
                x1, y1 = rot(p[2], p[3])
                bits.append(bl[y + y0, x + x0] < bl[y + y1, x + x1])
        bits = np.array(bits, np.uint8).reshape(nb, 8)
        des[i] = (bits << np.arange(8, dtype=np.uint8)).sum(1).astype(np.uint8)
        sc = orb_scale(l)
        kp[i] = [np.float32(x) * sc, np.float32(y) * sc, np.float32(31.0) * sc, np.float32(ang), np.float32(r), l]
    return kp, des
