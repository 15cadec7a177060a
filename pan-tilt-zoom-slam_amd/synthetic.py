"""
Synthetic PTZ keyframe x ray-landmark problems (SURVEY §8d "Synthetic inputs").

The reference feeds BA from SIFT detection + matching on real images (image_process.py:509-667);
neither the images nor OpenCV exist here, so this module generates the reference's own data
format directly: per-frame keypoint arrays, per-pair match index lists, and from them the
pair-form observation records that `bundle_adjustment._compute_residual`
(bundle_adjustment.py:25-106) iterates over.

Spec:
  camera u, v = 640, 360, image 1280 x 720; keyframe pans linspace(lo, hi, N);
  tilt ~ U[-12, -4] deg; f ~ U[2500, 3500] px;
  rays theta ~ U[lo-14, hi+14], phi ~ U[-19, 3];
  visibility 0<x<1280, 0<y<720, q2>0;
  pairs i<j with overlap_pan_angle > 5 and > 20 shared rays; cap 200 per pair (seeded permutation);
  keypoint noise N(0, 0.5 px); initial poses: frame 0 exact, others + N(0, [0.5, 0.2, 40]);
  initial rays from from_image_to_ray of the src observation, last writer wins.

Everything here is host-side problem *construction* (numpy): it is the stand-in for the
camera + feature front-end, not part of the solve.  The solve runs in libptzba.so.
"""
import math
from dataclasses import dataclass, field

import numpy as np

U0, V0 = 640.0, 360.0
WIDTH, HEIGHT = 1280, 720

CONFIGS = {
    # name: (n_kf, n_rays, pan_lo, pan_hi, tilt_rows)
    "config1": (10, 200, 50.0, 68.0, None),
    "config2": (50, 2000, 30.0, 70.0, None),
    "config3": (500, 20000, -60.0, 60.0, None),
    "config4": (5000, 200000, -60.0, 60.0, tuple(range(-65, 26, 10))),
}


def _project(u, v, f, pan, tilt, theta, phi):
    """Closed-form BA projection (q form): x = u + f q0/q2, y = v + f q1/|q2|.
    Broadcasting over arrays. Returns x, y, q2."""
    a = np.radians(pan); b = np.radians(tilt)
    th = np.radians(theta); ph = np.radians(phi)
    p0 = np.tan(th)
    p1 = -np.tan(ph) * np.sqrt(p0 * p0 + 1.0)  # sqrt(tan^2+1), not sec: ptz_camera.py:205 semantics
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    w0 = ca * p0 - sa
    w2 = sa * p0 + ca
    q1 = cb * p1 + sb * w2
    q2 = -sb * p1 + cb * w2
    return u + f * w0 / q2, v + f * q1 / np.abs(q2), q2


def image_to_ray(u, v, f, pan, tilt, x, y):
    """Back-projection (ray init rule of bundle_adjustment.py:193), vectorised closed form.
    Equivalent to TransFunction.from_image_to_ray (transformation.py:137-175)."""
    a = np.radians(pan); b = np.radians(tilt)
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    c0 = (x - u) / f
    c1 = (y - v) / f
    # camera ray c = [c0, c1, 1]; world direction d = R^T c, R = R_x(b) R_y(a)
    # R_x^T c:
    e0 = c0
    e1 = cb * c1 - sb
    e2 = sb * c1 + cb
    # R_y^T e:
    d0 = ca * e0 + sa * e2
    d1 = e1
    d2 = -sa * e0 + ca * e2
    theta = np.degrees(np.arctan(d0 / d2))
    phi = np.degrees(np.arctan(-d1 / np.sqrt(d0 * d0 + d2 * d2)))
    return theta, phi


def overlap_pan_angle(fl_1, pan_1, fl_2, pan_2, im_width):
    """util.py:49-72, vectorised."""
    w = im_width / 2.0
    d1 = np.degrees(np.arctan(w / np.asarray(fl_1, dtype=np.float64)))
    d2 = np.degrees(np.arctan(w / np.asarray(fl_2, dtype=np.float64)))
    a1 = np.maximum(pan_1 - d1, pan_2 - d2)
    a2 = np.minimum(pan_1 + d1, pan_2 + d2)
    return np.maximum(0.0, a2 - a1)


@dataclass
class Scene:
    """Ground-truth scene + per-frame keypoints (the 'detector output')."""
    gt_ptz: np.ndarray            # [N, 3] pan, tilt, f
    init_ptz: np.ndarray          # [N, 3] noisy initial poses (frame 0 exact)
    gt_rays: np.ndarray           # [M, 2] theta, phi (deg)
    kp_xy: list                   # N arrays [K_i, 2] noisy keypoints (fp64)
    kp_ray: list                  # N arrays [K_i] generator ray id per keypoint
    u: float = U0
    v: float = V0


@dataclass
class Problem:
    """Pair-form BA problem in the reference's residual order (bundle_adjustment.py:67-99)."""
    n_pose: int
    n_landmark: int
    frame: np.ndarray             # [R] int32 record frame      (record 2m = src, 2m+1 = dst of match m)
    landmark: np.ndarray          # [R] int32 record landmark id (first-seen rule, image_process.py:611-639)
    xy: np.ndarray                # [R, 2] fp64 observation
    init_ptz: np.ndarray          # [N, 3]
    init_rays: np.ndarray         # [M, 2] last-writer-wins init
    gt_ptz: np.ndarray            # [N, 3]
    gt_rays: np.ndarray           # [M, 2] ground truth for the relabelled landmarks
    u: float = U0
    v: float = V0
    n_pairs: int = 0
    meta: dict = field(default_factory=dict)

    @property
    def n_match(self):
        return len(self.frame) // 2


def _theta_window(f, pan, tilt, width=WIDTH, height=HEIGHT, u=U0, v=V0):
    """Conservative [lo, hi] (deg) of the ray azimuths theta a camera can see: a pixel ray
    c = [c0, c1, 1] has theta - pan = atan(c0 / (cos(tilt) + sin(tilt) c1)) while that denominator is
    positive, so |theta - pan| <= atan(max|c0| / min(cos + sin c1)).  None when the image reaches the
    horizon of the tilted frame (no bound: test every ray)."""
    b = math.radians(tilt)
    c0 = max(u, width - u) / f
    c1 = max(v, height - v) / f
    den = math.cos(b) - abs(math.sin(b)) * c1
    if den <= 1e-3:
        return None
    half = math.degrees(math.atan(c0 / den)) + 0.5
    return pan - half, pan + half


def make_scene(n_kf, n_rays, pan_lo, pan_hi, seed=0, tilt_rows=None, noise=0.5,
               init_sigma=(0.5, 0.2, 40.0)):
    rng = np.random.default_rng(seed)
    if tilt_rows is None:
        pans = np.linspace(pan_lo, pan_hi, n_kf)
        tilts = rng.uniform(-12.0, -4.0, n_kf)
        phi_lo, phi_hi = -19.0, 3.0
    else:
        # config 4: rows of keyframes at several tilts; a camera at tilt t sees elevations phi ~ t +- 7
        # (config 3: tilt U[-12, -4], phi U[-19, 3]), so phi spans [min row - 7, max row + 7]
        rows = np.asarray(tilt_rows, np.float64)
        per = n_kf // len(rows)
        pans = np.tile(np.linspace(pan_lo, pan_hi, per), len(rows))
        tilts = np.repeat(rows, per) + rng.uniform(-1.0, 1.0, per * len(rows))
        phi_lo, phi_hi = max(rows.min() - 7.0, -80.0), min(rows.max() + 7.0, 80.0)
    fs = rng.uniform(2500.0, 3500.0, len(pans))
    gt_ptz = np.stack([pans, tilts, fs], 1)
    theta = rng.uniform(pan_lo - 14.0, pan_hi + 14.0, n_rays)
    phi = rng.uniform(phi_lo, phi_hi, n_rays)
    gt_rays = np.stack([theta, phi], 1)
    # rays sorted by azimuth: a frame projects only the rays inside its theta window (same visible ids,
    # in the same ascending order, as projecting every ray)
    by_theta = np.argsort(theta, kind="stable")
    theta_sorted = theta[by_theta]
    kp_xy, kp_ray = [], []
    for i in range(len(pans)):
        win = _theta_window(fs[i], pans[i], tilts[i])
        if win is None:
            cand = np.arange(n_rays)
        else:
            lo, hi = np.searchsorted(theta_sorted, win[0]), np.searchsorted(theta_sorted, win[1], side="right")
            cand = np.sort(by_theta[lo:hi])
        x, y, q2 = _project(U0, V0, fs[i], pans[i], tilts[i], theta[cand], phi[cand])
        vis = (q2 > 0) & (x > 0) & (x < WIDTH) & (y > 0) & (y < HEIGHT)
        ids = cand[vis]
        pts = np.stack([x[vis], y[vis]], 1) + rng.normal(0.0, noise, (len(ids), 2))
        kp_xy.append(pts)
        kp_ray.append(ids.astype(np.int64))
    init = gt_ptz.copy()
    init[1:] += rng.normal(0.0, 1.0, (len(pans) - 1, 3)) * np.asarray(init_sigma)
    return Scene(gt_ptz=gt_ptz, init_ptz=init, gt_rays=gt_rays, kp_xy=kp_xy, kp_ray=kp_ray)


def scene_pairs(scene, seed=0, min_match=20, max_match=200, overlap_deg=5.0, cap=True):
    """Ordered list of (i, j, idx_i list, idx_j list) for i<j: overlap mask on the *initial*
    poses (bundle_adjustment.py:135-144), shared keypoints = ground-truth matches, keep if
    > min_match (image_process.py:590), cap to max_match with a seeded permutation.

    Candidate pairs come from the shared-ray counts of the frame x ray incidence matrix (one sparse
    product); the permutations are drawn for the kept pairs in (i, j) order, as a double loop would."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed + 7919)
    n = len(scene.kp_xy)
    ip = scene.init_ptz
    n_rays = len(scene.gt_rays)
    lens = np.array([len(r) for r in scene.kp_ray], np.int64)
    inc = sp.csr_matrix((np.ones(int(lens.sum()), np.int32),
                         (np.repeat(np.arange(n), lens), np.concatenate(scene.kp_ray) if n else [])),
                        shape=(n, n_rays))
    shared_cnt = sp.triu(inc @ inc.T, k=1).tocoo()
    keep = shared_cnt.data > min_match
    ci, cj = shared_cnt.row[keep].astype(np.int64), shared_cnt.col[keep].astype(np.int64)
    ov = overlap_pan_angle(ip[ci, 2], ip[ci, 0], ip[cj, 2], ip[cj, 0], WIDTH)
    sel = ov > overlap_deg
    ci, cj = ci[sel], cj[sel]
    order = np.lexsort((cj, ci))
    out = []
    for i, j in zip(ci[order].tolist(), cj[order].tolist()):
        ri, rj = scene.kp_ray[i], scene.kp_ray[j]          # ascending ray ids
        pos = np.searchsorted(rj, ri)
        hit = rj[np.minimum(pos, len(rj) - 1)] == ri
        a = np.flatnonzero(hit)                           # positions in frame i (ascending ray id)
        b = pos[hit]                                      # positions of the same rays in frame j
        if cap and len(a) > max_match:
            perm = rng.permutation(len(a))[:max_match]
            a, b = a[perm], b[perm]
        out.append((i, j, a, b))
    return out


def problem_from_pairs(scene, pairs):
    """Build the pair-form problem from ordered pair lists, reproducing the reference's
    first-seen landmark ids (image_process.py:611-639) and last-writer ray init
    (bundle_adjustment.py:184-194).  Ground-truth matches are consistent, so a keypoint's
    landmark is its generator ray and the first-seen rule reduces to first-occurrence order."""
    n = len(scene.kp_xy)
    if not pairs:
        raise ValueError("no matched pairs")
    mi = np.concatenate([np.full(len(a), i, np.int64) for i, j, a, b in pairs])
    mj = np.concatenate([np.full(len(a), j, np.int64) for i, j, a, b in pairs])
    k1 = np.concatenate([np.asarray(a, np.int64) for i, j, a, b in pairs])
    k2 = np.concatenate([np.asarray(b, np.int64) for i, j, a, b in pairs])
    # generator ray of every match (src keypoint's ray)
    kp_ray_flat = np.concatenate(scene.kp_ray)
    kp_off = np.concatenate([[0], np.cumsum([len(r) for r in scene.kp_ray])])
    kp_xy_flat = np.concatenate(scene.kp_xy)
    ray = kp_ray_flat[kp_off[mi] + k1]
    # first-seen relabelling
    uniq, first = np.unique(ray, return_index=True)
    order = np.argsort(first, kind="stable")
    relabel = np.full(len(scene.gt_rays), -1, np.int64)
    relabel[uniq[order]] = np.arange(len(uniq))
    lm = relabel[ray]
    m = len(uniq)
    R = 2 * len(mi)
    frame = np.empty(R, np.int32)
    frame[0::2] = mi
    frame[1::2] = mj
    landmark = np.repeat(lm, 2).astype(np.int32)
    xy = np.empty((R, 2))
    xy[0::2] = kp_xy_flat[kp_off[mi] + k1]
    xy[1::2] = kp_xy_flat[kp_off[mj] + k2]
    # last-writer-wins ray init from the src observation in frame i with the INITIAL pose
    # landmark ids are exactly 0..m-1, so unique() of the reversed array lists them in order
    src = len(lm) - 1 - np.unique(lm[::-1], return_index=True)[1]
    ip = scene.init_ptz[mi[src]]
    pts = kp_xy_flat[kp_off[mi[src]] + k1[src]]
    th, ph = image_to_ray(scene.u, scene.v, ip[:, 2], ip[:, 0], ip[:, 1], pts[:, 0], pts[:, 1])
    init_rays = np.stack([th, ph], 1)
    gt_rays = scene.gt_rays[uniq[order]]
    return Problem(n_pose=n, n_landmark=m, frame=frame, landmark=landmark, xy=xy,
                   init_ptz=scene.init_ptz.copy(), init_rays=init_rays, gt_ptz=scene.gt_ptz.copy(),
                   gt_rays=gt_rays, u=scene.u, v=scene.v, n_pairs=len(pairs),
                   meta=dict(match_i=mi, match_j=mj, kp1=k1, kp2=k2))


def _synth_lib():
    import ctypes
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libptzsynth.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: build it with `make -C pan-tilt-zoom-slam_amd/csrc`")
    L = ctypes.CDLL(path)
    L.ptzsynth_grid_new.restype = ctypes.c_void_p
    L.ptzsynth_grid_new.argtypes = [ctypes.c_void_p]
    L.ptzsynth_counts.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.ptzsynth_fetch.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 7
    L.ptzsynth_free.argtypes = [ctypes.c_void_p]
    return L


def make_grid_problem(n_kf, n_rays, lo, hi, rows, seed=0, threads=None, noise=0.5, init_sigma=(0.5, 0.2, 40.0),
                      min_match=20, max_match=200, overlap_deg=5.0):
    """Multi-row keyframe grid (config 4) from the threaded native generator (csrc/synth.cpp): same spec
    as make_scene/scene_pairs/problem_from_pairs with row-major frames, counter-based random streams."""
    import ctypes
    import os

    class Params(ctypes.Structure):
        _fields_ = [("n_kf", ctypes.c_int32), ("n_rays", ctypes.c_int32), ("n_rows", ctypes.c_int32),
                    ("threads", ctypes.c_int32), ("pan_lo", ctypes.c_double), ("pan_hi", ctypes.c_double),
                    ("rows", ctypes.c_void_p), ("seed", ctypes.c_uint64), ("noise", ctypes.c_double),
                    ("sig_pan", ctypes.c_double), ("sig_tilt", ctypes.c_double), ("sig_f", ctypes.c_double),
                    ("min_match", ctypes.c_int32), ("max_match", ctypes.c_int32), ("overlap_deg", ctypes.c_double)]

    L = _synth_lib()
    rows_a = np.ascontiguousarray(rows, np.float64)
    if threads is None:
        threads = min(16, len(os.sched_getaffinity(0)))
    p = Params(int(n_kf), int(n_rays), len(rows_a), int(threads), float(lo), float(hi), rows_a.ctypes.data,
               int(seed), float(noise), *[float(s) for s in init_sigma], int(min_match), int(max_match),
               float(overlap_deg))
    h = L.ptzsynth_grid_new(ctypes.byref(p))
    if not h:
        raise ValueError("bad grid parameters")
    try:
        c = np.zeros(4, np.int64)
        L.ptzsynth_counts(h, c.ctypes.data)
        n, m, r, npairs = (int(x) for x in c)
        frame = np.empty(r, np.int32)
        landmark = np.empty(r, np.int32)
        xy = np.empty((r, 2))
        init_ptz, gt_ptz = np.empty((n, 3)), np.empty((n, 3))
        init_rays, gt_rays = np.empty((m, 2)), np.empty((m, 2))
        L.ptzsynth_fetch(h, frame.ctypes.data, landmark.ctypes.data, xy.ctypes.data, init_ptz.ctypes.data,
                         gt_ptz.ctypes.data, init_rays.ctypes.data, gt_rays.ctypes.data)
    finally:
        L.ptzsynth_free(h)
    return Problem(n_pose=n, n_landmark=m, frame=frame, landmark=landmark, xy=xy, init_ptz=init_ptz,
                   init_rays=init_rays, gt_ptz=gt_ptz, gt_rays=gt_rays, n_pairs=npairs,
                   meta=dict(generator="csrc/synth.cpp", rows=list(rows_a)))


def make_problem(config="config3", seed=0):
    """Synthetic BA problem for one of the BASELINE configs.  Config 4 (tilt rows) comes from
    the native grid generator; configs 1-3 from the numpy path (the fixtures and the bench are pinned to
    its random streams)."""
    n_kf, n_rays, lo, hi, rows = CONFIGS[config]
    if rows is not None:
        prob = make_grid_problem(n_kf, n_rays, lo, hi, rows, seed=seed)
        prob.meta["config"] = config
        prob.meta["seed"] = seed
        return prob
    scene = make_scene(n_kf, n_rays, lo, hi, seed=seed, tilt_rows=rows)
    pairs = scene_pairs(scene, seed=seed)
    prob = problem_from_pairs(scene, pairs)
    prob.meta["config"] = config
    prob.meta["seed"] = seed
    return prob


def make_small_problem(n_kf, n_rays, lo, hi, seed=0, noise=0.5, init_sigma=(0.5, 0.2, 40.0)):
    scene = make_scene(n_kf, n_rays, lo, hi, seed=seed, noise=noise, init_sigma=init_sigma)
    return problem_from_pairs(scene, scene_pairs(scene, seed=seed))


def dedup_records(frame, landmark, xy):
    """Merge identical (frame, landmark, x, y) pair-form records into one weighted record.
    The weighted cost sum_k w_k rho(r_k^2) equals the pair-form cost exactly."""
    key = np.empty(len(frame), dtype=[("l", np.int64), ("f", np.int64), ("x", np.float64), ("y", np.float64)])
    key["l"] = landmark
    key["f"] = frame
    key["x"] = xy[:, 0]
    key["y"] = xy[:, 1]
    uniq, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    return (uniq["f"].astype(np.int32), uniq["l"].astype(np.int32),
            np.stack([uniq["x"], uniq["y"]], 1), cnt.astype(np.float64), inv)


def pose_rmse(a, b):
    """Per-component RMSE over keyframes 1..N-1."""
    d = np.asarray(a)[1:] - np.asarray(b)[1:]
    return np.sqrt(np.mean(d * d, axis=0))


def _selftest():
    p = make_problem("config1", seed=0)
    print(p.n_pose, p.n_landmark, p.n_pairs, p.n_match, len(p.frame))


if __name__ == "__main__":
    _selftest()


class SyntheticFrontEnd:
    """Correspondence source for the reference's front-end hooks (image_process.detect_compute_sift /
    match_sift_features): 'images' are frame ids of a Scene, descriptors carry the frame id, matches are
    the ground-truth shared rays (optionally with `corrupt` swapped matches per pair).  Stands in for
    OpenCV SIFT + BF matching, the same way the golden-fixture generator drives the reference."""

    def __init__(self, scene, corrupt=0, seed=0):
        self.scene = scene
        self.corrupt = corrupt
        self.seed = seed

    def detect(self, im, nfeatures=0, verbose=False):
        import image_process
        i = int(im)
        kps = [image_process.KeyPoint(x, y) for x, y in self.scene.kp_xy[i]]
        des = np.full((len(kps), 128), i, dtype=np.float32)
        if len(kps):
            des[:, 1] = np.arange(len(kps))
        return kps, des

    def match(self, kp1, des1, kp2, des2, pts_array=False, verbose=False):
        i = int(des1[0, 0])
        j = int(des2[0, 0])
        r1, r2 = self.scene.kp_ray[i], self.scene.kp_ray[j]
        pos2 = self._pos(j)
        p = pos2[r1]
        idx1 = np.flatnonzero(p >= 0)
        idx2 = p[idx1]
        if self.corrupt and len(idx2) > 4:
            rng = np.random.default_rng([self.seed, i, j])  # deterministic per pair, like a real matcher
            for _ in range(self.corrupt):
                a, b = rng.choice(len(idx2), 2, replace=False)
                idx2[a], idx2[b] = idx2[b], idx2[a]
        pts1 = np.asarray(self.scene.kp_xy[i], np.float64).reshape(-1, 2)[idx1]
        pts2 = np.asarray(self.scene.kp_xy[j], np.float64).reshape(-1, 2)[idx2]
        return pts1, idx1, pts2, idx2

    def _pos(self, j):
        """ray id -> keypoint position in frame j (-1: not seen), cached per frame."""
        cache = self.__dict__.setdefault("_pos_cache", {})
        if j not in cache:
            r2 = self.scene.kp_ray[j]
            pos = np.full(len(self.scene.gt_rays), -1, np.int64)
            pos[r2] = np.arange(len(r2))
            cache[j] = pos
        return cache[j]

    def install(self):
        import image_process
        image_process.detect_compute_sift = self.detect
        image_process.match_sift_features = self.match
        return self


class _KP:
    """cv2.KeyPoint stand-in (.pt only), usable where the product's image_process is not importable."""
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (float(x), float(y))


class RayFrontEnd:
    """Deterministic detector / matcher over a known ray set for relocalisation (relocalization.py):
    an 'image' is an integer id into `cams` ([n_img, 3] pan, tilt, f); its keypoints are the projections
    (from_ray_to_image, the BA camera model) of the rays strictly inside the image, in ray order, capped at
    `nfeatures`, with per-(image, ray) Gaussian pixel noise; descriptors carry (image id, ray id).
    `match` pairs keypoints by ray id and, like the reference's match_sift_features, returns
    (None, [], None, []) when 8 or fewer matches survive."""

    def __init__(self, rays, cams, u=640.0, v=360.0, width=1280, height=720, noise=0.3, seed=0):
        self.rays = np.asarray(rays, np.float64)
        self.cams = np.asarray(cams, np.float64)
        self.u, self.v, self.width, self.height = float(u), float(v), width, height
        self.noise, self.seed = noise, seed

    def keypoints(self, im, nfeatures=0):
        pan, tilt, f = self.cams[int(im)]
        n = len(self.rays)
        x, y, q2 = _project(self.u, self.v, np.full(n, f), np.full(n, pan), np.full(n, tilt), self.rays[:, 0],
                            self.rays[:, 1])
        vis = np.flatnonzero((q2 > 0) & (x > 0) & (x < self.width) & (y > 0) & (y < self.height))
        if nfeatures:
            vis = vis[:nfeatures]
        pts = np.stack([x[vis], y[vis]], 1)
        for k, r in enumerate(vis):
            g = np.random.default_rng(self.seed * 1000003 + int(im) * 100003 + int(r))
            pts[k] += g.normal(0, self.noise, 2)
        return pts, vis

    def detect(self, im, nfeatures=0, verbose=False):
        pts, vis = self.keypoints(im, nfeatures)
        des = np.zeros((len(vis), 128), np.float32)
        des[:, 0] = int(im)
        des[:, 1] = vis
        des[:, 2] = 1.0
        return [_KP(a, b) for a, b in pts], des

    def match(self, kp1, des1, kp2, des2, pts_array=False, verbose=False):
        r1 = np.asarray(des1)[:, 1].astype(np.int64) if len(des1) else np.zeros(0, np.int64)
        r2 = np.asarray(des2)[:, 1].astype(np.int64) if len(des2) else np.zeros(0, np.int64)
        pos2 = {int(r): j for j, r in enumerate(r2)}
        idx1 = [i for i, r in enumerate(r1) if int(r) in pos2]
        idx2 = [pos2[int(r1[i])] for i in idx1]
        if len(idx1) <= 8:
            return None, [], None, []
        p1 = np.array([kp1[i] if pts_array else kp1[i].pt for i in idx1], np.float64).reshape(-1, 2)
        p2 = np.array([kp2[j] if pts_array else kp2[j].pt for j in idx2], np.float64).reshape(-1, 2)
        return p1, idx1, p2, idx2


def reloc_scene(seed=3):
    """Rays + keyframe cameras + a lost camera for the relocalisation fixtures (reloc.npz)."""
    rng = np.random.default_rng(seed)
    n = 900
    rays = np.stack([rng.uniform(10, 95, n), rng.uniform(-20, 4, n)], 1)
    kf = np.array([[30.0, -8.0, 3000.0], [45.0, -8.5, 2900.0], [60.0, -7.5, 3100.0], [75.0, -8.0, 3000.0]])
    lost_true = np.array([52.0, -7.0, 3200.0])
    lost_init = lost_true + np.array([1.5, -0.6, 120.0])
    cams = np.vstack([kf, lost_true[None]])  # image ids 0..3 keyframes, 4 the lost frame
    return rays, cams, lost_init


# ------------------------------------------------------------------------------------------------
# Streaming sequence (BASELINE configs[4]: per-frame PTZ tracking on a 1080p synthetic court)
# ------------------------------------------------------------------------------------------------
def _hash_u64(*keys):
    """splitmix64 of a key tuple (vectorised over numpy uint64 arrays): counter-based random numbers that
    depend only on the keys, so every consumer (the reference run that made the fixture, this build)
    draws the same values for the same (frame, point) regardless of call order or float round-off."""
    with np.errstate(over="ignore"):
        z = np.uint64(0x9E3779B97F4A7C15)
        for k in keys:
            z = (z ^ np.asarray(k, dtype=np.uint64)) * np.uint64(0xBF58476D1CE4E5B9)
            z = z ^ (z >> np.uint64(31))
            z = z * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(29))
    return z


def _unit(*keys):
    return (_hash_u64(*keys) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _normal(*keys):
    u1 = np.maximum(_unit(*keys, 1), 1e-300)
    u2 = _unit(*keys, 2)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


class SynthImage:
    """One frame of a synthetic stream: the reference reads only `img.shape[0:2]` (ptz_slam.py:333, 434)
    and hands the object to the front-end, which recognises the frame by int(img)."""
    __slots__ = ("index", "shape")

    def __init__(self, index, height, width):
        self.index = int(index)
        self.shape = (int(height), int(width))

    def __int__(self):
        return self.index

    __index__ = __int__

    def __repr__(self):
        return f"SynthImage({self.index})"


class StreamScene:
    """A PTZ broadcast camera sweeping a court: ground-truth pan/tilt/focal per frame (smooth sweep with a
    zoom oscillation, 1920x1080, principal point at the centre) and a field of world rays the detector
    sees (theta U[-50, 50], phi U[-24, 4] deg)."""

    def __init__(self, n_frames, seed=0, n_rays=40000, width=1920, height=1080, pan_lo=-18.0, pan_hi=18.0):
        self.n, self.seed = int(n_frames), int(seed)
        self.width, self.height = int(width), int(height)
        self.u, self.v = width / 2.0, height / 2.0
        t = np.arange(self.n, dtype=np.float64)
        T = max(self.n - 1, 1)
        pan = pan_lo + (pan_hi - pan_lo) * 0.5 * (1.0 - np.cos(np.pi * t / T))
        tilt = -9.0 + 1.2 * np.sin(2.0 * np.pi * t / 97.0)
        f = 2600.0 + 300.0 * np.sin(2.0 * np.pi * t / 151.0)
        self.cams = np.stack([pan, tilt, f], 1)
        rng = np.random.default_rng(seed + 17)
        self.rays = np.stack([rng.uniform(-50.0, 50.0, n_rays), rng.uniform(-24.0, 4.0, n_rays)], 1)
        self.response = rng.permutation(n_rays)  # detector strength rank per ray (lower = stronger)

    def image(self, i):
        return SynthImage(i, self.height, self.width)

    def camera(self, i):
        """ptz_camera.PTZCamera of frame i (the ground truth; the sequence's first camera seeds the tracker)."""
        from ptz_camera import PTZCamera
        cam = PTZCamera((self.u, self.v), np.array([0.0, -16.0, 5.0]), np.eye(3))
        cam.set_ptz(self.cams[i].copy())
        return cam


def _back_project(u, v, f, pan, tilt, x, y):
    """Inverse of _project for points in front of the camera (q2 > 0): pixel -> ray (theta, phi) in degrees."""
    a = np.radians(pan); b = np.radians(tilt)
    ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
    q0, q1, q2 = (x - u) / f, (y - v) / f, 1.0
    v0, v1, v2 = q0, cb * q1 - sb * q2, sb * q1 + cb * q2
    d0, d1, d2 = ca * v0 + sa * v2, v1, -sa * v0 + ca * v2
    p0, p1 = d0 / d2, d1 / d2
    return np.degrees(np.arctan(p0)), np.degrees(np.arctan(-p1 / np.sqrt(p0 * p0 + 1.0)))


class RenderedStream:
    """8-bit grey 1080p frames of a StreamScene rendered from a textured panorama of the ray sphere (octaves of
    smoothed lattice noise over (theta, phi), cells 2.0 / 0.8 / 0.3 / 0.12 deg): every pixel is back-projected
    with the frame's TRUE camera (_back_project, the q-form model) and samples the panorama bilinearly.  Feeds the
    real front-end (GPU SIFT, pyramidal LK, homography RANSAC) instead of StreamFrontEnd's stand-in.
    Frames are rendered on first use and cached."""

    def __init__(self, scene, seed=0, res=0.02, octaves=((2.0, 55.0), (0.8, 40.0), (0.3, 28.0), (0.12, 14.0))):
        self.s = scene
        self.cams = scene.cams
        self.u, self.v, self.width, self.height = scene.u, scene.v, scene.width, scene.height
        W, H = scene.width, scene.height
        bx = np.array([0, W / 2, W - 1, 0, W - 1, 0, W / 2, W - 1], np.float64)
        by = np.array([0, 0, 0, H / 2, H / 2, H - 1, H - 1, H - 1], np.float64)
        th, ph = _back_project(scene.u, scene.v, self.cams[:, 2:3], self.cams[:, 0:1], self.cams[:, 1:2], bx, by)
        m = 1.0
        self.th0, self.ph0 = th.min() - m, ph.min() - m
        nx = int(np.ceil((th.max() + m - self.th0) / res)) + 2
        ny = int(np.ceil((ph.max() + m - self.ph0) / res)) + 2
        self.res = res
        rng = np.random.default_rng(seed + 101)
        gx = self.th0 + res * np.arange(nx)
        gy = self.ph0 + res * np.arange(ny)
        pano = np.full((ny, nx), 128.0, np.float32)
        for cell, amp in octaves:
            lx, ly = int(np.ceil(nx * res / cell)) + 3, int(np.ceil(ny * res / cell)) + 3
            lat = rng.uniform(-1.0, 1.0, (ly, lx)).astype(np.float32)
            fx, fy = (gx - self.th0) / cell, (gy - self.ph0) / cell
            ix, iy = np.floor(fx).astype(np.int64), np.floor(fy).astype(np.int64)
            sx, sy = fx - ix, fy - iy
            sx, sy = (sx * sx * (3 - 2 * sx)).astype(np.float32), (sy * sy * (3 - 2 * sy)).astype(np.float32)
            top = lat[iy][:, ix] * (1 - sx) + lat[iy][:, ix + 1] * sx
            bot = lat[iy + 1][:, ix] * (1 - sx) + lat[iy + 1][:, ix + 1] * sx
            pano += amp * (top * (1 - sy)[:, None] + bot * sy[:, None])
        self.pano = pano
        yy, xx = np.mgrid[0:H, 0:W]
        self._xy = (xx.astype(np.float64).ravel(), yy.astype(np.float64).ravel())
        self._cache = {}

    def image(self, i):
        if i not in self._cache:
            pan, tilt, f = self.cams[i]
            th, ph = _back_project(self.u, self.v, f, pan, tilt, *self._xy)
            fx, fy = (th - self.th0) / self.res, (ph - self.ph0) / self.res
            ix = np.clip(np.floor(fx).astype(np.int64), 0, self.pano.shape[1] - 2)
            iy = np.clip(np.floor(fy).astype(np.int64), 0, self.pano.shape[0] - 2)
            ax, ay = (fx - ix).astype(np.float32), (fy - iy).astype(np.float32)
            P = self.pano
            val = (P[iy, ix] * (1 - ax) + P[iy, ix + 1] * ax) * (1 - ay) + (P[iy + 1, ix] * (1 - ax) + P[iy + 1, ix + 1] * ax) * ay
            self._cache[i] = np.clip(np.rint(val), 0, 255).astype(np.uint8).reshape(self.height, self.width)
        return self._cache[i]

    def camera(self, i):
        return self.s.camera(i)


class StreamFrontEnd:
    """Stand-in for the reference's OpenCV front-end on a StreamScene (the way make_golden.py's FrontEnd
    stands in for SIFT + BF matching):
      * detect_compute_sift(img, n): the visible world rays of frame img, strongest first, capped at n;
        keypoint = true projection + N(0, 0.3 px); descriptor carries the ray id;
      * match_sift_features: ground-truth correspondences by ray id (as match_sift_features' ratio test
        would give on distinctive features); (None, [], None, []) below 9 matches, like the reference;
      * optical_flow_matching(img, next_img, points): a pure-rotation camera moves image content by the
        homography of the two TRUE poses: back-project with frame img's camera, project with next_img's,
        + N(0, 0.2 px); points leaving the image fail (image_process.py:393-415); 3 % of the points
        (keyed by (frame, index)) are displaced 6-20 px (players, flicker);
      * homography_ransac: the undisplaced points are the inliers (a 0.5 px RANSAC separates them).
    Every random number is keyed by (seed, frame, point), so the reference run and this build see the same
    data."""

    def __init__(self, scene, noise=0.3, flow_noise=0.2, outlier_rate=0.03):
        self.s = scene
        self.noise, self.flow_noise, self.outlier_rate = noise, flow_noise, outlier_rate
        self._last = None
        self.time = 0.0  # seconds spent inside the stand-in (reported separately by the stream driver)

    # ---- detection / matching (keyframes, init_system, add_rays)
    def _visible(self, i):
        pan, tilt, f = self.s.cams[i]
        r = self.s.rays
        x, y, q2 = _project(self.s.u, self.s.v, f, pan, tilt, r[:, 0], r[:, 1])
        vis = np.flatnonzero((q2 > 0) & (x > 0) & (x < self.s.width) & (y > 0) & (y < self.s.height))
        vis = vis[np.argsort(self.s.response[vis], kind="stable")]
        return vis, x[vis], y[vis]

    def detect(self, im, nfeatures=0, verbose=False):
        import time
        t0 = time.perf_counter()
        i = int(im)
        vis, x, y = self._visible(i)
        if nfeatures and nfeatures > 0:
            vis, x, y = vis[:nfeatures], x[:nfeatures], y[:nfeatures]
        x = x + self.noise * _normal(self.s.seed, 1, i, vis)
        y = y + self.noise * _normal(self.s.seed, 2, i, vis)
        ok = (x > 0) & (x < self.s.width) & (y > 0) & (y < self.s.height)
        vis, x, y = vis[ok], x[ok], y[ok]
        kps = [_KP(a, b) for a, b in zip(x, y)]
        des = np.zeros((len(vis), 128), np.float32)
        des[:, 0] = vis + 1
        des[:, 1] = i
        des[:, 2] = 1.0
        self.time += time.perf_counter() - t0
        return kps, des

    def match(self, kp1, des1, kp2, des2, pts_array=False, verbose=False):
        r1 = np.rint(np.asarray(des1)[:, 0]).astype(np.int64) if len(des1) else np.zeros(0, np.int64)
        r2 = np.rint(np.asarray(des2)[:, 0]).astype(np.int64) if len(des2) else np.zeros(0, np.int64)
        pos2 = {int(r): j for j, r in enumerate(r2)}
        idx1 = [i for i, r in enumerate(r1) if int(r) in pos2]
        idx2 = [pos2[int(r1[i])] for i in idx1]
        if len(idx1) <= 8:
            return None, [], None, []
        p1 = np.array([kp1[i] if pts_array else kp1[i].pt for i in idx1], np.float64).reshape(-1, 2)
        p2 = np.array([kp2[j] if pts_array else kp2[j].pt for j in idx2], np.float64).reshape(-1, 2)
        return p1, idx1, p2, idx2

    # ---- frame-to-frame tracking (ptz_slam.py:397 -> image_process.py:464-506)
    def optical_flow(self, img, next_img, points, ssd_threshold=20):
        import time
        t0 = time.perf_counter()
        i, j = int(img), int(next_img)
        p = np.asarray(points, np.float64).reshape(-1, 2)
        k = np.arange(len(p))
        a = self.s.cams[i]
        b = self.s.cams[j]
        th, ph = image_to_ray(self.s.u, self.s.v, a[2], a[0], a[1], p[:, 0], p[:, 1])
        x, y, q2 = _project(self.s.u, self.s.v, b[2], b[0], b[1], th, ph)
        x = x + self.flow_noise * _normal(self.s.seed, 3, j, k)
        y = y + self.flow_noise * _normal(self.s.seed, 4, j, k)
        bad = _unit(self.s.seed, 5, j, k) < self.outlier_rate
        mag = 6.0 + 14.0 * _unit(self.s.seed, 6, j, k)
        ang = 2.0 * np.pi * _unit(self.s.seed, 7, j, k)
        x = np.where(bad, x + mag * np.cos(ang), x)
        y = np.where(bad, y + mag * np.sin(ang), y)
        h, w = self.s.height, self.s.width
        ok = (q2 > 0) & (x > 0) & (x < w) & (y > 0) & (y < h)
        matched = [int(t) for t in np.flatnonzero(ok)]
        self._last = bad[ok]
        self.time += time.perf_counter() - t0
        return matched, np.stack([x[ok], y[ok]], 1).reshape(-1, 2)

    def ransac(self, points1, points2, reprojection_threshold=0.5, return_matrix=False):
        assert self._last is not None and len(self._last) == len(points1) == len(points2)
        index = [int(t) for t in np.flatnonzero(~self._last)]
        if return_matrix:
            return index, None
        return index

    def install(self, *modules):
        """Assign the hooks in image_process (this build) or in the given modules (e.g. the reference's
        image_process when generating fixtures)."""
        if not modules:
            import image_process
            modules = (image_process,)
        for m in modules:
            m.detect_compute_sift = self.detect
            m.match_sift_features = self.match
            m.optical_flow_matching = self.optical_flow
            m.homography_ransac = self.ransac
        return self
