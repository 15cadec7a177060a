"""
Bundle adjustment — drop-in replacement for slam_system/bundle_adjustment.py.

    bundle_adjustment(images, image_indices, feature_method, initial_ptzs, center, rotation, u, v,
                      save_path, verbose=False)  ->  (landmarks float64 [M, 2], list[KeyFrame])

Same signature, steps and outputs as the reference (bundle_adjustment.py:109-251):
  1. pair mask: overlap_pan_angle(f_i, pan_i, f_j, pan_j, 1280) > 5 deg          (:135-144)
  2. matching graph (image_process.build_matching_graph: front-end hooks + bit-exact bookkeeping)
  3. n_residual = sum 4 |matches|; x0 = [poses | rays], each ray from from_image_to_ray of its
     src observation in frame i with the LAST match in loop order winning          (:167-197)
  4. optimisation — the reference's scipy `least_squares(_compute_residual, x0, x_scale='jac',
     ftol=1e-4, method='trf')` (:200-202) is replaced by the GPU Levenberg-Marquardt of libptzba
     (exact Schur-complement steps, same ftol termination rule), frame 0 fixed     (:197)
  5. KeyFrame assembly with the reference's set() de-duplication order            (:214-248)
Steps 2, 3 and 5 run on correspondence.MatchGraph (native builder); pass a
correspondence.CorrespondenceCache as `correspondences=` to skip re-detection/re-matching.

Extra keyword arguments (all optional) select the numerics: precision ('fp64' default, 'fp32'),
loss ('linear' as the reference, or 'huber'), f_scale, ftol/xtol/max_iter, device.
`_compute_residual` keeps the reference signature and returns the identical residual vector
(computed by libptzba, record order == the reference's loop order).
"""
import time

import numpy as np

import image_process
import ptzba
from key_frame import KeyFrame
from util import overlap_pan_angle_half_fov

LAST_RESULT = {}


def _flatten(n_pose, src_pt_index, dst_pt_index, landmark_index):
    """Flat match arrays (m_i, m_j, k1, k2, lm) in the reference's residual loop order
    (bundle_adjustment.py:67-99: for i, for j, for each match)."""
    mi, mj, a, b, l = [], [], [], [], []
    for i in range(n_pose):
        for j in range(n_pose):
            s = src_pt_index[i][j]
            if len(s) == 0:
                continue
            a.append(np.asarray(s, np.int64))
            b.append(np.asarray(dst_pt_index[i][j], np.int64))
            l.append(np.asarray(landmark_index[i][j], np.int64))
            mi.append(np.full(len(s), i, np.int32))
            mj.append(np.full(len(s), j, np.int32))
    cat = lambda x, t: np.concatenate(x) if x else np.zeros(0, t)
    return cat(mi, np.int32), cat(mj, np.int32), cat(a, np.int64), cat(b, np.int64), cat(l, np.int64)


def _records(n_pose, keypoints, src_pt_index, dst_pt_index, landmark_index):
    """Pair-form records in the reference's residual order: for i, for j, for each match ->
    record (i, kp1) then (j, kp2)."""
    mi, mj, a, b, l = _flatten(n_pose, src_pt_index, dst_pt_index, landmark_index)
    pts = [np.asarray(k, np.float64).reshape(-1, 2) for k in keypoints]
    kp_off = np.concatenate([[0], np.cumsum([len(p) for p in pts])]).astype(np.int64)
    kp_xy = np.concatenate(pts) if pts else np.zeros((0, 2))
    n_lm = int(l.max()) + 1 if len(l) else 0
    fr, lm, xy, _ = ptzba.pack_records(n_pose, mi, mj, a, b, l, kp_off, kp_xy, n_lm)
    return fr, lm, xy


def _compute_residual(x, n_pose, n_landmark, n_residual, keypoints, src_pt_index, dst_pt_index, landmark_index, u, v,
                      reference_pose, verbose=False, precision=ptzba.FP64, device=0):
    """bundle_adjustment.py:25-106 — same arguments, same residual vector (computed on the GPU)."""
    assert x.shape[0] == (n_pose - 1) * 3 + n_landmark * 2
    assert len(keypoints) == n_pose and len(src_pt_index) == n_pose
    assert len(dst_pt_index) == n_pose and len(landmark_index) == n_pose
    assert np.asarray(reference_pose).shape[0] == 3
    frame, lm, xy = _records(n_pose, keypoints, src_pt_index, dst_pt_index, landmark_index)
    assert 2 * len(frame) == n_residual
    h = ptzba.BAHandle(device)
    try:
        h.set_problem(n_pose, n_landmark, frame, lm, xy, u, v, precision=precision)
        r = h.residual(np.concatenate([np.asarray(reference_pose, np.float64), np.asarray(x, np.float64)]))
    finally:
        h.close()
    if verbose:
        e = np.sqrt(r[0::2] ** 2 + r[1::2] ** 2)
        print("reprojection error is %f" % (e.sum() / (n_residual / 2)))
    return r


class _KeyframeLists:
    """The per-keyframe (local keypoint, global landmark) lists of one BA call in the reference's set() order
    (bundle_adjustment.py:218-239, native: MatchGraph.keyframe_features), formed for all keyframes at the first
    request."""

    def __init__(self, graph):
        self.graph = graph
        self.csr = None
        self.used = None
        self.counts = None

    def lists(self, i):
        if self.csr is None:
            self.csr = self.graph.keyframe_features()
            self.graph = None
            self.used = self.counts = None
        off, loc, glo = self.csr
        return loc[off[i]:off[i + 1]], glo[off[i]:off[i + 1]]

    def count(self, i):
        """len() of keyframe i's lists, without forming them (the verbose print of bundle_adjustment.py:238)."""
        if self.csr is not None:
            return int(self.csr[0][i + 1] - self.csr[0][i])
        if self.counts is None:
            g = self.graph
            self.counts = ptzba.keyframe_feature_counts(g.n_frames, g.m_i, g.m_j, g.k1, g.k2, g.lm)
        return int(self.counts[i])

    def nonempty(self, i):
        """keyframe i's list is non-empty: it takes part in a match of this call."""
        if self.csr is not None:
            return self.csr[0][i + 1] > self.csr[0][i]
        if self.used is None:
            g = self.graph
            self.used = (np.bincount(g.m_i, minlength=g.n_frames) + np.bincount(g.m_j, minlength=g.n_frames)) > 0
        return bool(self.used[i])


def bundle_adjustment(images, image_indices, feature_method, initial_ptzs, center, rotation, u, v, save_path,
                      verbose=False, precision="fp64", loss="linear", f_scale=1.0, ftol=1e-4, xtol=1e-8,
                      max_iter=100, device=0, correspondences=None):
    """bundle_adjustment.py:109-251 on the MI355X path.  Returns (landmarks [M,2], keyframes).
    `correspondences`: optional correspondence.CorrespondenceCache keyed by image_indices, so repeated
    calls over growing / sliding keyframe sets only detect new images and match new pairs."""
    import correspondence
    N = len(images)
    assert N >= 1
    assert len(image_indices) == N
    initial_ptzs = np.asarray(initial_ptzs, np.float64)
    assert initial_ptzs.shape[0] == N and initial_ptzs.shape[1] == 3
    assert np.asarray(center).shape[0] == 3 and np.asarray(rotation).shape == (3, 3)
    assert feature_method in ("sift", "orb", "latch")
    timing = {}
    t_start = time.time()

    # step 1: pair mask (bundle_adjustment.py:135-144): overlap_pan_angle(f_i, pan_i, f_j, pan_j, 1280) > 5 for every
    # pair, with each camera's half field of view formed once (the same float operations, so the same mask)
    half = np.array([overlap_pan_angle_half_fov(fl, 1280) for fl in initial_ptzs[:, 2].tolist()])
    pan = initial_ptzs[:, 0]
    overlap = (np.minimum((pan + half)[:, None], (pan + half)[None, :]) -
               np.maximum((pan - half)[:, None], (pan - half)[None, :]))
    image_match_mask = (overlap > 5).astype(np.int64).tolist()
    g = correspondence.build_graph(images, image_match_mask, feature_method, verbose, cache=correspondences,
                                   keys=list(image_indices))
    keypoints, descriptors, n_landmark = g.keypoints, g.descriptors, g.n_landmark
    if image_process.draw_matches is not None and save_path:
        pts = g.points()
        for p in range(len(g.pair_i)):
            i, j = int(g.pair_i[p]), int(g.pair_j[p])
            a, b = g.pair_off[p], g.pair_off[p + 1]
            image_process.draw_matches(images[i], images[j], pts[i][g.k1[a:b]], pts[j][g.k2[a:b]],
                                       save_path + "/" + str(i) + "_" + str(j) + ".jpg")
    timing["graph"] = time.time() - t_start
    timing.update(getattr(g, "timing", {}))

    # step 2: data (bundle_adjustment.py:167-197)
    t1 = time.time()
    n_residual = 4 * g.n_matches
    if verbose:
        print("residual number is %d." % n_residual)
    ref_pose = initial_ptzs[0]
    frame, lm, xy, src_rec = g.records()
    rays0 = np.zeros((n_landmark, 2))
    if n_landmark:
        # each ray from the src observation of the last match referencing it (last writer wins)
        has = src_rec >= 0
        lids = np.flatnonzero(has)
        rec = src_rec[has]
        fi = frame[rec]
        th, ph = ptzba.image_to_ray(u, v, initial_ptzs[fi, 2], initial_ptzs[fi, 0], initial_ptzs[fi, 1], xy[rec, 0],
                                    xy[rec, 1], device=device)
        rays0[lids, 0] = th
        rays0[lids, 1] = ph
    timing["records"] = time.time() - t1

    # step 3: optimisation on the GPU (replaces bundle_adjustment.py:200-202)
    t0 = time.time()
    all_poses = initial_ptzs.copy()
    landmarks = rays0.copy()
    res = None
    if len(frame):
        prec = ptzba.FP32 if precision == "fp32" else ptzba.FP64
        ls = ptzba.LOSS_HUBER if loss == "huber" else ptzba.LOSS_LINEAR
        all_poses, landmarks, res = ptzba.solve(N, n_landmark, frame, lm, xy, u, v, initial_ptzs, rays0, precision=prec,
                                                loss=ls, f_scale=f_scale, device=device, ftol=ftol, xtol=xtol,
                                                max_iter=max_iter)
        all_poses[0] = ref_pose
        if verbose:
            print(f"GPU LM: {res}")
    timing["solve"] = time.time() - t0
    timing.update({"solve_" + k: v for k, v in ptzba.LAST_SOLVE_TIMING.items()})

    # step 5: keyframes (bundle_adjustment.py:214-248), features in the reference's set() order -- formed for every
    # keyframe of this call at the first access to any of their feature lists (_KeyframeLists)
    t2 = time.time()
    lists = _KeyframeLists(g)
    keyframes = []
    for i in range(N):
        pan, tilt, fl = all_poses[i]
        key_frame = KeyFrame(images[i], image_indices[i], center, rotation, u, v, pan, tilt, fl)
        # feature_pts = [keypoints[i][k] for k in local_index], feature_des = descriptors[i][local_index],
        # landmark_index = global ids, on first use (KeyFrame.set_features_lazy)
        key_frame.set_features_lazy(keypoints[i], descriptors[i], lists, i)
        keyframes.append(key_frame)
        if verbose:  # (the list's length without forming it)
            print("frame %d, landmark number %d" % (image_indices[i], lists.count(i)))
    timing["keyframes"] = time.time() - t2
    LAST_RESULT.clear()
    LAST_RESULT.update(result=res, n_residual=n_residual, n_landmark=n_landmark, time=timing["solve"],
                       timing=timing, x0=np.concatenate([initial_ptzs[1:].reshape(-1), rays0.reshape(-1)]))
    return landmarks, keyframes
