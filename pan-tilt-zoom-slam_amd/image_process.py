"""
Feature front-end + matching-graph bookkeeping (reference: slam_system/image_process.py).

The reference detects SIFT/ORB features and matches them with OpenCV (image_process.py:14-506).  OpenCV
is not in this image, so the front-end the demo uses runs on the GPU through libptzba:
  * detect_compute_sift / detect_sift / detect_compute_sift_array  -> ptz_sift (OpenCV's SIFT defaults);
  * match_sift_features   -> ptz_match_knn2 (BF kNN-2) + the 0.7 ratio test + homography_ransac;
  * match_orb_features / match_latch_features -> ptz_match_hamming (cross-checked) + homography_ransac;
  * homography_ransac     -> ptz_homography_ransac;  optical_flow_matching -> ptz_lk_track (pyramidal LK);
  * detect_compute_orb / detect_compute_latch -> ptz_orb (OpenCV's ORB pipeline: 8-level pyramid, FAST-9,
    Harris retain-best, intensity-centroid angle; rBRIEF 32-byte or LATCH 64-byte descriptors with generated
    sampling tables -- OpenCV's learned tables are not available, so the bits are not cv2's).
Their agreement with cv2's own numbers is unpinned (cv2 cannot run here): each kernel is pinned to the
oracle's restatement of the published algorithm and to synthetic ground truth (tests/test_gpu_frontend.py).
A correspondence source (e.g. synthetic.SyntheticFrontEnd, or an OpenCV wrapper on a machine that has it)
may reassign any of these functions, exactly the way the reference's own tests monkeypatch the front-end.

The bookkeeping of `build_matching_graph` (image_process.py:509-667) keeps the reference's exact semantics:
  * pairs i < j in order, skipped when image_match_mask[i][j] == 0;
  * a pair is kept if it has MORE than 20 matches (`len > min_match_num`, :590);
  * pairs with more than 200 matches are capped by `random.shuffle` of the GLOBAL `random`
    module (:592-597), so a seeded `random` reproduces the reference bit for bit;
  * landmark ids by the first-seen rule (:611-639) — computed natively in libptzba
    (ptzba_build_landmarks), including the count of the reference's "in-consistent matching" warnings.
The graph itself is built by correspondence.build_graph (flat arrays, native cap-shuffle replay).
"""
import functools
import os
import operator

import numpy as np


class KeyPoint(tuple):
    """Stand-in for cv2.KeyPoint (the reference only reads `.pt`; size / angle / response / octave as the
    detectors set them).  An immutable record ((x, y), size, angle, response, octave): the detectors build their
    1500-keypoint lists with KeyPoint.from_rows at C speed (a keyframe's detection otherwise spent ~1 ms in
    per-keypoint constructors)."""
    __slots__ = ()

    def __new__(cls, x, y, size=0.0, angle=-1.0, response=0.0, octave=0):
        return tuple.__new__(cls, ((float(x), float(y)), float(size), float(angle), float(response), int(octave)))

    def __getnewargs__(self):
        return (self[0][0], self[0][1], self[1], self[2], self[3], self[4])

    pt = property(operator.itemgetter(0))
    size = property(operator.itemgetter(1))
    angle = property(operator.itemgetter(2))
    response = property(operator.itemgetter(3))
    octave = property(operator.itemgetter(4))

    def __repr__(self):
        return "KeyPoint(pt=%r, size=%r, angle=%r, response=%r, octave=%r)" % tuple(self)

    @classmethod
    def from_rows(cls, xy, size, angle, response, octave=None):
        """[KeyPoint] from columns: xy [n, 2], size / angle / response [n] (Python floats after tolist: the values
        the constructor's float() would give), octave [n] ints or None (0).  The list carries the points as an [n, 2]
        float64 array (`.xy`, == [k.pt for k in list]) for callers that want them without a loop."""
        n = len(size)
        xy64 = np.array(xy, np.float64).reshape(-1, 2)
        pts = list(map(tuple, xy64.tolist()))
        oc = [0] * n if octave is None else [int(o) for o in octave]
        rows = zip(pts, np.asarray(size, np.float64).tolist(), np.asarray(angle, np.float64).tolist(),
                   np.asarray(response, np.float64).tolist(), oc)
        out = KeyPointList(map(functools.partial(tuple.__new__, cls), rows))
        xy64.flags.writeable = False
        out.xy = xy64
        return out


class KeyPointList(list):
    """A plain list of KeyPoint plus `.xy`, the points as a read-only [n, 2] float64 array (slices and copies are
    plain lists: only the detector's own list carries it)."""
    xy = None


def keypoint_xy(kps):
    """[n, 2] float64 array of the keypoints' .pt (the detector's array when the list carries one)."""
    xy = getattr(kps, "xy", None)
    if xy is not None and len(xy) == len(kps):
        return xy
    return np.array([k.pt for k in kps], dtype=np.float64).reshape(-1, 2)


# detect_compute_* / detect_sift / match_*_features / homography_ransac / optical_flow_matching: GPU
# implementations below (SIFT, ORB / LATCH, kNN-2 + ratio test + RANSAC, Hamming + RANSAC, pyramidal LK); a
# correspondence source may still assign its own
draw_matches = None  # optional visualisation hook (bundle_adjustment.py:153-163)


def detect_compute_orb(im, nfeatures=1000, verbose=False):
    """image_process.py:105-126 on the GPU (libptzba ptz_orb, cv.ORB_create(nfeatures) defaults): keypoints
    (KeyPoint with .pt, .size, .angle, .response, .octave) and descriptors [n, 32] uint8, truncated to
    nfeatures as the reference does (the per-level cuts keep ties, so the detector may return more)."""
    import ptzba
    assert isinstance(im, np.ndarray)
    assert nfeatures > 0
    kp, des = ptzba.orb(_grey_u8(im), int(nfeatures), "orb")
    kp = np.asarray(kp)
    key_point = KeyPoint.from_rows(kp[:, 0:2], kp[:, 2], kp[:, 3], kp[:, 4], kp[:, 5].astype(np.int64).tolist())
    if len(key_point) > nfeatures:
        key_point = key_point[:nfeatures]
        des = des[:nfeatures]
    if verbose:
        print('detect: %d ORB keypoints.' % len(key_point))
    return key_point, des


def detect_compute_latch(im, nfeatures=1500, verbose=False):
    """image_process.py:129-155 on the GPU: ORB keypoints (cv.ORB_create(nfeatures).detect), LATCH(64)
    descriptors [n, 64] uint8 on them (points whose 48-px patch leaves the image are dropped, as LATCH does),
    truncated to nfeatures."""
    import ptzba
    assert isinstance(im, np.ndarray)
    kp, des = ptzba.orb(_grey_u8(im), int(nfeatures) if nfeatures > 0 else 500, "latch")
    kp = np.asarray(kp)
    key_point = KeyPoint.from_rows(kp[:, 0:2], kp[:, 2], kp[:, 3], kp[:, 4], kp[:, 5].astype(np.int64).tolist())
    if nfeatures > 0 and len(key_point) > nfeatures:
        key_point = key_point[:nfeatures]
        des = des[:nfeatures]
    if verbose:
        print('detect: %d LATCH keypoints.' % len(key_point))
    return key_point, des


def detect_compute_sift(im, nfeatures, verbose=False):
    """image_process.py:56-79 on the GPU (libptzba ptz_sift: OpenCV's SIFT defaults): keypoints (KeyPoint with
    .pt, .size, .angle, .response) strongest first, at most nfeatures (> 0), and descriptors [n, 128] float32."""
    import ptzba
    kp, resp, des = ptzba.sift(_grey_u8(im), int(nfeatures))
    key_point = KeyPoint.from_rows(kp[:, 0:2], kp[:, 2], kp[:, 3], resp)
    if verbose:
        print('detect: %d SIFT keypoints.' % len(key_point))
    return key_point, des


_gpu_detect_compute_sift = detect_compute_sift


def detect_sift(im, nfeatures=50):
    """image_process.py:14-33 on the GPU: SIFT keypoint locations [n, 2] float32."""
    import ptzba
    kp, _, _ = ptzba.sift(_grey_u8(im), int(nfeatures))
    return np.ascontiguousarray(kp[:, :2])


def detect_compute_sift_array(im, nfeatures, norm=True):
    """image_process.py:82-102: keypoints as an [N,2] array, descriptors (L2-normalised) [N,128]."""
    if detect_compute_sift is _gpu_detect_compute_sift:  # the GPU default: straight from the arrays
        import ptzba
        kp, _, des = ptzba.sift(_grey_u8(im), int(nfeatures))
        pts = kp[:, :2].astype(np.float64)
    else:  # a correspondence source assigned its own detector
        kps, des = detect_compute_sift(im, nfeatures)
        pts = np.array([k.pt for k in kps], dtype=np.float64).reshape(-1, 2)
    des = np.asarray(des)
    if norm and len(des):
        des = (des / np.linalg.norm(des, axis=1).reshape(-1, 1)).astype(np.float64)
    return pts, des


def match_sift_features(keypoint1, descriptor1, keypoint2, descriptor2, pts_array=False, verbose=False):
    """image_process.py:178-234 on the GPU: 2-nearest-neighbour L2 matching (cv.BFMatcher().knnMatch, k=2:
    libptzba ptz_match_knn2), Lowe's ratio test m < 0.7 n, then the homography RANSAC inliers (1 px).
    Returns (pts1, index1, pts2, index2) like the reference; (None, [], None, []) below 9 ratio-test
    survivors."""
    import ptzba
    d1 = np.asarray(descriptor1, dtype=np.float32)
    d2 = np.asarray(descriptor2, dtype=np.float32)
    idx, dist = ptzba.match_knn2(d1, d2)
    good = np.flatnonzero(dist[:, 0] < 0.7 * dist[:, 1]) if len(d2) >= 2 else np.zeros(0, np.int64)
    if verbose:
        print('%d matches passed the ratio test' % len(good))
    if len(good) <= 8:
        print('warning: match sift features failed, not enough matching')
        return None, [], None, []
    index1 = good.astype(np.int32)
    index2 = idx[good, 0].astype(np.int32)
    if pts_array:
        pts1 = np.asarray(keypoint1, np.float64).reshape(-1, 2)[index1]
        pts2 = np.asarray(keypoint2, np.float64).reshape(-1, 2)[index2]
    else:
        pts1 = np.array([keypoint1[i].pt for i in index1], np.float64).reshape(-1, 2)
        pts2 = np.array([keypoint2[j].pt for j in index2], np.float64).reshape(-1, 2)
    inlier_index = homography_ransac(pts1, pts2, 1.0)
    if verbose:
        print('%d matches passed the homography ransac' % len(inlier_index))
    return pts1[inlier_index, :], index1[inlier_index].tolist(), pts2[inlier_index, :], index2[inlier_index].tolist()


GPU_MATCH_SIFT = match_sift_features  # (correspondence.build_graph batches pairs only while this is the matcher)


def _pts(kp, index):
    """[len(index), 2] float64 positions of keypoints `index` (KeyPoint list or an [n, 2] array of .pt values)."""
    if isinstance(kp, np.ndarray):
        return np.asarray(kp, np.float64).reshape(-1, 2)[index]
    return np.array([kp[i].pt for i in index], np.float64).reshape(-1, 2)


def match_sift_features_batch(pairs, dev_sets=None):
    """match_sift_features for several descriptor pairs in three launches instead of five per pair: `pairs` is a
    list of (keypoints1, descriptors1, keypoints2, descriptors2) -- keypoints as KeyPoint lists or [n, 2] arrays of
    their .pt; pairs sharing the same train set (descriptors2
    object) run as ONE kNN-2 over their concatenated queries (a new keyframe against every overlapping window
    partner), the ratio test per pair, then ONE batched homography RANSAC (ptz_homography_ransac_batch, per pair
    the same seed and result as homography_ransac).  Returns [(index1 list, index2 list)] with exactly
    match_sift_features' (index1, index2) per pair (empty lists where it returns none).
    dev_sets: optional [((query set id, rows), (train set id, rows))] per pair -- the descriptors already on the
    device (ptzba.desc_put, correspondence.CorrespondenceCache.dev_set): the kNN-2 then reads them there
    (ptzba.match_knn2_sets, the same result) instead of concatenating and uploading every query set again."""
    import ptzba
    out = [([], []) for _ in pairs]
    groups = {}
    for q, (_, d1, _, d2) in enumerate(pairs):
        groups.setdefault(dev_sets[q][1][0] if dev_sets is not None else id(d2), []).append(q)
    if dev_sets is not None and len(groups) == 1 and all(isinstance(p[0], np.ndarray) for p in pairs) and \
            isinstance(pairs[0][2], np.ndarray) and os.environ.get("PTZ_MATCH_FUSED", "1") != "0":
        # one train set (a new keyframe against its window partners) and keypoint arrays: kNN-2, ratio tests,
        # point gathers and RANSAC in one native call (ptz_match_sets_ransac), per pair the same result
        res = ptzba.match_sets_ransac([dev_sets[q][0][0] for q in range(len(pairs))],
                                      [dev_sets[q][0][1] for q in range(len(pairs))], dev_sets[0][1][0],
                                      dev_sets[0][1][1], np.concatenate([np.asarray(p[0], np.float64).reshape(-1, 2)
                                                                         for p in pairs]), pairs[0][2], 1.0)
        for q, r in enumerate(res):
            if r is None:
                print('warning: match sift features failed, not enough matching')
            else:
                out[q] = (r[0].tolist(), r[1].tolist())
        return out
    cand = []  # (pair, index1, index2, pts1, pts2)
    for qs in groups.values():
        n2 = dev_sets[qs[0]][1][1] if dev_sets is not None else len(pairs[qs[0]][3])
        if dev_sets is not None:
            lens = [dev_sets[q][0][1] for q in qs]
            if sum(lens) == 0:
                continue
            idx, dist = ptzba.match_knn2_sets([dev_sets[q][0][0] for q in qs], lens, dev_sets[qs[0]][1][0])
        else:
            d2 = np.asarray(pairs[qs[0]][3], dtype=np.float32)
            d1s = [np.asarray(pairs[q][1], dtype=np.float32) for q in qs]
            lens = [len(d) for d in d1s]
            if sum(lens) == 0:
                continue
            idx, dist = ptzba.match_knn2(np.concatenate(d1s), d2)
        o = 0
        for q, n1 in zip(qs, lens):
            di, ii = dist[o:o + n1], idx[o:o + n1]
            o += n1
            good = np.flatnonzero(di[:, 0] < 0.7 * di[:, 1]) if n2 >= 2 else np.zeros(0, np.int64)
            if len(good) <= 8:
                print('warning: match sift features failed, not enough matching')
                continue
            index1 = good.astype(np.int32)
            index2 = ii[good, 0].astype(np.int32)
            pts1, pts2 = _pts(pairs[q][0], index1), _pts(pairs[q][2], index2)
            cand.append((q, index1, index2, pts1, pts2))
    res = ptzba.homography_ransac_batch([(c[3], c[4]) for c in cand], 1.0)
    for (q, index1, index2, _, _), (mask, _, _) in zip(cand, res):
        inl = np.flatnonzero(mask)
        out[q] = (index1[inl].tolist(), index2[inl].tolist())
    return out


def match_orb_features(keypiont1, descriptor1, keypoint2, descriptor2, verbose=False):
    """image_process.py:237-272 on the GPU: cross-checked Hamming matching (libptzba ptz_match_hamming), then
    the homography RANSAC inliers (1 px).  Returns (pts1, index1, pts2, index2)."""
    import ptzba
    assert len(keypiont1) >= 4  # assume homography matching
    q, t, _ = ptzba.match_hamming_cross(descriptor1, descriptor2)
    pts1 = np.array([keypiont1[i].pt for i in q], np.float64).reshape(-1, 2)
    pts2 = np.array([keypoint2[j].pt for j in t], np.float64).reshape(-1, 2)
    index1, index2 = q.astype(np.int32), t.astype(np.int32)
    inlier_index = homography_ransac(pts1, pts2, 1.0)
    if verbose:
        print('%d matches passed the homography ransac' % len(inlier_index))
    return pts1[inlier_index, :], index1[inlier_index].tolist(), pts2[inlier_index, :], index2[inlier_index].tolist()


def match_latch_features(keypiont1, descriptor1, keypoint2, descriptor2, verbose=False):
    """image_process.py:275-310: the same cross-checked Hamming matching + RANSAC for LATCH descriptors."""
    return match_orb_features(keypiont1, descriptor1, keypoint2, descriptor2, verbose)


def homography_ransac(points1, points2, reprojection_threshold=0.5, return_matrix=False):
    """image_process.py:418-441 on the GPU (libptzba ptz_homography_ransac: 2000 counter-keyed 4-point
    hypotheses, DLT, most inliers, least-squares refit): RANSAC inlier indices [, homography]."""
    import ptzba
    p1 = np.asarray(points1, np.float64).reshape(-1, 2)
    p2 = np.asarray(points2, np.float64).reshape(-1, 2)
    assert p1.shape[0] == p2.shape[0]
    assert p1.shape[0] >= 4
    mask, H, _ = ptzba.homography_ransac(p1, p2, reprojection_threshold)
    index = [int(i) for i in np.flatnonzero(mask)]
    if return_matrix:
        return index, H
    return index


def _grey_u8(img):
    a = np.asarray(img)
    if a.ndim == 3:  # BGR -> grey, ITU-R BT.601 weights (cv.COLOR_BGR2GRAY)
        a = a[..., 2] * 0.299 + a[..., 1] * 0.587 + a[..., 0] * 0.114
    return np.clip(np.rint(a), 0, 255).astype(np.uint8) if a.dtype != np.uint8 else a


def optical_flow_matching(img, next_img, points, ssd_threshold=20):
    """image_process.py:393-415 on the GPU (libptzba ptz_lk_track: pyramidal LK, 31 x 31 window, 4 levels,
    30 iterations, eps 0.01): indices of the points tracked with err < ssd_threshold and strictly inside
    the image, and their positions in next_img ([m, 2]).  The reference's filter exactly (:408-411): the LK
    status is NOT consulted, so a point that ends in the last pixel column / row (status 0 in ptz_lk_track,
    as in OpenCV) is kept when err and the bounds allow.  A window without texture (smaller structure-
    tensor eigenvalue below the threshold) reports err = inf and is dropped; OpenCV leaves err unset there
    (undefined), the one deliberate deviation."""
    import ptzba
    a, b = _grey_u8(img), _grey_u8(next_img)
    pts = np.asarray(points, np.float32).reshape(-1, 2)
    nxt, status, err = ptzba.lk_track(a, b, pts, win=31)
    h, w = a.shape[0], a.shape[1]
    x, y = nxt[:, 0], nxt[:, 1]
    keep = (err < ssd_threshold) & (x > 0) & (x < w) & (y > 0) & (y < h)
    matched_index = [int(i) for i in np.flatnonzero(keep)]
    return matched_index, np.array([nxt[i] for i in matched_index])


def compute_homography(keypiont1, descriptor1, keypoint2, descriptor2):
    """image_process.py:313-349 on the GPU: kNN-2 L2 matching (ptz_match_knn2), the 0.7 ratio test, then
    the RANSAC homography (1 px).  Returns H [3, 3]; below 9 ratio-test survivors the reference's
    (None, [], None, []) with its warning."""
    import ptzba
    d1 = np.asarray(descriptor1, dtype=np.float32)
    d2 = np.asarray(descriptor2, dtype=np.float32)
    idx, dist = ptzba.match_knn2(d1, d2)
    good = np.flatnonzero(dist[:, 0] < 0.7 * dist[:, 1]) if len(d2) >= 2 else np.zeros(0, np.int64)
    if len(good) <= 8:
        print('warning: match sift features failed, not enough matching')
        return None, [], None, []
    pts1 = np.array([keypiont1[i].pt for i in good], np.float64).reshape(-1, 2)
    pts2 = np.array([keypoint2[j].pt for j in idx[good, 0]], np.float64).reshape(-1, 2)
    _, H = homography_ransac(pts1, pts2, 1.0, return_matrix=True)
    return H


def detect_harris_corner_grid(gray_img, row, column):
    """image_process.py:352-390: per cell of a row x column grid, cv.goodFeaturesToTrack(gray, maxCorners=20,
    qualityLevel=0.2, minDistance=10, mask=cell) -- Shi-Tomasi corners.  The response map and its 3x3 local
    maxima come from the GPU (ptz_corner_min_eig); per cell (the last row / column take the remainder): the
    threshold 0.2 x the cell's maximum response, candidates ordered by response (ties: later pixel first, as
    OpenCV's pointer order), greedily kept when no kept corner lies within 10 px, at most 20.  Returns
    float32 [n, 2] (x, y), cells in row-major order."""
    import ptzba
    g = _grey_u8(gray_img)
    eig, locmax = ptzba.corner_min_eig(g)
    return _corner_grid_select(eig, locmax, row, column)


def _corner_grid_select(eig, locmax, row, column, max_corners=20, quality=0.2, min_distance=10.0):
    h, w = eig.shape
    gh, gw = h // row, w // column
    out = []
    for i in range(row):
        for j in range(column):
            y1, x1 = i * gh, j * gw
            y2 = h if i == row - 1 else y1 + gh
            x2 = w if j == column - 1 else x1 + gw
            cell = eig[y1:y2, x1:x2]
            if cell.size == 0:
                continue
            thr = np.float32(cell.max()) * np.float32(quality)
            ys, xs = np.nonzero(locmax[y1:y2, x1:x2] & (cell > thr))
            if len(ys) == 0:
                continue
            ys, xs = ys + y1, xs + x1
            v = eig[ys, xs]
            order = np.lexsort((-(ys.astype(np.int64) * w + xs), -v))  # response desc, then address desc
            kept = []
            for k in order:
                x, y = float(xs[k]), float(ys[k])
                if all((x - kx) ** 2 + (y - ky) ** 2 >= min_distance * min_distance for kx, ky in kept):
                    kept.append((x, y))
                    if len(kept) == max_corners:
                        break
            out.extend(kept)
    return np.asarray(out, np.float32).reshape(-1, 2)


def good_homography(h):
    """image_process.py:445-461: the reference marks this check as not working and asserts on entry; kept
    so callers behave identically (AssertionError)."""
    assert False, "good_homography: disabled in the reference (image_process.py:447)"


def keypoints_masking(kp, mask):
    """image_process.py:158-175: indices of keypoints whose (int x, int y) pixel has mask == 1."""
    if isinstance(kp, np.ndarray):
        xs = kp[:, 0].astype(np.int64) if len(kp) else np.zeros(0, np.int64)
        ys = kp[:, 1].astype(np.int64) if len(kp) else np.zeros(0, np.int64)
    else:
        xs = np.array([int(k.pt[0]) for k in kp], np.int64)
        ys = np.array([int(k.pt[1]) for k in kp], np.int64)
    if len(xs) == 0:
        return np.ndarray([0], dtype=np.int32)
    keep = np.asarray(mask)[ys, xs] == 1
    return np.flatnonzero(keep).astype(np.int32)


def matching_and_ransac(img1, img2, img1_keypoints, img1_keypoints_index, visualize=False):
    """image_process.py:464-506: LK flow + homography RANSAC -> (inlier kps, inlier ids, outlier ids)."""
    local_matched_index, current_keypoints = optical_flow_matching(img1, img2, img1_keypoints)
    current_keypoints_index = img1_keypoints_index[local_matched_index]
    previous_matched_keypoints = img1_keypoints[local_matched_index]
    local_inlier_index = homography_ransac(previous_matched_keypoints, current_keypoints, reprojection_threshold=0.5)
    inlier_keypoints = current_keypoints[local_inlier_index]
    inlier_index = current_keypoints_index[local_inlier_index]
    outlier_index = np.delete(current_keypoints_index, local_inlier_index, axis=0)
    return inlier_keypoints, inlier_index, outlier_index


def _detect(im, feature_method):
    if feature_method == "sift":
        return detect_compute_sift(im, 1500, False)
    if feature_method == "orb":
        return detect_compute_orb(im, 6000, False)
    if feature_method == "latch":
        return detect_compute_latch(im, 5000, False)
    raise AssertionError(feature_method)


def _match(kp1, des1, kp2, des2, feature_method):
    if feature_method == "sift":
        return match_sift_features(kp1, des1, kp2, des2, False)
    if feature_method == "orb":
        return match_orb_features(kp1, des1, kp2, des2, False)
    return match_latch_features(kp1, des1, kp2, des2, False)


def build_matching_graph(images, image_match_mask=[], feature_method="sift", verbose=False):
    """image_process.py:509-667.  Returns (keypoints, descriptors, points, src_pt_index, dst_pt_index,
    landmark_index, landmark_num) with identical contents and list ordering (built natively by
    correspondence.build_graph; see there for the cap-shuffle replay)."""
    import correspondence
    g = correspondence.build_graph(images, image_match_mask, feature_method, verbose)
    src, dst, lmk = g.lists()
    return g.keypoints, g.descriptors, g.points(), src, dst, lmk, g.n_landmark
