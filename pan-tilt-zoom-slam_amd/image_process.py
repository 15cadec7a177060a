"""
Correspondence front-end hooks + matching-graph bookkeeping (reference: slam_system/image_process.py).

The reference detects SIFT/ORB features and matches them with OpenCV (image_process.py:14-506).
OpenCV is not part of this build (the feature front-end is SURVEY §8f-4, out of scope for the BA
tier), so the front-end functions here are HOOKS: a correspondence source (e.g. synthetic.py's
SyntheticFrontEnd, or an OpenCV wrapper on a machine that has it) assigns them, exactly the way the
reference's own tests monkeypatch them.  Calling an unassigned hook raises.

What this module does implement is the bookkeeping of `build_matching_graph`
(image_process.py:509-667) with the reference's exact semantics:
  * pairs i < j in order, skipped when image_match_mask[i][j] == 0;
  * a pair is kept if it has MORE than 20 matches (`len > min_match_num`, :590);
  * pairs with more than 200 matches are capped by `random.shuffle` of the GLOBAL `random`
    module (:592-597), so a seeded `random` reproduces the reference bit for bit;
  * landmark ids by the first-seen rule (:611-639) — computed natively in libptzba
    (ptzba_build_landmarks), including the count of the reference's "in-consistent matching" warnings.
"""
import random

import numpy as np

import ptzba


class KeyPoint:
    """Minimal stand-in for cv2.KeyPoint: the reference only reads `.pt`."""
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (float(x), float(y))


def _hook(name):
    def f(*a, **k):
        raise NotImplementedError(
            f"image_process.{name} is a front-end hook (OpenCV SIFT/ORB/LK in the reference, image_process.py); "
            f"assign a correspondence source, e.g. synthetic.SyntheticFrontEnd(...).install()")
    f.__name__ = name
    return f


# ---- front-end hooks (assigned by a correspondence source) ----
detect_compute_sift = _hook("detect_compute_sift")              # (im, nfeatures, verbose) -> (kps, des)
detect_compute_orb = _hook("detect_compute_orb")
detect_compute_latch = _hook("detect_compute_latch")
match_sift_features = _hook("match_sift_features")              # (kp1, des1, kp2, des2, pts_array, verbose)
match_orb_features = _hook("match_orb_features")
match_latch_features = _hook("match_latch_features")
optical_flow_matching = _hook("optical_flow_matching")
homography_ransac = _hook("homography_ransac")
draw_matches = None  # optional visualisation hook (bundle_adjustment.py:153-163)


def detect_compute_sift_array(im, nfeatures, norm=True):
    """image_process.py:82-102: keypoints as an [N,2] array, descriptors (L2-normalised) [N,128]."""
    kps, des = detect_compute_sift(im, nfeatures)
    pts = np.array([k.pt for k in kps], dtype=np.float64).reshape(-1, 2)
    des = np.asarray(des)
    if norm and len(des):
        des = (des / np.linalg.norm(des, axis=1).reshape(-1, 1)).astype(np.float64)
    return pts, des


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
    landmark_index, landmark_num) with identical contents and list ordering."""
    assert feature_method in ("sift", "orb", "latch")
    n = len(images)
    if len(image_match_mask) != 0:
        assert len(image_match_mask) == n
        for m in image_match_mask:
            assert len(m) == n
    elif verbose:
        print("Warning: image match mask is NOT used, may have false positive matches!")
    keypoints, descriptors = [], []
    for im in images:
        kp, des = _detect(im, feature_method)
        keypoints.append(kp)
        descriptors.append(des)
    min_match_num, max_match_num = 20, 200
    pairs = []
    for i in range(n):
        for j in range(i + 1, n):
            if len(image_match_mask) != 0 and image_match_mask[i][j] == 0:
                continue
            _, index1, _, index2 = _match(keypoints[i], descriptors[i], keypoints[j], descriptors[j], feature_method)
            assert len(index1) == len(index2)
            if len(index1) > min_match_num:
                if len(index1) > max_match_num:
                    rand_list = list(range(len(index1)))
                    random.shuffle(rand_list)
                    rand_list = rand_list[0:max_match_num]
                    index1 = [index1[k] for k in rand_list]
                    index2 = [index2[k] for k in rand_list]
                pairs.append((i, j, [int(a) for a in index1], [int(b) for b in index2]))
                if verbose:
                    print("%d matches between image: %d and %d" % (len(index1), i, j))
            elif verbose:
                print("no enough matches between image: %d and %d" % (i, j))
    kp_count = [len(k) for k in keypoints]
    lm_lists, n_landmark, n_inconsistent = ptzba.build_landmarks(kp_count, pairs) if pairs else ([], 0, 0)
    if n_inconsistent and verbose:
        print("Warning: %d in-consistent matching results" % n_inconsistent)
    src = [[[] for _ in range(n)] for _ in range(n)]
    dst = [[[] for _ in range(n)] for _ in range(n)]
    lmk = [[[] for _ in range(n)] for _ in range(n)]
    for (i, j, a, b), lm in zip(pairs, lm_lists):
        src[i][j] = a
        dst[i][j] = b
        lmk[i][j] = [int(x) for x in lm]
    points = [np.array([k.pt for k in kps], dtype=np.float64).reshape(-1, 2) for kps in keypoints]
    if verbose:
        print("number of landmark is %d" % n_landmark)
    return keypoints, descriptors, points, src, dst, lmk, n_landmark
