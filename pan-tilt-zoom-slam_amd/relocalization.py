"""
Relocalisation (reference: slam_system/relocalization.py) — same functions and call order.

`relocalization_camera(map, img, pose)` picks the keyframe with the most feature matches, re-matches
it, back-projects the keyframe's matched points to rays with the keyframe's pose, and refines the lost
camera's (pan, tilt, f) with the rays fixed (relocalization.py:104-186).  The geometry runs on the GPU:
rays with the batched `from_image_to_ray` kernel, the pose with `ptz_refine_poses` (the whole
Levenberg-Marquardt loop on the device, relocalization.py:186's least_squares).  Detection and
matching are the image_process front-end hooks, as everywhere in this build.
"""
import numpy as np

import image_process
import ptzba
from image_process import keypoints_masking

_BOX = (slice(13, 51), slice(303, 976))  # relocalization.py:50-51, 110-111: scoreboard region


def _mask():
    m = np.ones([720, 1280])
    m[_BOX] = 0
    return m


def _compute_residual(pose, rays, points, u, v):
    """relocalization.py:22-40 (GPU projection): interleaved reprojection errors."""
    rays = np.asarray(rays, np.float64).reshape(-1, 2)
    points = np.asarray(points, np.float64).reshape(-1, 2)
    n = len(rays)
    x, y = ptzba.ray_to_image(u, v, np.full(n, pose[2]), np.full(n, pose[0]), np.full(n, pose[1]), rays[:, 0],
                              rays[:, 1])
    return np.stack([x - points[:, 0], y - points[:, 1]], 1).reshape(-1)


def _detect(img, n, feature_method):
    if feature_method == 'sift':
        kp, des = image_process.detect_compute_sift_array(img, n, norm=False)
        keep = keypoints_masking(kp, _mask())
        return kp[keep], des[keep]
    if feature_method == 'orb':
        return image_process.detect_compute_orb(img, 6000)
    if feature_method == 'latch':
        return image_process.detect_compute_latch(img, 5000)
    raise AssertionError(feature_method)


def _match(kp1, des1, kp2, des2, feature_method):
    if feature_method == 'sift':
        return image_process.match_sift_features(kp1, des1, kp2, des2, pts_array=True)
    if feature_method == 'orb':
        return image_process.match_orb_features(kp1, des1, kp2, des2)
    return image_process.match_latch_features(kp1, des1, kp2, des2)


def _recompute_matching_ray(keyframe, img, feature_method):
    """relocalization.py:43-101: points in img and the keyframe's matched points as rays."""
    kp, des = _detect(img, 1000, feature_method)
    kkp, kdes = _detect(keyframe.img, 1000, feature_method)
    pt1, index1, pt2, index2 = _match(kp, des, kkp, kdes, feature_method)
    if pt2 is None or len(index2) == 0:
        return np.ndarray([0, 2]), np.ndarray([0, 2])
    pt2 = np.asarray(pt2, np.float64).reshape(-1, 2)
    n = len(pt2)
    th, ph = ptzba.image_to_ray(keyframe.u, keyframe.v, np.full(n, keyframe.f), np.full(n, keyframe.pan),
                                np.full(n, keyframe.tilt), pt2[:, 0], pt2[:, 1])
    return np.asarray(pt1, np.float64).reshape(-1, 2), np.stack([th, ph], 1)


def relocalization_camera(map, img, pose, ftol=1e-4):
    """relocalization.py:104-186: the corrected camera pose [3] (or `pose` when no keyframe matches)."""
    kp, des = _detect(img, 300, map.feature_method)
    nearest_keyframe, max_matched_num = -1, 0
    for i, keyframe in enumerate(map.keyframe_list):
        keyframe_kp, keyframe_des = _detect(keyframe.img, 300, map.feature_method)
        if len(keyframe_kp) == 0:
            continue
        pt1, index1, pt2, index2 = _match(keyframe_kp, keyframe_des, kp, des, map.feature_method)
        if index1 is not None and len(index1) > max_matched_num:
            max_matched_num = len(index1)
            nearest_keyframe = i
    if nearest_keyframe == -1:
        print("No matching keyframe!")
        return pose
    keyframe = map.keyframe_list[nearest_keyframe]
    points, rays = _recompute_matching_ray(keyframe, img, map.feature_method)
    if len(rays) == 0:
        return pose
    ptz, cost, its, status = ptzba.refine_poses(keyframe.u, keyframe.v, np.asarray(pose, np.float64)[None], rays,
                                                points, ftol=ftol)
    return ptz[0]
