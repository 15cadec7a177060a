"""Incremental maps on the GPU BA: scene_map.Map.add_keyframe_with_ba over a growing keyframe
set and RandomForestMap's 10-keyframe sliding window, compared step by step with the reference's own runs
of the same sequences (tests/golden/map_incremental.npz, map_window.npz; make_golden.py gen_maps).
Bit-exact: keyframe order, image indices, feature coordinates and landmark ids (the correspondence cache,
the native cap-shuffle replay and set() order).  Poses/rays: both solvers stop at the same optimum,
1e-5 deg / 2e-3 px apart at most.  The cache must make each image detected once and each pair matched once
(the reference detects and matches everything again on every keyframe)."""
import random

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _scene(n_kf, n_rays, lo, hi, seed):
    import synthetic
    return synthetic.make_scene(n_kf, n_rays, lo, hi, seed=seed)


def _counting_frontend(scene):
    import synthetic
    fe = synthetic.SyntheticFrontEnd(scene)
    calls = {"detect": 0, "match": 0}

    def det(*a, **k):
        calls["detect"] += 1
        return fe.detect(*a, **k)

    def mat(*a, **k):
        calls["match"] += 1
        return fe.match(*a, **k)
    return det, mat, calls


def _compare(step, kfs, rays, d, feat_pos, ray_pos, ang=1e-5, fpx=2e-3):
    sel = np.flatnonzero(d["kf_step"] == step)
    assert [int(k.img) for k in kfs] == d["kf_img"][sel].tolist()
    assert [int(k.img_index) for k in kfs] == d["kf_index"][sel].tolist()
    nfeat_off = np.concatenate([[0], np.cumsum(d["kf_nfeat"])])
    for k, r in zip(kfs, sel):
        a, b = nfeat_off[r], nfeat_off[r + 1]
        pts = k.feature_pts
        xy = np.array([p.pt for p in pts]).reshape(-1, 2) if isinstance(pts, list) else np.asarray(pts).reshape(-1, 2)
        np.testing.assert_array_equal(xy, d["feat_xy"][a:b])
        np.testing.assert_array_equal(np.asarray(k.landmark_index, np.int64), d["feat_lmk"][a:b])
        p = np.array([k.pan, k.tilt, k.f]) - d["kf_ptz"][r]
        assert abs(p[0]) < ang and abs(p[1]) < ang and abs(p[2]) < fpx, (step, k.img, p)
    if rays is not None:
        ro = np.concatenate([[0], np.cumsum(d["ray_n"])])
        want = d["rays"][ro[ray_pos]:ro[ray_pos + 1]]
        assert rays.shape == want.shape
        np.testing.assert_allclose(rays, want, rtol=0, atol=ang)


def test_incremental_map_matches_reference(gpu_available):
    import image_process
    import key_frame
    import scene_map
    d = golden("map_incremental.npz")
    sc = _scene(6, 150, 54, 63, int(d["seed"]))
    np.testing.assert_array_equal(sc.init_ptz, d["init_ptz"])
    det, mat, calls = _counting_frontend(sc)
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = det, mat
    center, rot = np.array([0.0, -10.0, 5.0]), np.eye(3)
    try:
        random.seed(int(d["seed"]))
        m = scene_map.Map("sift")
        ip = sc.init_ptz
        m.add_first_keyframe(key_frame.KeyFrame(0, 100, center, rot, sc.u, sc.v, *ip[0]))
        for k in range(1, 6):
            m.add_keyframe_with_ba(key_frame.KeyFrame(k, 100 + k, center, rot, sc.u, sc.v, *ip[k]), "")
            _compare(k, m.keyframe_list, m.global_ray, d, None, k - 1)
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved
    assert calls["detect"] == 6 < int(d["ref_detect_calls"])
    assert calls["match"] == m.correspondences.n_match < int(d["ref_match_calls"])


def test_sliding_window_map_matches_reference(gpu_available):
    import image_process
    import key_frame
    import scene_map
    d = golden("map_window.npz")
    sc = _scene(12, 160, 50, 66, int(d["seed"]))
    np.testing.assert_array_equal(sc.init_ptz, d["init_ptz"])
    det, mat, calls = _counting_frontend(sc)
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = det, mat
    center, rot = np.array([0.0, -10.0, 5.0]), np.eye(3)
    try:
        random.seed(int(d["seed"]))
        rf = scene_map.RandomForestMap(max_ba_frame=10)
        ip = sc.init_ptz
        for k in range(12):
            rf.add_keyframe(key_frame.KeyFrame(k, 200 + k, center, rot, sc.u, sc.v, *ip[k]))
            _compare(k, rf.keyframe_list, None, d, None, None)
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved
    assert calls["detect"] == 12
    # the window dropped keyframes 0 and 1: their cache entries are gone
    assert all(key[0] >= 202 for key in rf.correspondences.detections)
