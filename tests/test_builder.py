"""Correspondence -> packed-observation builder (libptzba builder.cpp + correspondence.py),
CPU only.  Bit-exact against the reference's fixtures (tests/golden/ba_*.npz, matching_graph.npz, made by
running bundle_adjustment / build_matching_graph of the reference) and against the running interpreter
for the two interpreter-defined orderings the reference depends on (random.shuffle, set iteration)."""
import random

import numpy as np
import pytest

from conftest import golden


@pytest.mark.parametrize("name", ["ba_4x60", "ba_6x120", "ba_10x200"])
def test_keyframe_features_set_order_bit_exact(name):
    """bundle_adjustment.py:214-248: per-keyframe (local, landmark) lists in set() order."""
    import ptzba
    d = golden(name + ".npz")
    off, loc, glo = ptzba.keyframe_features(int(d["n_pose"]), d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"])
    np.testing.assert_array_equal(off, d["kf_off"])
    np.testing.assert_array_equal(loc, d["kf_local"])
    np.testing.assert_array_equal(glo, d["kf_lmk"])


@pytest.mark.parametrize("name", ["ba_4x60", "ba_10x200"])
def test_pack_records_and_x0_source(name):
    """Records in _compute_residual order and the x0 ray of every landmark from the last match's src
    observation (bundle_adjustment.py:186-195) == the reference's x0."""
    import ptzba
    from oracle import ptz_oracle as orc
    d = golden(name + ".npz")
    n, m = int(d["n_pose"]), int(d["n_landmark"])
    fr, lm, xy, src = ptzba.pack_records(n, d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"], d["points_off"],
                                         d["points"], m)
    np.testing.assert_array_equal(fr[0::2], d["m_i"])
    np.testing.assert_array_equal(fr[1::2], d["m_j"])
    np.testing.assert_array_equal(lm[0::2], d["m_lm"])
    pts, off = d["points"], d["points_off"]
    np.testing.assert_array_equal(xy[0::2], pts[off[d["m_i"]] + d["m_k1"]])
    np.testing.assert_array_equal(xy[1::2], pts[off[d["m_j"]] + d["m_k2"]])
    assert np.all(src >= 0) and np.all(src % 2 == 0)
    ip = d["init_ptz"]
    f = fr[src]
    th, ph = orc.from_image_to_ray(float(d["u"]), float(d["v"]), ip[f, 2], ip[f, 0], ip[f, 1], xy[src, 0], xy[src, 1])
    x0_rays = d["x0"][3 * (n - 1):].reshape(-1, 2)
    np.testing.assert_allclose(np.stack([th, ph], 1), x0_rays, rtol=0, atol=1e-10)


def test_shuffle_replay_matches_interpreter():
    """random.shuffle prefix + generator state afterwards, incl. lengths around powers of two."""
    import ptzba
    rng = np.random.default_rng(3)
    lens = [2, 3, 4, 5, 201, 255, 256, 257, 1023, 1024, 1025, 4096] + rng.integers(2, 3000, 40).tolist()
    for seed in (0, 1, 99):
        random.seed(seed)
        want = []
        for n in lens:
            lst = list(range(n))
            random.shuffle(lst)
            want += lst[:200]
        nxt = random.getrandbits(32)
        random.seed(seed)
        got = ptzba.py_shuffle_prefix(lens, 200)
        np.testing.assert_array_equal(got, want)
        assert random.getrandbits(32) == nxt


def test_set_order_matches_interpreter():
    import ptzba
    rng = np.random.default_rng(5)
    for n, hi in ((0, 1), (1, 1), (7, 3), (5000, 200), (120000, 60000)):
        a = rng.integers(0, hi, n)
        b = rng.integers(0, 4 * hi, n)
        oa, ob = ptzba.set_order_pairs(a, b)
        assert list(zip(oa.tolist(), ob.tolist())) == list(set(zip(a.tolist(), b.tolist())))


def _scene_frontend(n_kf=7, n_rays=700, seed=11):
    import synthetic
    sc = synthetic.make_scene(n_kf, n_rays, 50, 62, seed=seed)
    fe = synthetic.SyntheticFrontEnd(sc, corrupt=3, seed=seed)
    calls = {"detect": 0, "match": 0}

    def det(im, nf=0, verbose=False):
        calls["detect"] += 1
        return fe.detect(im, nf, verbose)

    def mat(*a, **k):
        calls["match"] += 1
        return fe.match(*a, **k)
    return sc, det, mat, calls


def _mask(ptz):
    from util import overlap_pan_angle
    n = len(ptz)
    return [[1 if overlap_pan_angle(ptz[i][2], ptz[i][0], ptz[j][2], ptz[j][0], 1280) > 5 else 0 for j in range(n)]
            for i in range(n)]


def test_cached_graph_equals_full_rebuild():
    """Incremental keyframe sets through a CorrespondenceCache == the reference's full rebuild on every
    call (same ids, same capped matches, same global `random` stream), with each image detected once and
    each pair matched once."""
    import correspondence
    import image_process
    sc, det, mat, calls = _scene_frontend()
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = det, mat
    try:
        cache = correspondence.CorrespondenceCache()
        n_all = len(sc.init_ptz)
        full_matches = 0
        for n in range(2, n_all + 1):
            ims = list(range(n))
            mask = _mask(sc.init_ptz[:n])
            random.seed(1000 + n)
            g_full = correspondence.build_graph(ims, mask, "sift")
            full_state = random.getstate()
            full_matches += sum(mask[i][j] for i in range(n) for j in range(i + 1, n))
            random.seed(1000 + n)
            g = correspondence.build_graph(ims, mask, "sift", cache=cache, keys=[100 + k for k in ims])
            assert random.getstate() == full_state
            for f in ("pair_i", "pair_j", "pair_off", "k1", "k2", "lm", "kp_xy"):
                np.testing.assert_array_equal(getattr(g, f), getattr(g_full, f))
            assert g.n_landmark == g_full.n_landmark and g.n_inconsistent == g_full.n_inconsistent
        assert cache.n_detect == n_all
        assert cache.n_match == sum(_mask(sc.init_ptz)[i][j] for i in range(n_all) for j in range(i + 1, n_all))
        assert calls["match"] == full_matches + cache.n_match
        # sliding window: drop the oldest images, nothing new to detect or match
        cache.retain([100 + k for k in range(3, n_all)])
        before = cache.n_match
        g = correspondence.build_graph(list(range(3, n_all)), _mask(sc.init_ptz[3:]), "sift", cache=cache,
                                       keys=[100 + k for k in range(3, n_all)])
        assert cache.n_match == before and g.n_matches > 0
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved


def test_cache_redetects_changed_image():
    import correspondence
    import image_process
    sc, det, mat, calls = _scene_frontend(4, 400)
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = det, mat
    try:
        cache = correspondence.CorrespondenceCache()
        mask = _mask(sc.init_ptz)
        correspondence.build_graph([0, 1, 2, 3], mask, "sift", cache=cache, keys=[0, 1, 2, 3])
        n0 = cache.n_detect
        # key 3 now shows a different image (frame 2's): re-detected, its pairs re-matched
        correspondence.build_graph([0, 1, 2, 2], mask, "sift", cache=cache, keys=[0, 1, 2, 3])
        assert cache.n_detect == n0 + 1
        # duplicate keys disable the cache for the call rather than mixing images up
        g = correspondence.build_graph([0, 1], [r[:2] for r in mask[:2]], "sift", cache=cache, keys=[5, 5])
        assert cache.n_detect == n0 + 1 and g.n_frames == 2
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved


def test_lazy_keyframe_lists_equal_eager_assembly():
    """bundle_adjustment's keyframes take their feature lists on first use (_KeyframeLists + KeyFrame.set_features_lazy):
    every keyframe's feature_pts / feature_des / landmark_index then equal the eager assembly of
    bundle_adjustment.py:214-248 (keyframe_features' set() order), and has_features() == get_feature_num() > 0
    without forming the lists first.  The vectorised pair mask equals overlap_pan_angle per pair."""
    import bundle_adjustment
    import correspondence
    import image_process
    from key_frame import KeyFrame
    sc, det, mat, calls = _scene_frontend()
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = det, mat
    try:
        n = len(sc.init_ptz)
        mask = _mask(sc.init_ptz)
        from util import overlap_pan_angle_half_fov
        ptz = np.asarray(sc.init_ptz, np.float64)
        half = np.array([overlap_pan_angle_half_fov(fl, 1280) for fl in ptz[:, 2].tolist()])
        ov = np.minimum((ptz[:, 0] + half)[:, None], (ptz[:, 0] + half)[None, :]) - \
            np.maximum((ptz[:, 0] - half)[:, None], (ptz[:, 0] - half)[None, :])
        assert (ov > 5).astype(np.int64).tolist() == mask
        random.seed(5)
        g = correspondence.build_graph(list(range(n)), mask, "sift")
        off, loc, glo = g.keyframe_features()
        lists = bundle_adjustment._KeyframeLists(g)
        for i in range(n):
            kf = KeyFrame(i, i, np.zeros(3), np.eye(3), 640, 360, 0.0, 0.0, 1000.0)
            kf.set_features_lazy(g.keypoints[i], g.descriptors[i], lists, i)
            assert kf.has_features() == (off[i + 1] > off[i])
            np.testing.assert_array_equal(kf.landmark_index, glo[off[i]:off[i + 1]].astype(np.int32))
            assert [k.pt for k in kf.feature_pts] == [g.keypoints[i][q].pt for q in loc[off[i]:off[i + 1]]]
            np.testing.assert_array_equal(kf.feature_des, np.asarray(g.descriptors[i])[loc[off[i]:off[i + 1]]])
            assert kf.get_feature_num() == off[i + 1] - off[i]
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved


@pytest.mark.parametrize("consistent", [True, False])
@pytest.mark.parametrize("wide", [False, True])
def test_keyframe_feature_counts_equal_list_lengths(consistent, wide):
    """ptz_keyframe_feature_counts (the verbose print's list lengths without the set() order: a keyframe x keypoint
    table, or per keyframe a keypoint map when the table is too large (`wide`: keypoint ids past 2^24 / frames), and a
    sort where a keypoint has two landmarks) == the lengths of ptz_keyframe_features' lists."""
    import ptzba
    rng = np.random.default_rng(3)
    n, mi, mj, k1, k2, lm = 12, [], [], [], [], []
    nxt = [0] * n
    for l in range(3000):
        f0 = int(rng.integers(0, n - 2))
        fs = list(range(f0, min(n, f0 + int(rng.integers(2, 5)))))
        ks = {f: nxt[f] for f in fs}
        for f in fs:
            nxt[f] += 1
        for a in range(len(fs)):
            for b in range(a + 1, len(fs)):
                mi.append(fs[a]); mj.append(fs[b]); k1.append(ks[fs[a]]); k2.append(ks[fs[b]]); lm.append(l)
    o = np.lexsort((np.arange(len(mi)), np.array(mj), np.array(mi)))
    mi, mj = np.array(mi, np.int32)[o], np.array(mj, np.int32)[o]
    k1, k2, lm = np.array(k1)[o], np.array(k2)[o], np.array(lm)[o]
    if not consistent:
        lm = lm.copy()
        lm[::97] = rng.integers(0, 3000, len(lm[::97]))  # keypoints seen with two landmarks
    if wide:
        k1 = k1 + (k1 % 7 == 3) * 3_000_000  # sparse large keypoint ids
    off, _, _ = ptzba.keyframe_features(n, mi, mj, k1, k2, lm)
    np.testing.assert_array_equal(ptzba.keyframe_feature_counts(n, mi, mj, k1, k2, lm), np.diff(off))
