"""GPU front-end through the C-ABI: ptz_match_knn2 (cv.BFMatcher().knnMatch(k=2),
image_process.py:191) and ptz_homography_ransac (cv.findHomography RANSAC, image_process.py:433), and
image_process.match_sift_features (:178-234) composed from them, against the oracle restatements
(oracle/ptz_oracle.py knn2 / homography_ransac) on synthetic SIFT-like data; ptz_lk_track
(cv.calcOpticalFlowPyrLK, image_process.py:402) and image_process.optical_flow_matching (:393-415) against
oracle lk_track and the known motion of synthetic textured views (positions within 0.02 px of the oracle:
the GPU pyramid is fp32 and the sums run in another order, so a Newton stop decision near eps = 0.01 px
can differ; err within 1e-3).
Exact: kNN indices and distances (integer-valued descriptors: every fp32 partial sum is exact), the RANSAC
inlier mask and count (same counter-keyed samples; H to 1e-9 relative).  OpenCV itself is not in the image,
so the oracle restates the published algorithms -- parity with cv2 is unpinned; the tests pin the GPU to
the restatement and both to the synthetic ground truth."""
import numpy as np
import pytest

import frontend_data

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n1,n2", [(550, 550), (1, 70), (130, 2), (1500, 1400)])
def test_knn2_matches_oracle(gpu_available, n1, n2):
    import ptzba
    from oracle import ptz_oracle as orc
    rng = np.random.default_rng(n1 + n2)
    a = rng.integers(0, 256, (n1, 128)).astype(np.float32)
    b = rng.integers(0, 256, (n2, 128)).astype(np.float32)
    if n2 > 10:
        b[5] = b[3]  # exact tie: lower index first
        a[0] = b[3]
    idx, dist = ptzba.match_knn2(a, b)
    ridx, rdist = orc.knn2(a, b)
    assert np.array_equal(idx, ridx)
    assert np.array_equal(dist, rdist.astype(np.float32))


@pytest.mark.parametrize("seed,n,frac", [(3, 600, 0.25), (4, 60, 0.4), (5, 2000, 0.1)])
def test_homography_ransac_matches_oracle(gpu_available, seed, n, frac):
    import ptzba
    from oracle import ptz_oracle as orc
    p1, p2, H, inl = frontend_data.homography_points(seed=seed, n=n, outlier_frac=frac)
    mask, Hg, cnt = ptzba.homography_ransac(p1, p2, 1.0, n_hyp=500, seed=seed)
    rmask, rH, rcnt = orc.homography_ransac(p1, p2, 1.0, n_hyp=500, seed=seed)
    assert np.array_equal(mask, rmask) and cnt == rcnt == mask.sum()
    np.testing.assert_allclose(Hg, rH, rtol=0, atol=1e-9 * np.abs(rH).max())
    assert (mask & ~inl).sum() == 0 and (inl & ~mask).sum() <= max(1, n // 200)


def test_match_sift_features_gpu(gpu_available):
    """image_process.match_sift_features (GPU default): ratio test + RANSAC keep the true correspondences
    of two PTZ views and drop the distractors."""
    import image_process
    from oracle import ptz_oracle as orc
    x1, d1, x2, d2, H, truth = frontend_data.two_views(seed=7)
    pts1, i1, pts2, i2 = image_process.match_sift_features(x1, d1, x2, d2, pts_array=True)
    assert len(i1) > 300
    assert all(truth.get(a) == b for a, b in zip(i1, i2))
    # same result as the oracle composition (knn2 -> ratio 0.7 -> RANSAC 1 px)
    ridx, rdist = orc.knn2(d1, d2)
    good = np.flatnonzero(rdist[:, 0] < 0.7 * rdist[:, 1])
    rmask, _, _ = orc.homography_ransac(x1[good], x2[ridx[good, 0]], 1.0, n_hyp=2000, seed=0)
    assert i1 == good[rmask].tolist() and i2 == ridx[good[rmask], 0].tolist()
    np.testing.assert_array_equal(pts1, x1[i1])


def test_homography_ransac_batch_equals_single_calls(gpu_available):
    """ptz_homography_ransac_batch: per set bit for bit the single-call result (masks, counts, H), sets of
    different sizes and outlier fractions in one call."""
    import ptzba
    sets = [frontend_data.homography_points(seed=s, n=n, outlier_frac=f)[:2]
            for s, n, f in ((3, 600, 0.25), (4, 60, 0.4), (5, 2000, 0.1), (6, 4, 0.0), (7, 333, 0.5))]
    got = ptzba.homography_ransac_batch(sets, 1.0, n_hyp=700, seed=11)
    for (p1, p2), (mask, H, cnt) in zip(sets, got):
        m1, H1, c1 = ptzba.homography_ransac(p1, p2, 1.0, n_hyp=700, seed=11)
        assert np.array_equal(mask, m1) and cnt == c1
        assert np.array_equal(H, H1)


def test_match_sift_features_batch_equals_per_pair(gpu_available):
    """image_process.match_sift_features_batch (one kNN-2 per train image, one RANSAC launch): every pair's
    (index1, index2) equals match_sift_features on that pair -- several partners against one shared train set (a
    new keyframe) plus an independent pair and a pair below the ratio-test floor."""
    import image_process
    x0, d0, xn, dn, _, _ = frontend_data.two_views(seed=7)

    class KP:
        def __init__(self, p):
            self.pt = (float(p[0]), float(p[1]))
    kn = [KP(p) for p in xn]
    pairs = []
    for s in (8, 9, 10):
        x1, d1, _, _, _, _ = frontend_data.two_views(seed=s)
        pairs.append(([KP(p) for p in x1], d1, kn, dn))  # shared train set dn
    pairs.append(([KP(p) for p in x0], d0, kn, dn))
    xa, da, xb, db, _, _ = frontend_data.two_views(seed=12)
    pairs.append(([KP(p) for p in xa], da, [KP(p) for p in xb], db))
    pairs.append(([KP(p) for p in xa[:5]], da[:5], kn, dn))  # too few ratio-test survivors
    got = image_process.match_sift_features_batch(pairs)
    for (k1, d1, k2, d2), (a, b) in zip(pairs, got):
        _, i1, _, i2 = image_process.match_sift_features(k1, d1, k2, d2)
        assert list(a) == list(i1) and list(b) == list(i2)
    assert len(got[3][0]) > 300 and got[5] == ([], [])
    # the same pairs with their descriptors resident on the device (ptz_desc_put / ptz_match_knn2_sets): identical
    import ptzba
    ids = {}

    def dev(d):
        if id(d) not in ids:
            ids[id(d)] = (1000 + len(ids), ptzba.desc_put_new(1000 + len(ids), d))
        return ids[id(d)]
    try:
        got_dev = image_process.match_sift_features_batch(pairs, dev_sets=[(dev(p[1]), dev(p[3])) for p in pairs])
        assert got_dev == got
        idx, dist = ptzba.match_knn2(np.concatenate([pairs[0][1], pairs[1][1]]), dn)
        idx2, dist2 = ptzba.match_knn2_sets([ids[id(pairs[0][1])][0], ids[id(pairs[1][1])][0]],
                                            [len(pairs[0][1]), len(pairs[1][1])], ids[id(dn)][0])
        assert np.array_equal(idx, idx2) and np.array_equal(dist, dist2)
        with pytest.raises(ptzba.PtzbaError):  # a row count that disagrees with the resident sets
            ptzba.match_knn2_sets([ids[id(pairs[0][1])][0]], [len(pairs[0][1]) + 1], ids[id(dn)][0])
    finally:
        ptzba.desc_drop([v[0] for v in ids.values()])
    with pytest.raises(ptzba.PtzbaError):  # dropped
        ptzba.match_knn2_sets([1000], [len(pairs[0][1])], 1001)


def test_fused_native_matcher_equals_per_pair(gpu_available, capsys):
    """One train set (a new keyframe) against several resident query sets with keypoint arrays: the batch matcher
    takes ptz_match_sets_ransac (kNN-2, ratio tests, point gathers, RANSAC in one native call) -- per pair exactly
    match_sift_features' (index1, index2), the too-few-survivors pair included (and its warning printed)."""
    import image_process
    import ptzba
    x0, d0, xn, dn, _, _ = frontend_data.two_views(seed=7)
    pairs = []
    for s in (8, 9, 10):
        x1, d1, _, _, _, _ = frontend_data.two_views(seed=s)
        pairs.append((np.asarray(x1, np.float64), d1, np.asarray(xn, np.float64), dn))
    pairs.append((np.asarray(x0, np.float64), d0, np.asarray(xn, np.float64), dn))
    pairs.append((np.asarray(x0[:5], np.float64), d0[:5], np.asarray(xn, np.float64), dn))  # too few survivors
    keys = {}

    def dev(d, k):
        if k not in keys:
            keys[k] = (2000 + len(keys), ptzba.desc_put_new(2000 + len(keys), d))
        return keys[k]
    try:
        dev_sets = [(dev(p[1], q), dev(dn, "train")) for q, p in enumerate(pairs)]
        capsys.readouterr()
        got = image_process.match_sift_features_batch(pairs, dev_sets=dev_sets)
        warned = capsys.readouterr().out.count("not enough matching")
    finally:
        ptzba.desc_drop([v[0] for v in keys.values()])
    for (k1, d1, k2, d2), (a, b) in zip(pairs, got):
        _, i1, _, i2 = image_process.match_sift_features(k1, d1, k2, d2, pts_array=True)
        assert list(a) == list(i1) and list(b) == list(i2)
    assert warned == capsys.readouterr().out.count("not enough matching") >= 1  # the same warnings as per pair
    assert len(got[3][0]) > 300 and got[4] == ([], [])


def test_homography_ransac_hook_signature(gpu_available):
    """homography_ransac(points1, points2, threshold, return_matrix) as image_process.py:418 calls it."""
    import image_process
    p1, p2, H, inl = frontend_data.homography_points(seed=9, n=200)
    idx, Hm = image_process.homography_ransac(p1, p2, 1.0, return_matrix=True)
    assert idx == np.flatnonzero(inl).tolist() or len(set(idx) ^ set(np.flatnonzero(inl).tolist())) <= 1
    np.testing.assert_allclose(Hm, H, rtol=0, atol=2e-3 * np.abs(H).max())


def _lk_points(seed, n, w, h, margin=20):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(margin, w - margin, n), rng.uniform(margin, h - margin, n)], 1).astype(np.float32)


def _lk_compare(I, J, p, **kw):
    import ptzba
    from oracle import ptz_oracle as orc
    nxt, st, err = ptzba.lk_track(I, J, p, **kw)
    rn, rst, rerr = orc.lk_track(I, J, p.astype(np.float64), **kw)
    both = (st == 1) & (rst == 1)
    assert (st != rst).sum() <= max(1, len(p) // 100)
    assert np.abs(nxt[both] - rn[both]).max() < 0.02
    assert np.abs(err[both] - rerr[both]).max() < 1e-3
    same = st == rst  # err is inf exactly where the eigenvalue test failed (a point that left the image keeps it)
    assert np.array_equal(np.isinf(err[same]), np.isinf(rerr[same]))
    return nxt, st, err


@pytest.mark.parametrize("seed,w,h,kw", [(1, 320, 240, {}), (2, 257, 199, {"win": 21, "levels": 3}),
                                         (3, 640, 360, {"levels": 5})])
def test_lk_track_matches_oracle(gpu_available, seed, w, h, kw):
    I, J, H = frontend_data.textured_pair(seed=seed, width=w, height=h, flat_box=(0, 0, 40, 40))
    p = _lk_points(seed, 300, w, h)
    p[:3] = [[15.0, 15.0], [20.0, 22.0], [w - 1.0, h - 1.0]]  # flat patch (fails) and the image corner
    nxt, st, err = _lk_compare(I, J, p, **kw)
    assert st[:2].sum() == 0
    good = st == 1
    e = np.linalg.norm(nxt[good] - frontend_data.apply_h(H, p[good].astype(np.float64)), axis=1)
    assert good.mean() > 0.9 and np.median(e) < 0.06


def test_lk_track_1080p_known_motion(gpu_available):
    """Full-size frame (1920 x 1080, the stream's size), 2000 points: tracked against the true motion."""
    import ptzba
    I, J, H = frontend_data.textured_pair(seed=4, width=1920, height=1080, f=2500.0, d_pan=0.25, d_tilt=0.1)
    p = _lk_points(4, 2000, 1920, 1080, margin=30)
    nxt, st, err = ptzba.lk_track(I, J, p)
    e = np.linalg.norm(nxt - frontend_data.apply_h(H, p.astype(np.float64)), axis=1)
    assert st.all() and np.median(e) < 0.05 and np.percentile(e, 99) < 0.3 and err.max() < 8
    # the oracle on a subset
    _lk_compare(I, J, p[:100])


def test_lk_track_edge_cases(gpu_available):
    import ptzba
    I, J, _ = frontend_data.textured_pair(seed=5)
    nxt, st, err = ptzba.lk_track(I, J, np.zeros((0, 2), np.float32))
    assert nxt.shape == (0, 2) and st.shape == (0,)
    flat = np.full((64, 64), 90, np.uint8)
    nxt, st, err = ptzba.lk_track(flat, flat, np.array([[30.0, 30.0]], np.float32))
    assert st[0] == 0 and np.isinf(err[0])
    with pytest.raises(ptzba.PtzbaError):
        ptzba.lk_track(I, J, np.array([[5.0, 5.0]], np.float32), win=32)
    with pytest.raises(ValueError):
        ptzba.lk_track(I, J[:10], np.array([[5.0, 5.0]], np.float32))


def test_optical_flow_matching_gpu(gpu_available):
    """image_process.optical_flow_matching (GPU default) as image_process.py:393-415 calls it: points with
    err < 20 strictly inside the image, in order, and their next positions; colour input converts to grey."""
    import image_process
    from oracle import ptz_oracle as orc
    I, J, H = frontend_data.textured_pair(seed=6, width=480, height=270, d_pan=1.2)
    p = _lk_points(6, 400, 480, 270, margin=2).astype(np.float64)
    idx, nxt = image_process.optical_flow_matching(I, J, p)
    rn, rst, rerr = orc.lk_track(I, J, p)
    # the reference's filter (image_process.py:408-411): err and the bounds, the LK status is not consulted
    keep = (rerr < 20) & (rn[:, 0] > 0) & (rn[:, 0] < 480) & (rn[:, 1] > 0) & (rn[:, 1] < 270)
    assert len(set(idx) ^ set(np.flatnonzero(keep).tolist())) <= 2
    assert nxt.shape == (len(idx), 2) and idx == sorted(idx)
    idx3, nxt3 = image_process.optical_flow_matching(np.dstack([I] * 3), np.dstack([J] * 3), p)
    assert idx3 == idx and np.array_equal(nxt3, nxt)


def test_lk_edge_points_follow_reference_filter(gpu_available):
    """A point that ends in the last pixel column / row: ptz_lk_track reports status 0 (outside the
    [0, w-1] sample range, as OpenCV), but the reference keeps any point with err < 20 and 0 < x < w,
    0 < y < h whatever the status (image_process.py:408-411) -- so optical_flow_matching keeps it; a point
    on a textureless window (err = inf) and one that ends past the border are dropped."""
    import image_process
    import ptzba
    I, _, _ = frontend_data.textured_pair(seed=7, width=320, height=240)
    I = I.copy()
    I[100:140, 0:60] = 90  # a flat patch: the eigenvalue test fails there
    p = np.array([[319.5, 120.0],   # last column, inside (w-1, w): status 0, kept by the reference filter
                  [160.0, 239.4],   # last row
                  [318.0, 60.0],    # inside, status 1
                  [30.0, 120.0],    # flat window: err = inf, dropped
                  [100.0, 100.0]], np.float32)
    nxt, st, err = ptzba.lk_track(I, I, p)
    assert st.tolist() == [0, 0, 1, 0, 1], st
    assert np.all(err[[0, 1, 2, 4]] < 1e-3) and np.isinf(err[3])
    idx, pts = image_process.optical_flow_matching(I, I, p.astype(np.float64))
    assert idx == [0, 1, 2, 4], idx
    np.testing.assert_allclose(pts, nxt[[0, 1, 2, 4]])


def _sift_match(kg, ko):
    """index pairs (gpu, oracle) of keypoints at the same place and orientation"""
    pairs = []
    for i, k in enumerate(ko):
        d = np.abs(kg[:, :2] - k[:2]).max(1) + np.minimum(np.abs(kg[:, 3] - k[3]), 360 - np.abs(kg[:, 3] - k[3])) / 360
        j = int(np.argmin(d)) if len(kg) else -1
        if j >= 0 and d[j] < 2e-3:
            pairs.append((j, i))
    return np.array(pairs, np.int64).reshape(-1, 2)


@pytest.mark.parametrize("seed,w,h", [(2, 192, 144), (3, 257, 181)])
def test_sift_matches_oracle(gpu_available, seed, w, h):
    """ptz_sift against the oracle restatement: the float32 pyramid is bit-identical (no contraction, same
    operation order) and the fp64 refinement follows the same evaluation order, so the keypoint set, positions,
    sizes and responses agree exactly; angles to 1e-3 deg (atan2 / exp of different libraries); descriptors
    (rounded integers of a renormalised histogram summed in another order) within 1, identical for >= 99 %
    of keypoints (measured: 100 %, profiles/r02_sift_check.txt)."""
    import ptzba
    from oracle import ptz_oracle as orc
    I, _, _ = frontend_data.textured_pair(seed=seed, width=w, height=h, d_pan=0.5, f=400.0)
    kg, rg, dg = ptzba.sift(I, 0)
    ko, ro, do = orc.sift_detect_compute(I, 0)
    assert len(kg) == len(ko) > 50
    pr = _sift_match(kg, ko)
    assert len(pr) == len(ko)
    assert np.array_equal(kg[pr[:, 0], :3], ko[pr[:, 1], :3]) and np.array_equal(rg[pr[:, 0]], ro[pr[:, 1]])
    da = np.abs(kg[pr[:, 0], 3] - ko[pr[:, 1], 3])
    assert np.minimum(da, 360 - da).max() < 1e-3
    dd = np.abs(dg[pr[:, 0]] - do[pr[:, 1]])
    assert dd.max() <= 1 and np.mean(dd.max(1) == 0) >= 0.99
    assert np.all(np.diff(rg) <= 0)


def test_sift_same_image_reuses_pyramid(gpu_available, monkeypatch):
    """A call on the image of the previous call reuses its pyramid and oriented keypoints (a stream detects a frame
    with 500 features, then again with 1500 when it becomes a keyframe): the results equal fresh detections
    (PTZ_SIFT_REUSE=0), and a changed image of the same size is detected afresh."""
    import ptzba
    I, J, _ = frontend_data.textured_pair(seed=5, width=320, height=240, d_pan=0.7, f=450.0)
    monkeypatch.setenv("PTZ_SIFT_REUSE", "0")
    fresh = {(k, n): ptzba.sift(X, n) for k, X in (("I", I), ("J", J)) for n in (50, 0, 200)}
    monkeypatch.setenv("PTZ_SIFT_REUSE", "1")
    for k, X, n in (("I", I, 50), ("I", I, 0), ("I", I, 200), ("J", J, 200), ("J", J, 50), ("I", I, 0)):
        got = ptzba.sift(X.copy(), n)  # a copy: reuse is decided by content, not by the array object
        for a, b in zip(got, fresh[(k, n)]):
            assert np.array_equal(a, b)
    K = I.copy()
    K[7, 11] ^= 1  # one pixel differs: a new detection
    monkeypatch.setenv("PTZ_SIFT_REUSE", "0")
    want = ptzba.sift(K, 0)
    monkeypatch.setenv("PTZ_SIFT_REUSE", "1")
    ptzba.sift(I, 0)
    for a, b in zip(ptzba.sift(K, 0), want):
        assert np.array_equal(a, b)


def test_sift_front_end_recovers_homography(gpu_available):
    """The whole GPU front-end on two 640 x 360 textured views: SIFT (ptz_sift) -> kNN-2 + ratio test ->
    homography RANSAC (image_process.match_sift_features) recovers the true PTZ homography."""
    import image_process
    I, J, H = frontend_data.textured_pair(seed=7, width=640, height=360, d_pan=1.5, d_tilt=-0.5, f=900.0, df=12.0)
    k1, d1 = image_process.detect_compute_sift(I, 1500)
    k2, d2 = image_process.detect_compute_sift(J, 1500)
    assert 200 < len(k1) <= 1500 and d1.shape == (len(k1), 128) and d1.dtype == np.float32
    pts1, i1, pts2, i2 = image_process.match_sift_features(k1, d1, k2, d2)
    assert len(i1) >= 100
    err = np.linalg.norm(frontend_data.apply_h(H, pts1) - pts2, axis=1)
    assert np.median(err) < 0.2 and err.max() < 1.5
    _, Hm = image_process.homography_ransac(pts1, pts2, 1.0, return_matrix=True)
    probe = np.array([[100.0, 80.0], [540.0, 300.0], [320.0, 180.0]])
    assert np.abs(frontend_data.apply_h(Hm, probe) - frontend_data.apply_h(H, probe)).max() < 0.5


def test_sift_hooks_signature(gpu_available):
    """detect_compute_sift(im, nfeatures, verbose) / detect_sift(im, nfeatures) / detect_compute_sift_array as
    image_process.py:14-102 define them; colour input is converted to grey; nfeatures caps the count."""
    import image_process
    I, _, _ = frontend_data.textured_pair(seed=8, width=320, height=200, f=500.0)
    kps, des = image_process.detect_compute_sift(I, 50)
    assert len(kps) == 50 and des.shape == (50, 128) and all(hasattr(k, "pt") for k in kps)
    pts = image_process.detect_sift(np.dstack([I] * 3), 50)
    assert pts.shape == (50, 2) and np.allclose(pts, [k.pt for k in kps])
    arr, ades = image_process.detect_compute_sift_array(I, 50)
    assert arr.shape == (50, 2) and np.allclose(np.linalg.norm(ades, axis=1), 1.0)


@pytest.mark.parametrize("nbytes", [32, 64, 30])
def test_hamming_cross_matches_oracle(gpu_available, nbytes):
    """ptz_match_hamming (cv.BFMatcher(NORM_HAMMING, crossCheck=True)) == the oracle, ties included."""
    import ptzba
    from oracle import ptz_oracle as orc
    x1, d1, x2, d2, H, truth = frontend_data.binary_views(seed=nbytes, nbytes=nbytes)
    d2[7] = d2[3]  # an exact tie on the train side
    q, t, d = ptzba.match_hamming_cross(d1, d2)
    rq, rt, rd = orc.hamming_cross(d1, d2)
    assert np.array_equal(q, rq) and np.array_equal(t, rt) and np.array_equal(d, rd)
    assert sum(truth.get(int(a)) == int(b) for a, b in zip(q, t)) >= 290


def test_match_orb_features_gpu(gpu_available):
    """image_process.match_orb_features / match_latch_features (GPU default): cross-checked Hamming matching +
    RANSAC keep the true correspondences of two PTZ views and drop the distractors."""
    import image_process
    x1, d1, x2, d2, H, truth = frontend_data.binary_views(seed=11)
    k1 = [image_process.KeyPoint(*p) for p in x1]
    k2 = [image_process.KeyPoint(*p) for p in x2]
    for fn in (image_process.match_orb_features, image_process.match_latch_features):
        pts1, i1, pts2, i2 = fn(k1, d1, k2, d2)
        assert len(i1) >= 280 and all(truth.get(a) == b for a, b in zip(i1, i2))
        np.testing.assert_allclose(pts1, x1[i1])


@pytest.mark.parametrize("seed,w,h", [(11, 320, 240), (12, 257, 131), (13, 1280, 720)])
def test_corner_min_eig_matches_oracle(gpu_available, seed, w, h):
    """ptz_corner_min_eig (cv.cornerMinEigenVal, blockSize 3, ksize 3 -- goodFeaturesToTrack's measure) equals the
    oracle's float32 restatement bit for bit, and so do the 3x3 local-maximum candidates (parity vs cv2 unpinned:
    cv2 cannot run here)."""
    import ptzba
    from oracle import ptz_oracle as orc
    I, _, _ = frontend_data.textured_pair(seed=seed, width=w, height=h)
    eig, loc = ptzba.corner_min_eig(I)
    reig, rloc = orc.corner_min_eig(I)
    assert eig.shape == (h, w) and eig.dtype == np.float32
    np.testing.assert_array_equal(eig, reig)
    np.testing.assert_array_equal(loc, rloc)
    assert loc.sum() > 0 and not loc[0].any() and not loc[:, -1].any()


def test_detect_harris_corner_grid(gpu_available):
    """image_process.detect_harris_corner_grid (image_process.py:352-390): per grid cell at most 20 corners, each
    inside its cell, pairwise >= 10 px apart within the cell, responses above 0.2 x the cell maximum and in
    decreasing order; a flat image gives none.  compute_homography / good_homography keep the reference's
    behaviour."""
    import image_process
    from oracle import ptz_oracle as orc
    I, _, _ = frontend_data.textured_pair(seed=14, width=640, height=360)
    pts = image_process.detect_harris_corner_grid(I, 3, 4)
    assert pts.dtype == np.float32 and pts.ndim == 2 and pts.shape[1] == 2 and len(pts) > 12
    eig, _ = orc.corner_min_eig(I)
    gh, gw = 360 // 3, 640 // 4
    cells = (pts[:, 1] // gh).astype(int) * 4 + (pts[:, 0] // gw).astype(int)
    assert np.all(np.diff(cells) >= 0)  # row-major cells
    for c in np.unique(cells):
        p = pts[cells == c]
        assert len(p) <= 20
        i, j = divmod(int(c), 4)
        thr = eig[i * gh:(i + 1) * gh, j * gw:(j + 1) * gw].max() * np.float32(0.2)
        v = eig[p[:, 1].astype(int), p[:, 0].astype(int)]
        assert np.all(v > thr) and np.all(np.diff(v) <= 0)
        d = np.linalg.norm(p[:, None] - p[None], axis=2) + np.eye(len(p)) * 1e9
        assert d.min() >= 10.0
    assert len(image_process.detect_harris_corner_grid(np.full((120, 160), 77, np.uint8), 2, 2)) == 0
    with pytest.raises(AssertionError):
        image_process.good_homography(np.eye(3))


@pytest.mark.parametrize("seed,w,h,nf,kind", [(21, 320, 240, 500, "orb"), (22, 257, 181, 300, "orb"),
                                              (23, 320, 240, 500, "latch"), (24, 640, 360, 1500, "orb")])
def test_orb_matches_oracle(gpu_available, seed, w, h, nf, kind):
    """ptz_orb against the oracle restatement (OpenCV's ORB pipeline with generated sampling tables; parity
    with cv2 unpinned): the integer stages (pyramid, FAST, suppression, Sobel sums, moments) and the fp32
    Harris response follow the same operations, so the keypoint set, positions, sizes, octaves and responses
    agree exactly; angles to 1e-6 deg (atan2 of two libraries); descriptors bit for bit."""
    import ptzba
    from oracle import ptz_oracle as orc
    I, _, _ = frontend_data.textured_pair(seed=seed, width=w, height=h, d_pan=0.5, f=400.0)
    kg, dg = ptzba.orb(I, nf, kind)
    ko, do = orc.orb_detect_compute(I, nf, kind)
    assert len(kg) == len(ko) > 50
    assert np.array_equal(kg[:, [0, 1, 2, 4, 5]], ko[:, [0, 1, 2, 4, 5]])
    da = np.abs(kg[:, 3].astype(np.float64) - ko[:, 3])
    assert np.minimum(da, 360 - da).max() < 1e-3
    assert dg.shape == (len(kg), 64 if kind == "latch" else 32)
    assert np.array_equal(dg, do)
    per = orc.orb_level_counts(nf)
    for l in range(8):  # retain-best: n_l per level plus ties at the cut
        assert (kg[:, 5] == l).sum() >= min(per[l], (ko[:, 5] == l).sum())


def test_orb_front_end_recovers_homography(gpu_available):
    """ORB / LATCH detection (image_process.detect_compute_orb / detect_compute_latch, GPU) -> cross-checked
    Hamming matching + RANSAC (match_orb_features / match_latch_features) on two 640 x 360 views recovers the
    true PTZ homography; nfeatures caps the count as the reference's truncation does."""
    import image_process
    I, J, H = frontend_data.textured_pair(seed=9, width=640, height=360, d_pan=1.2, d_tilt=-0.4, f=900.0, df=6.0)
    for det, match, nb in ((image_process.detect_compute_orb, image_process.match_orb_features, 32),
                           (image_process.detect_compute_latch, image_process.match_latch_features, 64)):
        k1, d1 = det(I, 1500)
        k2, d2 = det(J, 1500)
        assert 300 < len(k1) <= 1500 and d1.shape == (len(k1), nb) and d1.dtype == np.uint8
        assert all(hasattr(k, "pt") and hasattr(k, "octave") for k in k1)
        pts1, i1, pts2, i2 = match(k1, d1, k2, d2)
        assert len(i1) >= 60, (det.__name__, len(i1))
        err = np.linalg.norm(frontend_data.apply_h(H, pts1) - pts2, axis=1)
        assert np.median(err) < 1.0, (det.__name__, np.median(err))
    kc, dc = image_process.detect_compute_orb(I, 100)
    assert len(kc) == 100 and dc.shape == (100, 32)


@pytest.mark.parametrize("n1,n2,vmax", [(1000, 1500, 256), (37, 70, 256), (130, 1, 256), (300, 400, 2048)])
def test_knn2_matrix_core_sets_equal_fp32_pair(gpu_available, monkeypatch, n1, n2, vmax):
    """ptz_match_knn2_sets on integer-valued 128-d descriptor sets (SIFT's) runs k_knn2_mf (f16 MFMA dot products,
    exact integer distances, running top 2 per lane): the same indices and distances, bit for bit, as the fp32
    k_sqdist + k_top2 pair (ptz_match_knn2, and the sets path with PTZ_KNN_MF=0) -- duplicated train rows included
    (ties to the lower index), ragged sizes, a single train row.  Integers beyond 255 (vmax 2048) would leave the
    f16 sums inexact: the sets path then takes the fp32 pair by itself, still bit for bit match_knn2."""
    import ptzba
    rng = np.random.default_rng(n1 + n2)
    q = rng.integers(0, vmax, (n1, 128)).astype(np.float32)
    t = rng.integers(0, vmax, (n2, 128)).astype(np.float32)
    if n2 > 10:
        t[5] = t[3]          # an exact tie between two train rows
        q[:4] = t[[3, 7, 7, 9]]  # distance-0 queries
    qa, qb = q[: n1 // 2], q[n1 // 2:]
    ref_i, ref_d = ptzba.match_knn2(q, t)
    keys = [501, 502, 503]
    try:
        ptzba.desc_put_new(keys[0], qa)
        ptzba.desc_put_new(keys[1], qb)
        ptzba.desc_put_new(keys[2], t)
        for mf in ("1", "0"):
            monkeypatch.setenv("PTZ_KNN_MF", mf)
            i, d = ptzba.match_knn2_sets(keys[:2], [len(qa), len(qb)], keys[2])
            assert np.array_equal(i, ref_i) and np.array_equal(d, ref_d), mf
    finally:
        ptzba.desc_drop(keys)


def test_knn2_sets_with_empty_sets(gpu_available):
    """A keyframe without SIFT keypoints: an empty train set gives every query (-1, -1) at infinite distance, and an
    empty query set gives no rows -- whatever column count the empty arrays carry (round 4 failed with 'query set has
    dim 128, train 1')."""
    import ptzba
    rng = np.random.default_rng(7)
    q = rng.integers(0, 256, (20, 128)).astype(np.float32)
    t = rng.integers(0, 256, (30, 128)).astype(np.float32)
    keys = [601, 602, 603, 604]
    try:
        ptzba.desc_put_new(keys[0], q)
        ptzba.desc_put_new(keys[1], np.zeros((0, 128), np.float32))
        ptzba.desc_put_new(keys[2], [])
        ptzba.desc_put_new(keys[3], t)
        for empty_train in (keys[1], keys[2]):
            i, d = ptzba.match_knn2_sets([keys[0]], [len(q)], empty_train)
            assert i.shape == (20, 2) and np.all(i == -1) and np.all(np.isinf(d))
        i, d = ptzba.match_knn2_sets([keys[1], keys[0]], [0, len(q)], keys[3])
        ri, rd = ptzba.match_knn2(q, t)
        assert np.array_equal(i, ri) and np.array_equal(d, rd)
        i, d = ptzba.match_knn2_sets([keys[1]], [0], keys[3])
        assert i.shape == (0, 2) and d.shape == (0, 2)
    finally:
        ptzba.desc_drop(keys)
