"""CPU checks of the front-end oracle (oracle/ptz_oracle.py knn2 / homography_ransac / lk_track, test
infrastructure): the kNN restatement against an explicit per-query sort, the RANSAC restatement against the
ground truth of synthetic correspondences, the LK restatement's pyramid / gradient kernels against known
answers and its tracks against the known motion of synthetic textured views (the GPU kernels are compared
with these in test_gpu_frontend.py)."""
import numpy as np

import frontend_data


def test_knn2_matches_explicit_sort():
    from oracle import ptz_oracle as orc
    rng = np.random.default_rng(1)
    a = rng.integers(0, 4, (50, 8)).astype(np.float32)  # many ties
    b = rng.integers(0, 4, (70, 8)).astype(np.float32)
    idx, dist = orc.knn2(a, b)
    for i in range(len(a)):
        d = ((a[i].astype(np.float64) - b) ** 2).sum(1)
        order = sorted(range(len(b)), key=lambda j: (d[j], j))[:2]
        assert idx[i].tolist() == order
        np.testing.assert_allclose(dist[i], np.sqrt(d[order]))


def test_ransac_oracle_recovers_truth():
    from oracle import ptz_oracle as orc
    p1, p2, H, inl = frontend_data.homography_points(seed=2, n=300)
    mask, Hh, cnt = orc.homography_ransac(p1, p2, 1.0, n_hyp=300, seed=5)
    assert cnt == mask.sum() and np.array_equal(mask, inl)
    np.testing.assert_allclose(Hh, H, rtol=0, atol=1e-3 * np.abs(H).max())


def test_pyr_down_and_scharr_known_answers():
    from oracle import ptz_oracle as orc
    # a constant image stays constant; a linear ramp keeps its slope (x2 per level) away from the border
    assert np.allclose(orc.pyr_down(np.full((9, 13), 7.0)), 7.0)
    assert orc.pyr_down(np.zeros((9, 13))).shape == (5, 7)
    yy, xx = np.mgrid[0:20, 0:30].astype(np.float64)
    ramp = 3.0 * xx - 2.0 * yy
    d = orc.pyr_down(ramp)
    assert np.allclose(d[2:-2, 2:-2], 3.0 * 2 * np.mgrid[0:10, 0:15][1][2:-2, 2:-2] - 2.0 * 2 * np.mgrid[0:10, 0:15][0][2:-2, 2:-2])
    gx, gy = orc.scharr(ramp)
    assert np.allclose(gx[1:-1, 1:-1], 3.0) and np.allclose(gy[1:-1, 1:-1], -2.0)  # Scharr / 32 = the slope
    # bilinear sampling reproduces a plane exactly and clamps outside
    assert np.allclose(orc.bilinear(ramp, np.array([3.25, -5.0]), np.array([4.5, 2.0])), [3 * 3.25 - 9.0, -4.0])


def test_lk_oracle_tracks_known_motion():
    """lk_track on two textured views a PTZ homography apart (9 px / 5 px motion): every interior point is
    tracked, median error vs the true motion < 0.05 px, all < 0.5 px; a flat (textureless) patch fails."""
    from oracle import ptz_oracle as orc
    I, J, H = frontend_data.textured_pair(seed=1, flat_box=(240, 150, 320, 240))
    rng = np.random.default_rng(0)
    p = np.stack([rng.uniform(20, 230, 200), rng.uniform(20, 140, 200)], 1)
    flat = np.array([[285.0, 200.0], [290.0, 205.0]])
    nxt, st, err = orc.lk_track(I, J, np.r_[p, flat])
    e = np.linalg.norm(nxt[:200] - frontend_data.apply_h(H, p), axis=1)
    assert st[:200].all() and np.median(e) < 0.05 and e.max() < 0.5 and err[:200].max() < 5
    assert not st[200:].any() and np.isinf(err[200:]).all()


def test_sift_oracle_matches_under_known_motion():
    """sift_detect_compute on two textured views a PTZ homography apart: the ratio-test matches of its
    descriptors land within 1 px of the true motion; keypoints are ordered by response and cut to nfeatures."""
    from oracle import ptz_oracle as orc
    I, J, H = frontend_data.textured_pair(seed=2, width=192, height=144, d_pan=0.5, f=400.0)
    kp1, r1, d1 = orc.sift_detect_compute(I, 80)
    kp2, r2, d2 = orc.sift_detect_compute(J, 80)
    assert len(kp1) == 80 and np.all(np.diff(r1) <= 0)
    assert np.all((d1 >= 0) & (d1 <= 255)) and np.array_equal(d1, np.rint(d1))
    idx, dist = orc.knn2(d1, d2)
    good = np.flatnonzero(dist[:, 0] < 0.7 * dist[:, 1])
    err = np.linalg.norm(frontend_data.apply_h(H, kp1[good, :2].astype(np.float64)) - kp2[idx[good, 0], :2], axis=1)
    assert len(good) >= 30 and np.mean(err < 1.0) > 0.9


def test_sift_gaussian_weights_and_border():
    from oracle import ptz_oracle as orc
    w = orc.sift_gauss_kernel(1.6)
    assert len(w) == 15 and abs(float(w.sum()) - 1) < 1e-6 and np.allclose(w, w[::-1])
    assert orc._refl101(np.array([-3, -1, 0, 4, 5, 7, 9]), 5).tolist() == [3, 1, 0, 4, 3, 1, 1]


def test_hamming_cross_oracle_matches_bruteforce():
    from oracle import ptz_oracle as orc
    rng = np.random.default_rng(3)
    a = rng.integers(0, 4, (40, 4), dtype=np.uint8)  # many ties
    b = rng.integers(0, 4, (55, 4), dtype=np.uint8)
    q, t, d = orc.hamming_cross(a, b)
    pc = lambda x, y: sum(bin(int(u) ^ int(v)).count("1") for u, v in zip(x, y))
    D = np.array([[pc(x, y) for y in b] for x in a])
    nn12 = [min(range(len(b)), key=lambda j: (D[i, j], j)) for i in range(len(a))]
    nn21 = [min(range(len(a)), key=lambda i: (D[i, j], i)) for j in range(len(b))]
    exp = [i for i in range(len(a)) if nn21[nn12[i]] == i]
    assert q.tolist() == exp and t.tolist() == [nn12[i] for i in exp] and d.tolist() == [D[i, nn12[i]] for i in exp]


def test_orb_oracle_building_blocks():
    """The ORB restatement's pieces against first principles: FAST scores equal a per-pixel brute force of
    the corner definition (largest t with 9 contiguous circle pixels all > p + t or all < p - t), the
    resize is the identity at scale 1 and exact on constant images, the per-level split sums to nfeatures,
    the sampling tables are in range, and the umax rows are OpenCV's for a 31-px patch."""
    from oracle import ptz_oracle as orc
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (24, 26)).astype(np.uint8)
    img[8:16, 8:16] = 250
    s = orc.fast_score(img, 20)
    circ = list(zip(orc._FAST_DX, orc._FAST_DY))
    for y in range(3, 21):
        for x in range(3, 23):
            p = int(img[y, x])
            best = 0
            for t in range(20, 256):
                ok = False
                for k in range(16):
                    arc = [int(img[y + circ[(k + m) % 16][1], x + circ[(k + m) % 16][0]]) for m in range(9)]
                    if all(v > p + t for v in arc) or all(v < p - t for v in arc):
                        ok = True
                        break
                if not ok:
                    break
                best = t
            assert s[y, x] == best, (x, y, s[y, x], best)
    assert (s[:3] == 0).all() and (s[:, -3:] == 0).all()
    assert np.array_equal(orc.orb_resize(img, 26, 24), img)
    assert (orc.orb_resize(np.full((50, 60), 77, np.uint8), 41, 33) == 77).all()
    for nf in (500, 1000, 1500, 5000, 6000):
        assert sum(orc.orb_level_counts(nf)) == nf
    pat, trip = orc.orb_tables()
    assert pat.shape == (256, 4) and np.abs(pat).max() <= 13 and 4.5 < np.abs(pat).mean() < 6.0
    assert trip.shape == (512, 6) and ((trip[:, 0::2] ** 2 + trip[:, 1::2] ** 2) <= 361).all()
    assert orc.orb_umax()[:16] == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
