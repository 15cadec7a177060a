"""GPU front-end through the C-ABI: ptz_match_knn2 (cv.BFMatcher().knnMatch(k=2),
image_process.py:191) and ptz_homography_ransac (cv.findHomography RANSAC, image_process.py:433), and
image_process.match_sift_features (:178-234) composed from them, against the oracle restatements
(oracle/ptz_oracle.py knn2 / homography_ransac) on synthetic SIFT-like data.
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


def test_homography_ransac_hook_signature(gpu_available):
    """homography_ransac(points1, points2, threshold, return_matrix) as image_process.py:418 calls it."""
    import image_process
    p1, p2, H, inl = frontend_data.homography_points(seed=9, n=200)
    idx, Hm = image_process.homography_ransac(p1, p2, 1.0, return_matrix=True)
    assert idx == np.flatnonzero(inl).tolist() or len(set(idx) ^ set(np.flatnonzero(inl).tolist())) <= 1
    np.testing.assert_allclose(Hm, H, rtol=0, atol=2e-3 * np.abs(H).max())
