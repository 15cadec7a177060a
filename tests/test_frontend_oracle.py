"""CPU checks of the front-end oracle (oracle/ptz_oracle.py knn2 / homography_ransac, test infrastructure):
the kNN restatement against an explicit per-query sort, and the RANSAC restatement against the ground
truth of synthetic correspondences (the GPU kernels are compared with these in test_gpu_frontend.py)."""
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
