"""CPU tests of the native multi-row grid generator (csrc/synth.cpp, the config-4 input): the data follow
the reference's pair-form conventions (bundle_adjustment.py:67-99 record order, first-seen landmark ids of
image_process.py:611-639, last-writer ray init of bundle_adjustment.py:184-194), the output does not depend
on the thread count, and the grid really has landmarks with gaps in their frame range."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def grid():
    import synthetic
    return synthetic.make_grid_problem(120, 6000, -20.0, 20.0, (-10.0, 0.0, 10.0), seed=3, threads=4)


def test_thread_count_independent(grid):
    import synthetic
    g1 = synthetic.make_grid_problem(120, 6000, -20.0, 20.0, (-10.0, 0.0, 10.0), seed=3, threads=1)
    for k in ("frame", "landmark", "xy", "init_ptz", "init_rays", "gt_rays"):
        assert np.array_equal(getattr(grid, k), getattr(g1, k)), k
    g2 = synthetic.make_grid_problem(120, 6000, -20.0, 20.0, (-10.0, 0.0, 10.0), seed=4, threads=4)
    assert not np.array_equal(grid.xy[:100], g2.xy[:100])


def test_pair_form_conventions(grid):
    from oracle import ptz_oracle as orc
    p = grid
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    # records 2m / 2m+1: same landmark, frame i < j, pairs in lexicographic (i, j) order
    assert np.array_equal(lm[0::2], lm[1::2])
    assert np.all(fr[0::2] < fr[1::2])
    key = fr[0::2] * p.n_pose + fr[1::2]
    assert np.all(np.diff(key) >= 0)
    # first-seen landmark ids: the first occurrences appear in increasing id order
    _, first = np.unique(lm, return_index=True)
    assert np.all(np.diff(first) > 0) and lm.max() + 1 == p.n_landmark
    # <= 200 matches and > 20 per pair
    _, cnt = np.unique(key, return_counts=True)
    assert cnt.max() <= 200 and cnt.min() > 20 and len(cnt) == p.n_pairs
    # last-writer ray init: from_image_to_ray of the last src record of each landmark with the initial pose
    src = np.arange(0, len(lm), 2)
    last = np.full(p.n_landmark, -1)
    last[lm[src]] = src  # later writes win
    f = fr[last]
    th, ph = orc.from_image_to_ray(p.u, p.v, p.init_ptz[f, 2], p.init_ptz[f, 0], p.init_ptz[f, 1], p.xy[last, 0],
                                   p.xy[last, 1])
    np.testing.assert_allclose(np.stack([th, ph], 1), p.init_rays, atol=1e-9)
    # ground truth reproduces the observations to the keypoint noise (0.5 px)
    x = np.concatenate([p.gt_ptz.reshape(-1), p.gt_rays.reshape(-1)])
    r = orc.compute_residual_records(x, p.n_pose, p.u, p.v, fr, lm, p.xy)
    assert 0.4 < np.sqrt(np.mean(r * r)) < 0.6


def test_grid_landmarks_have_frame_gaps(grid):
    """Landmarks whose frame set is not contiguous (the case the Schur chunk filter must handle)."""
    p = grid
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    seg = np.unique(lm * p.n_pose + fr)
    sl, sf = seg // p.n_pose, seg % p.n_pose
    first = np.full(p.n_landmark, 1 << 30)
    last = np.full(p.n_landmark, -1)
    np.minimum.at(first, sl, sf)
    np.maximum.at(last, sl, sf)
    cnt = np.bincount(sl, minlength=p.n_landmark)
    assert np.any(last - first + 1 > cnt + 20)
