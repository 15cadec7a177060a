"""Synthetic SIFT-like correspondence data for the front-end tests (test infrastructure): integer-valued
128-d descriptors (0..255, as OpenCV's SIFT returns) of world features seen by two PTZ views, keypoints =
projections under the two true cameras (a pure-rotation homography apart) + noise, a fraction of
distractors on both sides."""
import numpy as np


def ptz_homography(u, v, cam1, cam2):
    """x2 ~ K2 R2 R1^T K1^-1 x1 for two pan/tilt/focal views (ptz_camera.py:73-79 rotations)."""
    def K(f):
        return np.array([[f, 0, u], [0, f, v], [0, 0, 1.0]])

    def R(pan, tilt):
        a, b = np.radians(pan), np.radians(tilt)
        ry = np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]])
        rx = np.array([[1, 0, 0], [0, np.cos(b), np.sin(b)], [0, -np.sin(b), np.cos(b)]])
        return rx @ ry
    H = K(cam2[2]) @ R(cam2[0], cam2[1]) @ R(cam1[0], cam1[1]).T @ np.linalg.inv(K(cam1[2]))
    return H / H[2, 2]


def apply_h(H, p):
    q = np.c_[p, np.ones(len(p))] @ H.T
    return q[:, :2] / q[:, 2:3]


def two_views(seed=0, n_common=400, n_only=150, noise=0.3, des_noise=3):
    rng = np.random.default_rng(seed)
    u, v = 640.0, 360.0
    cam1, cam2 = np.array([30.0, -8.0, 2800.0]), np.array([34.0, -7.5, 2900.0])
    H = ptz_homography(u, v, cam1, cam2)
    p1 = np.stack([rng.uniform(200, 1200, n_common), rng.uniform(40, 700, n_common)], 1)
    p2 = apply_h(H, p1)
    F = rng.integers(0, 256, (n_common, 128))
    d1 = np.clip(F + rng.integers(-des_noise, des_noise + 1, F.shape), 0, 255)
    d2 = np.clip(F + rng.integers(-des_noise, des_noise + 1, F.shape), 0, 255)
    x1 = np.r_[p1 + rng.normal(0, noise, p1.shape), np.stack([rng.uniform(0, 1280, n_only), rng.uniform(0, 720, n_only)], 1)]
    x2 = np.r_[p2 + rng.normal(0, noise, p2.shape), np.stack([rng.uniform(0, 1280, n_only), rng.uniform(0, 720, n_only)], 1)]
    D1 = np.r_[d1, rng.integers(0, 256, (n_only, 128))].astype(np.float32)
    D2 = np.r_[d2, rng.integers(0, 256, (n_only, 128))].astype(np.float32)
    perm1, perm2 = rng.permutation(len(x1)), rng.permutation(len(x2))
    # true correspondences after shuffling: query i1 -> train i2
    inv2 = np.argsort(perm2)
    truth = {int(np.flatnonzero(perm1 == k)[0]): int(inv2[k]) for k in range(n_common)}
    return x1[perm1], D1[perm1], x2[perm2], D2[perm2], H, truth


def homography_points(seed=0, n=600, outlier_frac=0.25, noise=0.3):
    rng = np.random.default_rng(seed)
    H = ptz_homography(640.0, 360.0, np.array([20.0, -9.0, 2600.0]), np.array([23.5, -8.2, 2750.0]))
    p1 = np.stack([rng.uniform(0, 1280, n), rng.uniform(0, 720, n)], 1)
    p2 = apply_h(H, p1) + rng.normal(0, noise, (n, 2))
    out = rng.random(n) < outlier_frac
    p2[out] += rng.uniform(5, 60, (out.sum(), 2)) * rng.choice([-1, 1], (out.sum(), 2))
    return p1, p2, H, ~out
