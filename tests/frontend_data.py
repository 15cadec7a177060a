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


def _mix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def value_noise(x, y, seed=0, cells=(40.0, 17.0, 7.0, 3.0), amps=(55.0, 40.0, 28.0, 14.0)):
    """Smooth procedural texture T(x, y) (continuous in x, y, defined everywhere): octaves of lattice value
    noise with smoothstep interpolation; lattice values are a hash of (seed, octave, i, j)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    out = np.full(np.broadcast(x, y).shape, 128.0)
    for o, (c, a) in enumerate(zip(cells, amps)):
        gx, gy = x / c, y / c
        i0, j0 = np.floor(gx), np.floor(gy)
        fx, fy = gx - i0, gy - j0
        sx, sy = fx * fx * (3 - 2 * fx), fy * fy * (3 - 2 * fy)
        base = np.uint64((seed * 1315423911 + o * 2654435761) & 0xFFFFFFFFFFFF)

        def lat(di, dj):
            ii = (i0 + di).astype(np.int64).astype(np.uint64)
            jj = (j0 + dj).astype(np.int64).astype(np.uint64)
            with np.errstate(over="ignore"):
                h = _mix64(base * np.uint64(0x9E3779B97F4A7C15) + ii * np.uint64(0x632BE59BD9B4E019) +
                           jj * np.uint64(0x85EBCA77C2B2AE63))
            return (h >> np.uint64(11)).astype(np.float64) / float(1 << 53) * 2.0 - 1.0
        top = lat(0, 0) * (1 - sx) + lat(1, 0) * sx
        bot = lat(0, 1) * (1 - sx) + lat(1, 1) * sx
        out += a * (top * (1 - sy) + bot * sy)
    return out


def textured_pair(seed=0, width=320, height=240, d_pan=0.6, d_tilt=-0.3, f=600.0, df=8.0, flat_box=None):
    """Two 8-bit grey views of a textured scene under a PTZ motion: I(p) = T(p), J(p) = T(H^-1 p) with H the
    pure-rotation homography between the views.  flat_box = (x0, y0, x1, y1) paints a constant region in both
    (untrackable).  Returns (I, J, H)."""
    u, v = width / 2.0, height / 2.0
    H = ptz_homography(u, v, np.array([10.0, -5.0, f]), np.array([10.0 + d_pan, -5.0 + d_tilt, f + df]))
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float64)
    Hi = np.linalg.inv(H)
    q = np.stack([xx.ravel(), yy.ravel(), np.ones(xx.size)], 1) @ Hi.T
    I = value_noise(xx, yy, seed)
    J = value_noise((q[:, 0] / q[:, 2]).reshape(xx.shape), (q[:, 1] / q[:, 2]).reshape(xx.shape), seed)
    I8 = np.clip(np.rint(I), 0, 255).astype(np.uint8)
    J8 = np.clip(np.rint(J), 0, 255).astype(np.uint8)
    if flat_box is not None:
        x0, y0, x1, y1 = flat_box
        I8[y0:y1, x0:x1] = 100
        J8[y0:y1, x0:x1] = 100
    return I8, J8, H


def binary_views(seed=0, n_common=300, n_only=100, nbytes=32, flips=6):
    """ORB/LATCH-like binary descriptors of world features in two PTZ views: a few flipped bits between
    views, distractors on both sides, keypoints under the true homography (+ noise)."""
    rng = np.random.default_rng(seed)
    H = ptz_homography(640.0, 360.0, np.array([12.0, -6.0, 2200.0]), np.array([14.5, -5.2, 2300.0]))
    p1 = np.stack([rng.uniform(50, 1200, n_common), rng.uniform(40, 680, n_common)], 1)
    p2 = apply_h(H, p1) + rng.normal(0, 0.2, p1.shape)
    F = rng.integers(0, 256, (n_common, nbytes), dtype=np.uint8)
    G = F.copy()
    for i in range(n_common):
        for b in rng.choice(nbytes * 8, flips, replace=False):
            G[i, b // 8] ^= np.uint8(1 << (b % 8))
    D1 = np.r_[F, rng.integers(0, 256, (n_only, nbytes), dtype=np.uint8)]
    D2 = np.r_[G, rng.integers(0, 256, (n_only, nbytes), dtype=np.uint8)]
    x1 = np.r_[p1, rng.uniform(0, 1280, (n_only, 2))]
    x2 = np.r_[p2, rng.uniform(0, 1280, (n_only, 2))]
    perm = rng.permutation(len(x2))
    inv = np.argsort(perm)
    truth = {k: int(inv[k]) for k in range(n_common)}
    return x1, D1, x2[perm], D2[perm], H, truth
