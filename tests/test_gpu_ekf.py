"""GPU parity of the EKF tracking path through the C-ABI (ptzekf_*).

Anchors:
  * ekf_R50 / ekf_R300 fixtures: PtzSlam.ekf_update and compute_h_jacobian run by the reference
    itself (tests/golden/make_golden.py gen_ekf);
  * oracle.ptz_oracle.ekf_update (pinned to those fixtures by test_oracle_golden.py) on larger and
    edge-case states (unsorted / duplicate / out-of-view observation indices, no match).
Tolerances: pan/tilt 1e-9 deg, f 1e-6 px, rays 1e-9 deg, covariance rtol 1e-7 (the GPU solves with a
Cholesky factorisation where the reference forms inv(S); both are fp64).
"""
import copy

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _state(d):
    R = len(d["rays0"])
    cov0 = np.diag(d["cov_base_diag"]).astype(np.float64)
    cov0[2, 2] = float(d["f_var"])
    cov0 = cov0 + d["cov_B"] @ d["cov_B"].T
    return d["rays0"].copy(), cov0


def _check_against_golden(d, ptz, vel, rays1, cov1, cov0):
    assert abs(ptz[0] - float(d["pan1"])) < 1e-9
    assert abs(ptz[1] - float(d["tilt1"])) < 1e-9
    assert abs(ptz[2] - float(d["f1"])) < 1e-6
    np.testing.assert_allclose(vel, d["velocity"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(rays1, d["rays1"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(cov1[:3, :3], d["cov1_pose"], rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(np.diag(cov1), d["cov1_diag"], rtol=1e-7, atol=1e-12)
    pk = d["cov1_pick"]
    np.testing.assert_allclose(cov1[pk[:, 0], pk[:, 1]], d["cov1_pick_val"], rtol=1e-6, atol=1e-12)
    assert int(np.sum(cov1 != cov0)) == int(d["n_changed"])
    assert abs(cov1.sum() - float(d["cov1_sum"])) <= 1e-9 * abs(float(d["cov1_sum"]))


@pytest.mark.parametrize("name", ["ekf_R50.npz", "ekf_R300.npz"])
def test_ekf_update_matches_reference(gpu_available, name):
    import ptzba
    d = golden(name)
    rays0, cov0 = _state(d)
    h = ptzba.EKFHandle(0)
    h.set_state(rays0, cov0)
    ptz, vel, nm = h.update(float(d["u"]), float(d["v"]), [float(d["pan0"]), float(d["tilt0"]), float(d["f0"])],
                            d["obs"], d["obs_idx"], int(d["height"]), int(d["width"]), 0.1)
    rays1, cov1 = h.get_state()
    h.close()
    assert nm > 0
    _check_against_golden(d, ptz, vel, rays1, cov1, cov0)


@pytest.mark.parametrize("name", ["ekf_R50.npz", "ekf_R300.npz"])
def test_ptzslam_ekf_update_drop_in(gpu_available, name):
    """The reference's call sequence on the drop-in class: attributes assigned, ekf_update called."""
    import ptz_camera
    import ptz_slam
    d = golden(name)
    rays0, cov0 = _state(d)
    cam = ptz_camera.PTZCamera((float(d["u"]), float(d["v"])), np.array([0.0, -10.0, 5.0]), np.eye(3))
    cam.set_ptz([float(d["pan0"]), float(d["tilt0"]), float(d["f0"])])
    slam = ptz_slam.PtzSlam()
    slam.cameras = [cam]
    slam.rays = rays0.copy()
    slam.state_cov = cov0.copy()
    slam.current_camera = copy.deepcopy(cam)
    H = slam.compute_h_jacobian(float(d["pan0"]), float(d["tilt0"]), float(d["f0"]), d["H_rays"])
    np.testing.assert_allclose(H, d["H"], rtol=0, atol=1e-6)
    slam.ekf_update(d["obs"], d["obs_idx"], int(d["height"]), int(d["width"]))
    c = slam.current_camera
    _check_against_golden(d, [c.pan, c.tilt, c.focal_length], slam.velocity, slam.rays, slam.state_cov, cov0)


def _random_state(R, seed, frac_obs=0.8, shuffle=False, dup=False):
    from oracle import ptz_oracle as orc
    rng = np.random.default_rng(seed)
    u, v, pan, tilt, f = 960.0, 540.0, 20.0, -10.0, 2500.0
    pts = np.stack([rng.uniform(-100, 2020, R), rng.uniform(-60, 1140, R)], 1)  # some rays out of view
    rays = orc.back_project_to_rays(u, v, f, pan, tilt, pts) + rng.normal(0, 0.02, (R, 2))
    ns = 3 + 2 * R
    B = rng.normal(0, 3e-3, (ns, 6))
    cov = 0.001 * np.eye(ns) + B @ B.T
    cov[2, 2] += 1.0
    keep = np.sort(rng.choice(R, int(R * frac_obs), replace=False))
    if dup:
        keep = np.sort(np.concatenate([keep, keep[::7]]))
    if shuffle:
        keep = keep.copy()
        rng.shuffle(keep)
    obs = orc.project_rays(u, v, f + 6.0, pan + 0.06, tilt - 0.04, rays[keep]) + rng.normal(0, 0.3, (len(keep), 2))
    state = dict(u=u, v=v, pan=pan + 0.01, tilt=tilt, f=f, displacement=None, rays=rays, state_cov=cov)
    return state, obs, keep


@pytest.mark.parametrize("R,seed,shuffle,dup", [(700, 11, False, False), (180, 12, True, False),
                                                (240, 13, False, True), (1, 14, False, False)])
def test_ekf_update_matches_oracle(gpu_available, R, seed, shuffle, dup):
    import ptzba
    from oracle import ptz_oracle as orc
    s, obs, keep = _random_state(R, seed, frac_obs=1.0 if R == 1 else 0.8, shuffle=shuffle, dup=dup)
    ref = orc.ekf_update(s, obs, keep, 1080, 1920)
    h = ptzba.EKFHandle(0)
    h.set_state(s["rays"], s["state_cov"])
    ptz, vel, nm = h.update(s["u"], s["v"], [s["pan"], s["tilt"], s["f"]], obs, keep, 1080, 1920, 0.1)
    rays1, cov1 = h.get_state()
    h.close()
    assert abs(ptz[0] - ref["pan"]) < 1e-9 and abs(ptz[1] - ref["tilt"]) < 1e-9 and abs(ptz[2] - ref["f"]) < 1e-6
    np.testing.assert_allclose(vel, ref["velocity"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(rays1, ref["rays"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(cov1, ref["state_cov"], rtol=1e-7, atol=1e-13)
    # same entries written back (the reference's partial write-back pattern)
    assert np.array_equal(cov1 != s["state_cov"], ref["state_cov"] != s["state_cov"])


@pytest.mark.parametrize("R,seed", [(300, 21), (40, 22)])
def test_ekf_update_indefinite_innovation(gpu_available, R, seed):
    """The reference's covariance write-back (ptz_slam.py:282-289) leaves the state covariance indefinite
    after a few dozen frames (measured on the reference's own PtzSlam run: make_golden.py gen_stream
    stream), so S = H P H^T + R gets negative eigenvalues; the reference inverts it with np.linalg.inv
    (ptz_slam.py:258).  The GPU update factors S = L Sigma L^T (signed) and must equal the oracle."""
    import ptzba
    from oracle import ptz_oracle as orc
    s, obs, keep = _random_state(R, seed)
    s["state_cov"][0:3, 0:3] -= 0.02 * np.eye(3)  # pose block pushed negative: S loses definiteness
    # the innovation covariance really is indefinite (oracle's own S)
    pred, pidx = orc.project_rays_visible(s["u"], s["v"], s["f"], s["pan"], s["tilt"], s["rays"], 1080, 1920)
    o1, _ = orc.get_overlap_index(keep, pidx)
    m = np.asarray(keep)[o1]
    pr = np.concatenate([[0, 1, 2], np.stack([2 * m + 3, 2 * m + 4], -1).reshape(-1)])
    H = orc.compute_h_jacobian(s["u"], s["v"], s["pan"], s["tilt"], s["f"], s["rays"][m])
    S = H @ s["state_cov"][np.ix_(pr, pr)] @ H.T + 0.1 * np.eye(2 * len(m))
    assert np.linalg.eigvalsh(S).min() < 0
    ref = orc.ekf_update(s, obs, keep, 1080, 1920)
    h = ptzba.EKFHandle(0)
    h.set_state(s["rays"], s["state_cov"])
    ptz, vel, nm = h.update(s["u"], s["v"], [s["pan"], s["tilt"], s["f"]], obs, keep, 1080, 1920, 0.1)
    rays1, cov1 = h.get_state()
    h.close()
    scale = np.abs(ref["velocity"]).max()
    np.testing.assert_allclose(vel, ref["velocity"], rtol=0, atol=1e-7 * scale + 1e-9)
    np.testing.assert_allclose(rays1, ref["rays"], rtol=0, atol=1e-8)
    np.testing.assert_allclose(cov1, ref["state_cov"], rtol=1e-6, atol=1e-10)


def test_ekf_update_no_match_leaves_state(gpu_available):
    import ptzba
    s, obs, keep = _random_state(50, 3)
    h = ptzba.EKFHandle(0)
    h.set_state(s["rays"], s["state_cov"])
    ptz, vel, nm = h.update(s["u"], s["v"], [s["pan"], s["tilt"], s["f"]], obs[:0], keep[:0], 1080, 1920, 0.1)
    rays1, cov1 = h.get_state()
    assert nm == 0 and np.all(vel == 0)
    np.testing.assert_array_equal(ptz, [s["pan"], s["tilt"], s["f"]])
    np.testing.assert_array_equal(rays1, s["rays"])
    np.testing.assert_array_equal(cov1, s["state_cov"])


def test_ekf_state_ops_match_numpy(gpu_available):
    """remove_rays (np.delete on rays and both covariance axes), add_rays (zero rows/cols, var on the
    diagonal), predict (pose block += Q) — ptz_slam.py:291-315, 376-384, 424-426."""
    import ptzba
    rng = np.random.default_rng(5)
    R = 90
    rays = rng.normal(0, 10, (R, 2))
    cov = rng.normal(0, 1, (3 + 2 * R, 3 + 2 * R))
    h = ptzba.EKFHandle(0)
    h.set_state(rays, cov)
    q = 5 * np.diag([0.001, 0.001, 1.0])
    h.add_pose_cov(q)
    cov[0:3, 0:3] += q
    idx = np.array([3, 17, 17, -1, 40])
    h.remove_rays(idx)
    rays = np.delete(rays, idx, axis=0)
    p = np.concatenate([2 * np.mod(idx, R) + 3, 2 * np.mod(idx, R) + 4])
    cov = np.delete(np.delete(cov, p, axis=0), p, axis=1)
    new = rng.normal(0, 10, (7, 2))
    h.add_rays(new, 0.001)
    for j in range(len(new)):
        rays = np.vstack([rays, new[j]])
        cov = np.vstack([cov, np.zeros([2, cov.shape[1]])])
        cov = np.hstack([cov, np.zeros([cov.shape[0], 2])])
        cov[-2, -2] = 0.001
        cov[-1, -1] = 0.001
    r1, c1 = h.get_state()
    assert h.n_ray == len(rays)
    np.testing.assert_array_equal(r1, rays)
    np.testing.assert_array_equal(c1, cov)
    with pytest.raises(ptzba.PtzbaError):
        h.remove_rays([10 ** 6])
    h.close()


def test_project_visible_matches_reference_rule(gpu_available):
    """PTZCamera.project_rays(rays, h, w): strictly-inside points in ray order, float indices."""
    import ptzba
    from oracle import ptz_oracle as orc
    s, _, _ = _random_state(400, 21)
    h = ptzba.EKFHandle(0)
    h.set_state(s["rays"], s["state_cov"])
    xy, idx = h.project_visible(s["u"], s["v"], [s["pan"], s["tilt"], s["f"]], 1080, 1920)
    ref_xy, ref_idx = orc.project_rays_visible(s["u"], s["v"], s["f"], s["pan"], s["tilt"], s["rays"], 1080, 1920)
    np.testing.assert_array_equal(idx, ref_idx)
    np.testing.assert_allclose(xy, ref_xy, rtol=0, atol=1e-8)
    h.close()
