"""GPU pose-only refinement / relocalisation (relocalization.py) through the C-ABI
(`ptz_refine_poses`).  Anchors: tests/golden/reloc.npz, made by running the reference's
least_squares(_compute_residual, ...) (relocalization.py:186) and relocalization_camera end to end with a
deterministic ray front-end (synthetic.RayFrontEnd), and the oracle (pinned to that fixture).
Tolerances: pan/tilt 1e-7 deg and f 1e-5 px against tight optima; 1e-5 deg / 5e-3 px against the
reference's own ftol=1e-4 results (both solvers stop at the same optimum to within their tolerance)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _close(p, q, ang, fpx):
    assert abs(p[0] - q[0]) < ang and abs(p[1] - q[1]) < ang and abs(p[2] - q[2]) < fpx, (p, q)


def test_refine_matches_reference_optimum(gpu_available):
    import ptzba
    d = golden("reloc.npz")
    u, v = float(d["u"]), float(d["v"])
    ptz, cost, its, st = ptzba.refine_poses(u, v, d["pose0"][None], d["rays"], d["points"], ftol=1e-14, xtol=1e-14)
    _close(ptz[0], d["x_tight"], 1e-7, 1e-5)
    assert abs(cost[0] - float(d["cost_tight"])) <= 1e-9 * float(d["cost_tight"])
    # the reference's own setting (ftol=1e-4)
    ptz, cost, its, st = ptzba.refine_poses(u, v, d["pose0"][None], d["rays"], d["points"])
    _close(ptz[0], d["x_ftol"], 1e-5, 5e-3)
    assert st[0] in (2, 3)


def test_reloc_residual_drop_in(gpu_available):
    import relocalization
    from oracle import ptz_oracle as orc
    d = golden("reloc.npz")
    u, v = float(d["u"]), float(d["v"])
    for pose in (d["pose0"], d["x_tight"]):
        np.testing.assert_allclose(relocalization._compute_residual(pose, d["rays"], d["points"], u, v),
                                   orc.reloc_residual(pose, d["rays"], d["points"], u, v), rtol=0, atol=1e-8)


def test_relocalization_camera_drop_in(gpu_available):
    """The reference's call sequence: Map of keyframes, lost image, front-end hooks -> pose."""
    import image_process
    import key_frame
    import relocalization
    import scene_map
    import synthetic
    d = golden("reloc.npz")
    rays, cams = d["scene_rays"], d["scene_cams"]
    fe = synthetic.RayFrontEnd(rays, cams)
    saved = image_process.detect_compute_sift, image_process.match_sift_features
    image_process.detect_compute_sift, image_process.match_sift_features = fe.detect, fe.match
    try:
        m = scene_map.Map('sift')
        for k in range(4):
            pan, tilt, f = cams[k]
            m.keyframe_list.append(key_frame.KeyFrame(k, k, np.zeros(3), np.eye(3), float(d["u"]), float(d["v"]),
                                                      pan, tilt, f))
        pose = relocalization.relocalization_camera(m, 4, d["lost_init"].copy())
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved
    _close(pose, d["reloc_pose"], 1e-5, 5e-3)


def test_multistart_hypotheses_converge(gpu_available):
    import ptzba
    d = golden("reloc.npz")
    u, v = float(d["u"]), float(d["v"])
    rng = np.random.default_rng(0)
    init = d["x_tight"] + rng.uniform(-1, 1, (64, 3)) * np.array([2.0, 1.0, 200.0])
    ptz, cost, its, st = ptzba.refine_poses(u, v, init, d["rays"], d["points"], ftol=1e-14, xtol=1e-14)
    for k in range(64):
        _close(ptz[k], d["x_tight"], 1e-7, 1e-5)


@pytest.mark.parametrize("loss", [0, 1])
def test_subset_hypotheses_match_oracle(gpu_available, loss):
    """Preemptive-RANSAC style batch: each hypothesis refines on its own 32-correspondence sample."""
    import ptzba
    from scipy.optimize import least_squares
    from oracle import ptz_oracle as orc
    d = golden("reloc.npz")
    u, v = float(d["u"]), float(d["v"])
    rng = np.random.default_rng(1)
    n = len(d["rays"])
    subsets = [rng.choice(n, 32, replace=False) for _ in range(16)]
    init = np.repeat(d["pose0"][None], 16, 0)
    ptz, cost, its, st = ptzba.refine_poses(u, v, init, d["rays"], d["points"], subsets=subsets, ftol=1e-14,
                                            xtol=1e-14, loss=loss, f_scale=1.0)
    for k, s in enumerate(subsets):
        ref = least_squares(orc.reloc_residual, d["pose0"], x_scale='jac', ftol=1e-15, xtol=1e-15, gtol=1e-15,
                            method='trf', loss='huber' if loss else 'linear', f_scale=1.0,
                            args=(d["rays"][s], d["points"][s], u, v))
        _close(ptz[k], ref.x, 1e-6, 1e-4)
        assert abs(cost[k] - ref.cost) <= 1e-7 * ref.cost
