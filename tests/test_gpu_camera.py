"""GPU camera-model kernels vs the reference's own outputs (tests/golden/kat_projection.npz,
ekf_R*.npz), produced by running transformation.py / ptz_camera.py / ptz_slam.py in place.

Tolerances: projections 1e-7 px (fp64, closed form vs q form differ only by rounding);
back-projection 1e-9 deg; FD Jacobian 1e-5 (the reference's central differences amplify the
projection's rounding by 1/(2*0.001 deg))."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def test_ray_to_image_kat(gpu_available):
    import ptzba
    d = golden("kat_projection.npz")
    x, y = ptzba.ray_to_image(float(d["u"]), float(d["v"]), d["f"], d["cam_pan"], d["cam_tilt"], d["theta"], d["phi"])
    np.testing.assert_allclose(x, d["xy"][:, 0], rtol=0, atol=1e-7 * np.abs(d["xy"][:, 0]).max() / 1e3)
    np.testing.assert_allclose(y, d["xy"][:, 1], rtol=0, atol=1e-7 * np.abs(d["xy"][:, 1]).max() / 1e3)


def test_image_to_ray_kat(gpu_available):
    import ptzba
    d = golden("kat_projection.npz")
    th, ph = ptzba.image_to_ray(float(d["u"]), float(d["v"]), d["bp_f"], d["bp_pan"], d["bp_tilt"], d["bp_x"], d["bp_y"])
    np.testing.assert_allclose(th, d["bp_ray"][:, 0], rtol=0, atol=1e-9)
    np.testing.assert_allclose(ph, d["bp_ray"][:, 1], rtol=0, atol=1e-9)


def test_ptz_camera_project_backproject_kat(gpu_available):
    import ptzba
    d = golden("kat_projection.npz")
    u, v = float(d["u"]), float(d["v"])
    for row in d["cam_rows"]:
        has_d, cp, ct, f, th, ph, px, py, ix, iy, bth, bph = row
        disp = d["displacement"] if has_d else None
        xy = ptzba.project_rays(u, v, f, cp, ct, [[th, ph]], displacement=disp)[0]
        assert abs(xy[0] - px) < 1e-7 and abs(xy[1] - py) < 1e-7
        r = ptzba.back_project_rays(u, v, f, cp, ct, [[ix, iy]], displacement=disp)[0]
        assert abs(r[0] - bth) < 1e-9 and abs(r[1] - bph) < 1e-9


@pytest.mark.parametrize("name", ["ekf_R50.npz", "ekf_R300.npz"])
def test_h_jacobian_matches_reference(gpu_available, name):
    import ptzba
    d = golden(name)
    H = ptzba.h_jacobian(float(d["u"]), float(d["v"]), float(d["f0"]), float(d["pan0"]), float(d["tilt0"]), d["H_rays"])
    np.testing.assert_allclose(H, d["H"], rtol=0, atol=1e-5)
