"""GPU parity tests for the bundle-adjustment hot path (libptzba.so through its C-ABI).

Oracles:
  * golden fixtures made by running the reference itself (tests/golden/make_golden.py):
    residual vectors of bundle_adjustment._compute_residual and scipy trf optima (tight tolerance)
  * the CPU restatement in oracle/ptz_oracle.py (pinned to those fixtures by test_oracle_golden.py)

Tolerances (stated per test): fp64 residuals 1e-8 px; fp32 residuals 2e-3 px; fp64 optimum vs the
reference's tight optimum: 1e-6 deg / 1e-4 px; fp32 LM vs fp64 optimum: pan/tilt/f RMSE <= 1e-4
(the north-star gate)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _problem_from_golden(d):
    """Rebuild the pair-form records (record 2m = src of match m, 2m+1 = dst) from a BA fixture."""
    pts = d["points"]
    off = d["points_off"]
    mi, mj, k1, k2, lm = d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"]
    R = 2 * len(mi)
    frame = np.empty(R, np.int32)
    frame[0::2] = mi
    frame[1::2] = mj
    landmark = np.repeat(lm, 2).astype(np.int32)
    xy = np.empty((R, 2))
    xy[0::2] = pts[off[mi] + k1]
    xy[1::2] = pts[off[mj] + k2]
    return int(d["n_pose"]), int(d["n_landmark"]), frame, landmark, xy, float(d["u"]), float(d["v"])


def _observed(n_pose, n_lm, frame, landmark):
    """Parameter mask (free params, frame 0 excluded) of observed frames / landmarks."""
    fo = np.zeros(n_pose, bool)
    fo[frame] = True
    lo = np.zeros(n_lm, bool)
    lo[landmark] = True
    return np.concatenate([np.repeat(fo[1:], 3), np.repeat(lo, 2)])


@pytest.mark.parametrize("name", ["ba_4x60", "ba_6x120", "ba_10x200"])
@pytest.mark.parametrize("precision", [0, 1])
def test_residual_matches_reference(gpu_available, name, precision):
    import ptzba
    d = golden(name + ".npz")
    n, m, frame, landmark, xy, u, v = _problem_from_golden(d)
    h = ptzba.BAHandle(0)
    h.set_problem(n, m, frame, landmark, xy, u, v, precision=precision)
    tol = 1e-8 if precision == 0 else 2e-3
    for x, r_ref in zip(d["xs"], d["rs"]):
        x_full = np.concatenate([d["ref_pose"], x])
        r = h.residual(x_full)
        assert r.shape == r_ref.shape
        # perturbed states can push rays behind a camera; the reference's |q2| semantics must hold there too
        np.testing.assert_allclose(r, r_ref, rtol=0, atol=tol * max(1.0, np.abs(r_ref).max() / 1e3))
    h.close()


@pytest.mark.parametrize("name", ["ba_6x120", "ba_10x200"])
def test_solve_matches_reference_tight_optimum(gpu_available, name):
    """fp64 LM to convergence == the reference's scipy trf optimum at ftol=xtol=gtol=1e-15."""
    import ptzba
    d = golden(name + ".npz")
    n, m, frame, landmark, xy, u, v = _problem_from_golden(d)
    x0 = np.concatenate([d["ref_pose"], d["x0"]])
    ptz0 = x0[:3 * n].reshape(n, 3)
    rays0 = x0[3 * n:].reshape(m, 2)
    ptz, rays, res = ptzba.solve(n, m, frame, landmark, xy, u, v, ptz0, rays0, precision=ptzba.FP64,
                                 ftol=1e-14, xtol=1e-14, max_iter=200)
    x = np.concatenate([ptz.reshape(-1)[3:], rays.reshape(-1)])
    mask = _observed(n, m, frame, landmark)
    xt = d["x_tight"]
    assert abs(res.cost - float(d["tight_cost"])) <= 1e-9 * float(d["tight_cost"]) + 1e-9
    # pose: 1e-6 deg (pan, tilt) and 1e-4 px (f); rays 1e-6 deg
    diff = np.abs(x - xt)[mask]
    scale = np.concatenate([np.tile([1e-6, 1e-6, 1e-4], n - 1), np.full(2 * m, 1e-6)])[mask]
    assert np.all(diff <= scale), (diff / scale).max()


def test_solve_4x60_observed_params(gpu_available):
    """ba_4x60 has a frame without any matched pair: the reference's trf wanders along its zero
    Jacobian columns; parity is asserted on the observed parameters and the cost."""
    import ptzba
    d = golden("ba_4x60.npz")
    n, m, frame, landmark, xy, u, v = _problem_from_golden(d)
    x0 = np.concatenate([d["ref_pose"], d["x0"]])
    ptz, rays, res = ptzba.solve(n, m, frame, landmark, xy, u, v, x0[:3 * n].reshape(n, 3), x0[3 * n:].reshape(m, 2),
                                 ftol=1e-14, xtol=1e-14, max_iter=200)
    x = np.concatenate([ptz.reshape(-1)[3:], rays.reshape(-1)])
    mask = _observed(n, m, frame, landmark)
    assert abs(res.cost - float(d["tight_cost"])) <= 1e-8 * float(d["tight_cost"])
    np.testing.assert_allclose(x[mask], d["x_tight"][mask], rtol=0, atol=1e-4)


@pytest.mark.parametrize("precision", [0, 1])
def test_config2_optimum(gpu_available, precision):
    """Config 2 (50 KF x 2k rays): GPU LM vs the scipy tight optimum of the pinned oracle
    (tests/golden/config2_optimum.npz).  Gate: pan/tilt/f RMSE <= 1e-4 (north star)."""
    import ptzba
    import synthetic
    d = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    assert len(p.frame) == int(d["n_records"]) and int(p.frame.sum()) == int(d["frame_sum"])
    ptz, rays, res = ptzba.solve(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, p.init_ptz, p.init_rays,
                                 precision=precision, ftol=1e-12, xtol=1e-12, max_iter=100)
    xt = d["x_tight"]
    ptz_t = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
    rmse = synthetic.pose_rmse(ptz, ptz_t)
    assert np.all(rmse <= 1e-4), rmse
    rays_t = xt[3 * (p.n_pose - 1):].reshape(-1, 2)
    assert np.sqrt(np.mean((rays - rays_t) ** 2)) <= 1e-4
    assert abs(res.cost - float(d["tight_cost"])) <= 1e-6 * float(d["tight_cost"])


def test_config2_huber(gpu_available):
    import ptzba
    import synthetic
    d = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    ptz, rays, res = ptzba.solve(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, p.init_ptz, p.init_rays,
                                 precision=ptzba.FP32, loss=ptzba.LOSS_HUBER, f_scale=1.0, ftol=1e-12, xtol=1e-12,
                                 max_iter=100)
    xt = d["x_tight_huber"]
    ptz_t = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
    assert np.all(synthetic.pose_rmse(ptz, ptz_t) <= 1e-4)
    assert abs(res.cost - float(d["tight_cost_huber"])) <= 1e-5 * float(d["tight_cost_huber"])


def test_dedup_equals_pair_form(gpu_available):
    """Weighted de-duplicated records give the same optimum as the pair form."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config2", seed=0)
    f, l, xy, w, _ = synthetic.dedup_records(p.frame, p.landmark, p.xy)
    assert len(f) < len(p.frame)
    kw = dict(precision=ptzba.FP64, ftol=1e-12, xtol=1e-12, max_iter=60)
    a = ptzba.solve(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, p.init_ptz, p.init_rays, **kw)
    b = ptzba.solve(p.n_pose, p.n_landmark, f, l, xy, p.u, p.v, p.init_ptz, p.init_rays, weight=w, **kw)
    np.testing.assert_allclose(a[0], b[0], rtol=0, atol=1e-7)
    assert abs(a[2].cost - b[2].cost) <= 1e-9 * a[2].cost


def test_residual_matches_oracle_config2(gpu_available):
    """Record-order residual at x0 (588k residuals) vs the oracle and the reference sample."""
    import ptzba
    import synthetic
    from oracle import ptz_oracle as orc
    d = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v)
    x0 = d["x0"]
    r = h.residual(x0)
    r_o = orc.compute_residual_records(x0, p.n_pose, p.u, p.v, p.frame.astype(np.int64), p.landmark.astype(np.int64), p.xy)
    np.testing.assert_allclose(r, r_o, rtol=0, atol=1e-8)
    np.testing.assert_allclose(r[d["r_ref_sample_idx"]], d["r_ref_sample"], rtol=0, atol=1e-8)
    assert abs(float(np.sum(r * r)) - float(d["r_ref_sumsq"])) <= 1e-9 * float(d["r_ref_sumsq"])
