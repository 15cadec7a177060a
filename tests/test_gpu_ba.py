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



def _angle_f_maxdiff(x, xr, n):
    """max |x - xr| over the angles (pan, tilt, rays; deg) and over f (px) of a free-parameter vector."""
    d = np.abs(np.asarray(x) - np.asarray(xr))
    p = d[:3 * (n - 1)].reshape(-1, 3)
    return float(max(p[:, :2].max(), d[3 * (n - 1):].max())), float(p[:, 2].max())


@pytest.mark.parametrize("name", ["ba_6x120", "ba_10x200"])
def test_ftol_stop_matches_reference_x_ls(gpu_available, name):
    """The reference's OWN termination (bundle_adjustment.py:200-202: least_squares(..., x_scale='jac', ftol=1e-4,
    method='trf')): the fixture's x_ls is what the reference's scipy call returned on these inputs (4 Jacobians).  The
    GPU LM with its default options (ptzba.LAMBDA0: Gauss-Newton start, as trf's step inside its trust region) stopped
    by the same rule lands within 1e-6 deg / 1e-4 px of it -- the gate of the tight-optimum tests -- in no more
    Jacobian evaluations than the reference took."""
    import ptzba
    d = golden(name + ".npz")
    n, m, frame, landmark, xy, u, v = _problem_from_golden(d)
    x0 = np.concatenate([d["ref_pose"], d["x0"]])
    for device_loop in (True, False):
        h = ptzba.BAHandle(0)
        h.set_problem(n, m, frame, landmark, xy, u, v, precision=ptzba.FP64)
        h.set_state(x0[:3 * n].reshape(n, 3), x0[3 * n:].reshape(m, 2))
        res = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, device_loop=device_loop).run()
        ptz, rays = h.get_state()
        h.close()
        x = np.concatenate([ptz.reshape(-1)[3:], rays.reshape(-1)])
        da, df = _angle_f_maxdiff(x, d["x_ls"], n)
        print(f"{name} device_loop={device_loop}: {res}; vs x_ls max {da:.3e} deg / {df:.3e} px "
              f"(reference njev {int(d['ls_njev'])})")
        assert res.status == 2, res
        assert da <= 1e-6 and df <= 1e-4, (da, df)
        assert res.njev <= int(d["ls_njev"]), (res.njev, int(d["ls_njev"]))
        assert abs(res.cost - float(d["ls_cost"])) <= 1e-9 * float(d["ls_cost"])


def test_config2_ftol_stop_matches_scipy_trf(gpu_available):
    """Config 2 (50 KF x 2k rays) at the reference's termination: tests/golden/config2_ftol.npz holds where the pinned
    oracle's scipy trf stops with the reference's option set (x_scale='jac', ftol=1e-4, '2-point' FD Jacobian with the
    pair structure as jac_sparsity; make_golden.py gen_config2_ftol).  Linear loss (the reference's): the GPU's
    ftol=1e-4 solve in fp64 and in fp32 is within the north-star 1e-4 (pan / tilt deg, f px RMSE) of scipy's stop and
    of the tight optimum, in no more Jacobians than scipy.  Huber: scipy's trf + loss='huber' stops at ftol=1e-4 three
    Jacobians in, ~0.5 deg from the Huber optimum (its robust scaling drops the curvature of the residuals beyond the
    unit, which at x0 is nearly all of them); the GPU's IRLS / curvature-switch solve meets the 1e-4 gate there."""
    import ptzba
    import synthetic
    d = golden("config2_ftol.npz")
    t = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    assert len(p.frame) == int(d["n_records"]) and int(p.frame.sum()) == int(d["frame_sum"])
    full = lambda xf: np.concatenate([p.init_ptz[0], xf[:3 * (p.n_pose - 1)]]).reshape(-1, 3)  # noqa: E731
    for prec, loss, key in ((ptzba.FP64, ptzba.LOSS_LINEAR, ""), (ptzba.FP32, ptzba.LOSS_LINEAR, ""),
                            (ptzba.FP32, ptzba.LOSS_HUBER, "_huber")):
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec, loss=loss)
        h.set_state(p.init_ptz, p.init_rays)
        res = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8).run()
        ptz, rays = h.get_state()
        h.close()
        r_tight = synthetic.pose_rmse(ptz, full(t["x_tight" + key]))
        r_scipy = synthetic.pose_rmse(ptz, full(d["x_ftol" + key]))
        print(f"config2 prec={prec} loss={loss}: {res}; RMSE vs tight {r_tight}, vs scipy ftol stop {r_scipy} "
              f"(scipy njev {int(d['njev' + key])})")
        assert res.status == 2, res
        assert np.all(r_tight <= 1e-4), r_tight
        if key == "":
            assert np.all(r_scipy <= 1e-4), r_scipy
            assert res.njev <= int(d["njev"]), (res.njev, int(d["njev"]))
        else:
            scipy_off = synthetic.pose_rmse(full(d["x_ftol_huber"]), full(t["x_tight_huber"]))
            assert np.all(r_tight < scipy_off), (r_tight, scipy_off)


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


def _install_fixture_frontend(d):
    """Front-end hooks replaying the fixture's detector/matcher output (what the reference saw)."""
    import image_process
    off = d["points_off"]
    n = len(off) - 1
    pts = [d["points"][off[i]:off[i + 1]] for i in range(n)]
    raw = {}
    o = 0
    for i, j, c in zip(d["raw_pi"], d["raw_pj"], d["raw_cnt"]):
        raw[(int(i), int(j))] = (list(d["raw_a"][o:o + c]), list(d["raw_b"][o:o + c]))
        o += c
    kp_store = {}

    def detect(im, nfeatures, verbose=False):
        i = int(im)
        kps = [image_process.KeyPoint(x, y) for x, y in pts[i]]
        kp_store[i] = kps
        des = np.full((len(kps), 128), i, np.float32)
        des[:, 1] = np.arange(len(kps))
        return kps, des

    def match(kp1, des1, kp2, des2, pts_array=False, verbose=False):
        a, b = raw[(int(des1[0, 0]), int(des2[0, 0]))]
        return None, list(a), None, list(b)

    saved = (image_process.detect_compute_sift, image_process.match_sift_features)
    image_process.detect_compute_sift, image_process.match_sift_features = detect, match
    return saved, kp_store


@pytest.mark.parametrize("name", ["ba_6x120", "ba_10x200"])
def test_dropin_bundle_adjustment_matches_reference(gpu_available, name):
    """bundle_adjustment() drop-in on the reference's own inputs: landmark ids, keyframe feature order
    (set() order) bit-exact; poses/rays at the reference's tight optimum (1e-6 deg, 1e-4 px)."""
    import random
    import image_process
    import bundle_adjustment as ba
    d = golden(name + ".npz")
    n = int(d["n_pose"])
    saved, kp_store = _install_fixture_frontend(d)
    try:
        random.seed(int(d["seed"]))
        landmarks, keyframes = ba.bundle_adjustment(list(range(n)), list(range(100, 100 + n)), "sift",
                                                    d["init_ptz"].copy(), np.array([0.0, -10.0, 5.0]), np.eye(3),
                                                    float(d["u"]), float(d["v"]), "", ftol=1e-14, xtol=1e-14,
                                                    max_iter=200)
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved
    assert landmarks.shape == (int(d["n_landmark"]), 2)
    off = d["kf_off"]
    for i, kf in enumerate(keyframes):
        np.testing.assert_array_equal(kf.landmark_index.astype(np.int64), d["kf_lmk"][off[i]:off[i + 1]])
        pos = {id(o): k for k, o in enumerate(kp_store[i])}
        np.testing.assert_array_equal([pos[id(o)] for o in kf.feature_pts], d["kf_local"][off[i]:off[i + 1]])
        assert kf.img_index == 100 + i
    assert int(ba.LAST_RESULT["n_residual"]) == int(d["n_residual"])
    np.testing.assert_allclose(ba.LAST_RESULT["x0"], d["x0"], rtol=0, atol=1e-9)
    xt = d["x_tight"]
    ptz = np.array([[k.pan, k.tilt, k.f] for k in keyframes])
    ptz_t = np.concatenate([d["ref_pose"], xt[:3 * (n - 1)]]).reshape(-1, 3)
    np.testing.assert_allclose(ptz[:, :2], ptz_t[:, :2], rtol=0, atol=1e-6)
    np.testing.assert_allclose(ptz[:, 2], ptz_t[:, 2], rtol=0, atol=1e-4)
    np.testing.assert_allclose(landmarks.reshape(-1), xt[3 * (n - 1):], rtol=0, atol=1e-6)



@pytest.mark.parametrize("name", ["ba_6x120", "ba_10x200"])
def test_dropin_default_termination_matches_reference(gpu_available, name):
    """bundle_adjustment() with its default options (the reference's ftol=1e-4 stop) returns what the reference's
    bundle_adjustment() returned on the same inputs (the fixture's x_ls, landmarks, keyframe poses): 1e-6 deg / 1e-4 px."""
    import random
    import image_process
    import bundle_adjustment as ba
    d = golden(name + ".npz")
    n = int(d["n_pose"])
    saved, _ = _install_fixture_frontend(d)
    try:
        random.seed(int(d["seed"]))
        landmarks, keyframes = ba.bundle_adjustment(list(range(n)), list(range(100, 100 + n)), "sift",
                                                    d["init_ptz"].copy(), np.array([0.0, -10.0, 5.0]), np.eye(3),
                                                    float(d["u"]), float(d["v"]), "")
    finally:
        image_process.detect_compute_sift, image_process.match_sift_features = saved
    ptz = np.array([[k.pan, k.tilt, k.f] for k in keyframes])
    np.testing.assert_allclose(ptz, d["kf_ptz"], rtol=0, atol=1e-4)  # the reference's keyframes (f in px)
    np.testing.assert_allclose(ptz[:, :2], d["kf_ptz"][:, :2], rtol=0, atol=1e-6)
    np.testing.assert_allclose(landmarks, d["landmarks"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(landmarks.reshape(-1), d["x_ls"][3 * (n - 1):], rtol=0, atol=1e-6)


def test_compute_residual_dropin_signature(gpu_available):
    """bundle_adjustment._compute_residual keeps the reference signature and output."""
    import bundle_adjustment as ba
    from test_oracle_golden import _lists_from_flat
    d = golden("ba_10x200.npz")
    n, m = int(d["n_pose"]), int(d["n_landmark"])
    src, dst, lmk = _lists_from_flat(n, d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"])
    off = d["points_off"]
    pts = [d["points"][off[i]:off[i + 1]] for i in range(n)]
    for x, r_ref in zip(d["xs"][:2], d["rs"][:2]):
        r = ba._compute_residual(x, n, m, int(d["n_residual"]), pts, src, dst, lmk, float(d["u"]), float(d["v"]),
                                 d["ref_pose"])
        np.testing.assert_allclose(r, r_ref, rtol=0, atol=1e-8)


@pytest.mark.parametrize("cfg,ordering", [("config1", 0), ("config2", 0), ("config2", 2), ("config2", 1)])
@pytest.mark.parametrize("precision", [0, 1])
def test_single_gauss_newton_step_is_exact(gpu_available, precision, cfg, ordering):
    """One undamped step (lambda = 0) == the exact solution of J^T J dx = -J^T r with the oracle's
    analytic Jacobian (sparse normal equations), i.e. linearisation + Schur + Cholesky +
    back-substitution are exact.  config2 spans five 32x32 Cholesky tiles and >32 segments per
    Schur wave chunk (the multi-tile / odd-tail paths config1 never reaches).
    ordering 2 forces the nested-dissection system order ([A | B reversed | C], padded tiles, two
    back-substitution chains) that config3 selects on its own.
    Tolerance: fp64 1e-7 relative to |dx|; fp32 2e-3 relative (fp32 normal-equation blocks)."""
    import scipy.sparse.linalg as spla
    import ptzba
    import synthetic
    from oracle import ptz_oracle as orc
    p = synthetic.make_problem(cfg, seed=0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, ordering=ordering)
    if ordering == 2:
        assert h.solver_info()["ordering"] == "nested"
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    h.build_reduced(0.0)
    h.solve_reduced()
    s = h.read_scalars()
    assert s[5] == 0
    h.accept(True)
    ptz1, rays1 = h.get_state()
    h.close()
    dx_gpu = np.concatenate([(ptz1 - p.init_ptz)[1:].reshape(-1), (rays1 - p.init_rays).reshape(-1)])
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm).tocsc()
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    dx = spla.spsolve((J.T @ J).tocsc(), -(J.T @ r))
    tol = 1e-7 if precision == 0 else 2e-3
    err = np.abs(dx_gpu - dx).max() / np.abs(dx).max()
    assert err < tol, err


@pytest.mark.gpu
def test_analytic_jacobian_matches_fd_cpu():
    """CPU check of the Appendix-A Jacobian used by K1 (oracle mirror) against central FD."""
    import synthetic
    from oracle import ptz_oracle as orc
    p = synthetic.make_problem("config1", seed=0)
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm).toarray()
    f = lambda x: orc.compute_residual_records(np.concatenate([p.init_ptz[0], x]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    rng = np.random.default_rng(0)
    for c in rng.choice(len(x0), 40, replace=False):
        e = np.zeros_like(x0)
        e[c] = 1e-5 if c < 3 * (p.n_pose - 1) and c % 3 != 2 else (1e-3 if c < 3 * (p.n_pose - 1) else 1e-5)
        fd = (f(x0 + e) - f(x0 - e)) / (2 * e[c])
        np.testing.assert_allclose(J[:, c], fd, rtol=1e-5, atol=1e-5 * max(1.0, np.abs(fd).max()))


@pytest.mark.parametrize("packed", [False, True])
def test_exchange_region_sums_over_landmark_shards(gpu_available, packed):
    """The N>1 protocol on one device: two landmark-shard handles' exchange regions sum to the
    whole-problem handle's reduced system; after writing the sum back, each shard takes the same pose
    step and its own landmarks' step (bench.py all-reduces exactly these buffers over RCCL)."""
    import torch
    import bench
    import ptzba
    import synthetic
    p = synthetic.make_problem("config2", seed=0)
    win = ptzba.frame_coupling_window(p.n_pose, p.frame, p.landmark)  # global window, as bench.py passes
    hs = []
    for sel in [np.ones(len(p.frame), bool)] + [bench.shard_by_landmark(p.landmark, p.n_landmark, r, 2)
                                                 for r in range(2)]:
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame[sel], p.landmark[sel], p.xy[sel], p.u, p.v, frame_win_hi=win,
                      ordering=ptzba.ORDER_NESTED_FORCE)
        h.set_state(p.init_ptz, p.init_rays)
        h.linearize()
        h.build_reduced(1e-3)
        h.sync()
        hs.append((h, sel))
    views = []
    for h, _ in hs:
        if packed:
            sp, n = h.exchange_packed()
            h.pack()
            h.sync()
        else:
            sp, n, _ = h.exchange()
        views.append(torch.as_tensor(bench._DevArray(sp, n), device="cuda:0"))
    assert len({int(v.numel()) for v in views}) == 1  # same layout on every "rank"
    full = views[0].cpu().numpy()
    summed = (views[1] + views[2])
    err = np.abs(summed.cpu().numpy() - full).max() / np.abs(full).max()
    assert err < 1e-12, err
    views[1].copy_(summed)
    views[2].copy_(summed)
    torch.cuda.synchronize()
    if packed:
        for h, _ in hs[1:]:
            h.unpack()
    for h, _ in hs:
        h.solve_reduced()
    s = [h.read_scalars() for h, _ in hs]
    # trial cost is rank-local: the shards' values add up to the whole problem's
    assert abs(s[1][1] + s[2][1] - s[0][1]) <= 1e-10 * s[0][1]
    for h, _ in hs:
        h.accept(True)
    ptz0, rays0 = hs[0][0].get_state()
    for h, sel in hs[1:]:
        ptz, rays = h.get_state()
        np.testing.assert_allclose(ptz, ptz0, rtol=0, atol=1e-9)
        own = np.unique(p.landmark[sel])
        np.testing.assert_allclose(rays[own], rays0[own], rtol=0, atol=1e-9)
    for h, _ in hs:
        h.close()


@pytest.mark.parametrize("config,precision,loss", [("config1", 0, 0), ("config1", 1, 1), ("config2", 1, 1)])
def test_device_loop_equals_host_loop(gpu_available, config, precision, loss):
    """The device-driven LM (ptzba_lm_*: decisions on the GPU, pipelined trials, single linearisation
    slot with re-linearisation after a rejected trial) takes exactly the host loop's decisions: same
    accepted-iteration count, status and (bitwise-deterministic kernels) the same state."""
    import ptzba
    import synthetic
    p = synthetic.make_problem(config, seed=1)
    out = []
    for device_loop in (False, True):
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, loss=loss,
                      f_scale=1.0)
        h.set_state(p.init_ptz, p.init_rays)
        res = ptzba.LMSolver(h, ftol=1e-8, xtol=1e-12, max_iter=40, device_loop=device_loop).run()
        ptz, rays = h.get_state()
        out.append((res, ptz, rays))
        h.close()
    (rh, ph, yh), (rd, pd, yd) = out
    assert rd.njev == rh.njev and rd.status == rh.status and rd.nfev == rh.nfev, (rh, rd)
    assert abs(rd.cost - rh.cost) <= 1e-12 * rh.cost
    np.testing.assert_allclose(pd, ph, rtol=0, atol=1e-10)
    np.testing.assert_allclose(yd, yh, rtol=0, atol=1e-10)


def test_device_loop_rejections_and_limits(gpu_available):
    """A huge initial damping forces rejected trials (re-linearisation path) and max_iter stops early."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config1", seed=2)
    for kw in (dict(lambda0=1e-9, max_iter=3), dict(lambda0=1e6, max_iter=25)):
        res = []
        for device_loop in (False, True):
            h = ptzba.BAHandle(0)
            h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=0)
            h.set_state(p.init_ptz, p.init_rays)
            res.append((ptzba.LMSolver(h, ftol=1e-10, xtol=1e-14, device_loop=device_loop, **kw).run(), h.get_state()))
            h.close()
        (a, sa), (b, sb) = res
        assert (a.njev, a.nfev, a.status) == (b.njev, b.nfev, b.status), (a, b)
        np.testing.assert_allclose(sb[0], sa[0], rtol=0, atol=1e-10)


def test_save_restore_state_restarts_identically(gpu_available):
    """ptzba_save_state / ptzba_restore_state (device-resident restart point, no host upload): the
    restored state is x0 bit for bit, and a second solve from it repeats the first one exactly
    (deterministic kernels; the Marquardt scaling is reset as by set_state)."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config1", seed=3)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=1, loss=1, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    h.save_state()
    runs = []
    for _ in range(2):
        h.restore_state()
        ptz0, rays0 = h.get_state()
        assert np.array_equal(ptz0, np.asarray(p.init_ptz, np.float64).reshape(ptz0.shape))
        assert np.array_equal(rays0, np.asarray(p.init_rays, np.float64).reshape(rays0.shape))
        res = ptzba.LMSolver(h, ftol=1e-6, xtol=1e-10, max_iter=30).run()
        runs.append((res, h.get_state()))
    (a, sa), (b, sb) = runs
    assert (a.njev, a.nfev, a.status) == (b.njev, b.nfev, b.status) and a.cost == b.cost
    assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
    h.close()


@pytest.mark.parametrize("config,loss", [("config2", "linear"), ("config3", "huber")])
def test_reduced_system_matrix_core_k2_matches_fp64(gpu_available, config, loss):
    """K2 of the fp32 path runs on the matrix cores (k_schur_mf: fp16 hi/lo operand splits with power-of-
    two landmark scaling); the fp64 path keeps the VALU kernel.  At the same linearisation point the two reduced camera systems (S | b | g_pose
    | diag U, the exchange region) agree to the fp32 record precision, element by element against each row's
    scale."""
    import torch
    import bench
    import ptzba
    import synthetic
    p = synthetic.make_problem(config, seed=0)
    lo = ptzba.LOSS_LINEAR if loss == "linear" else ptzba.LOSS_HUBER
    out = []
    for prec in (ptzba.FP64, ptzba.FP32):
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec, loss=lo)
        h.set_state(p.init_ptz, p.init_rays)
        h.linearize()
        h.build_reduced(1e-3)
        h.sync()
        sp, n, _ = h.exchange()
        out.append(torch.as_tensor(bench._DevArray(sp, n), device="cuda:0").cpu().numpy().copy())
        h.close()
    s64, s32 = out
    ld = int(round((-3 + np.sqrt(9 + 4 * len(s64))) / 2))  # region = S [ld x ld] | b | g_pose | diag U
    assert ld * ld + 3 * ld == len(s64)
    S64 = s64[:ld * ld].reshape(ld, ld)
    S32 = s32[:ld * ld].reshape(ld, ld)
    # entry (i, j) against sqrt(|S_ii| |S_jj|), the scale of a symmetric positive semi-definite block
    d = np.sqrt(np.abs(np.diag(S64)) + 1e-300)
    rel = np.abs(S32 - S64) / (np.outer(d, d) + 1e-300)
    low = np.tril(np.ones_like(S64, dtype=bool))
    live = low & (np.outer(d, d) > 0)
    err = rel[live].max()
    print(f"{config}: max |S32 - S64| / sqrt(S_ii S_jj) = {err:.3e}")
    assert err < 1e-4, err
    tail = np.abs(s32[ld * ld:] - s64[ld * ld:]).max() / max(np.abs(s64[ld * ld:]).max(), 1e-300)
    assert tail < 1e-5, tail


@pytest.mark.parametrize("config,knob", [("config2", "PTZBA_BS_PERSIST=0"), ("grid", "PTZBA_BS_PERSIST=0")])
def test_single_launch_schedules_bitwise_equal(gpu_available, config, knob, monkeypatch):
    """Schedule-only forms of the back-substitution give bit-identical LM iterates: PTZBA_BS_PERSIST=0 -- the per-step
    blocked back-substitution against the single-launch one (the default, per-column counters).  config 2 (natural /
    one-level plan) and the 3-row grid (delayed trailing updates: the second panel pair and 2 x 2 trailing blocks); 3
    solves of 3 LM iterations per handle, so the counters run over several epochs."""
    import ptzba
    import synthetic
    if config == "grid":
        p = synthetic.make_grid_problem(120, 6000, -20.0, 20.0, (-10.0, 0.0, 10.0), seed=3)
    else:
        p = synthetic.make_problem(config, seed=0)
    name, val = knob.split("=")
    out = []
    for v in ("0" if val == "1" else "1", val):
        monkeypatch.setenv(name, v)
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
        h.set_state(p.init_ptz, p.init_rays)
        h.save_state()
        rs = [h.solve_resident(restore=True, ftol=1e-14, xtol=1e-16, max_iter=3) for _ in range(3)]
        out.append((h.get_state(), [(r.cost, r.njev, r.nfev, r.status) for r in rs]))
        h.close()
    (a_ptz, a_rays), a_res = out[0]
    (b_ptz, b_rays), b_res = out[1]
    assert a_res == b_res
    assert np.array_equal(a_ptz, b_ptz) and np.array_equal(a_rays, b_rays)


def test_fused_prepare_matches_separate_prepare(gpu_available, monkeypatch):
    """The single-GPU build writes the augmented row, the padding pivots and the pose damping itself (fused prepare,
    k_build_prologue + the Schur kernel); PTZBA_NO_FUSED_PREP=1 runs k_chol_prepare before the factorisation instead.
    Config 2's system has padding rows 147-159 (index mod 32 = 19-31: rows whose diagonal lies in a double2 another
    wave zeroes -- the race ADVICE r3 found): the LM iterates agree bit for bit over 3 solves."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config2", seed=0)
    out = []
    for v in (None, "1"):
        if v is None:
            monkeypatch.delenv("PTZBA_NO_FUSED_PREP", raising=False)
        else:
            monkeypatch.setenv("PTZBA_NO_FUSED_PREP", v)
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                      loss=ptzba.LOSS_HUBER)
        si = h.solver_info()
        assert si["ld"] > si["n_aug"]  # padding rows present
        h.set_state(p.init_ptz, p.init_rays)
        h.save_state()
        rs = [h.solve_resident(restore=True, ftol=1e-14, xtol=1e-16, max_iter=4) for _ in range(3)]
        out.append((h.get_state(), [(r.cost, r.njev, r.nfev, r.status) for r in rs]))
        h.close()
    (a_ptz, a_rays), a_res = out[0]
    (b_ptz, b_rays), b_res = out[1]
    assert a_res == b_res
    assert np.array_equal(a_ptz, b_ptz) and np.array_equal(a_rays, b_rays)


def test_setup_timing_reports_set_problem_phases(gpu_available):
    """ptzba_setup_timing: the host phases of the last set_problem (names and ms), replacing round 4's env knob."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config2", seed=0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32)
    t = h.setup_timing()
    h.close()
    assert len(t) >= 4 and all(v >= 0.0 for v in t.values()), t
    assert "upload+alloc" in t, t


def test_host_loop_curvature_does_not_carry_over(gpu_available):
    """a host-driven Huber run that took the curvature switch must not leave its reduced curvature on the
    handle.  Two host runs on one handle (the first switches, the second runs with curvature_switch=0, i.e. IRLS
    throughout) equal the IRLS run on a fresh handle bit for bit, and a direct linearize() after a switched run gives
    the IRLS cost again (the handle is back at curvature 1)."""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config1", seed=5)

    def handle():
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64,
                      loss=ptzba.LOSS_HUBER, f_scale=1.0)
        return h

    kw = dict(ftol=1e-10, xtol=1e-14, max_iter=20, device_loop=False)
    h = handle()
    h.set_state(p.init_ptz, p.init_rays)
    r1 = ptzba.LMSolver(h, curvature_switch=0.25, **kw).run()
    assert r1.njev > 0
    h.set_state(p.init_ptz, p.init_rays)
    r2 = ptzba.LMSolver(h, curvature_switch=0.0, **kw).run()
    s2 = h.get_state()
    r1b = ptzba.LMSolver(h, curvature_switch=0.25, **kw).run()  # switches again, then the handle must be back at IRLS

    def one_step(hh):  # a direct step: its predicted reduction depends on the curvature of the linearisation
        hh.set_state(p.init_ptz, p.init_rays)
        hh.linearize()
        hh.build_reduced(1e-3)
        hh.solve_reduced()
        return np.asarray(hh.read_scalars()[:3], np.float64)

    c_after = one_step(h)
    h.close()
    f = handle()
    c_fresh = one_step(f)
    f.set_state(p.init_ptz, p.init_rays)
    rf = ptzba.LMSolver(f, curvature_switch=0.0, **kw).run()
    sf = f.get_state()
    f.close()
    assert (r2.njev, r2.nfev, r2.status, r2.cost) == (rf.njev, rf.nfev, rf.status, rf.cost), (r2, rf)
    assert np.array_equal(s2[0], sf[0]) and np.array_equal(s2[1], sf[1])
    assert r1b.njev > 0 and np.array_equal(c_after, c_fresh), (c_after, c_fresh)


def test_lm_opts_zero_filled_curvature_fields(gpu_available):
    """ptzba_lm_init reads huber_curvature / curvature_switch for the Huber loss only, and 0 selects the
    default curvature, so a caller that zero-fills the two fields added in ABI 0.2 is not rejected: a linear-loss solve
    with both fields 0 equals the default-option solve, and a Huber solve with both 0 runs IRLS throughout (equal to
    curvature_switch=0)."""
    import ptzba
    import synthetic
    assert "0.2" in ptzba.lib().ptzba_version().decode()
    p = synthetic.make_problem("config1", seed=6)
    for loss in (ptzba.LOSS_LINEAR, ptzba.LOSS_HUBER):
        out = []
        for hc, cs in ((0.0, 0.0), (ptzba.HUBER_CURVATURE, 0.0 if loss == ptzba.LOSS_HUBER else ptzba.CURVATURE_SWITCH)):
            h = ptzba.BAHandle(0)
            h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64, loss=loss,
                          f_scale=1.0)
            h.set_state(p.init_ptz, p.init_rays)
            r = ptzba.LMSolver(h, ftol=1e-10, xtol=1e-14, max_iter=20, huber_curvature=hc, curvature_switch=cs).run()
            out.append((r.njev, r.status, r.cost, h.get_state()[0].copy()))
            h.close()
        assert out[0][:3] == out[1][:3], (loss, out[0][:3], out[1][:3])
        assert np.array_equal(out[0][3], out[1][3])


@pytest.mark.parametrize("config,precision,weighted", [("config2", 0, False), ("config2", 1, False), ("config2", 1, True),
                                                       ("config2", 0, True), ("config3", 1, False), ("config3", 0, True)])
def test_device_and_host_setup_fronts_bitwise_equal(gpu_available, config, precision, weighted):
    """set_problem's device front (rocPRIM sort, segment / record kernels; the default from 64K records) and
    the host front (counting sorts) build the same arrays bit for bit.  ptzba_set_setup_front picks the front per
    handle; the record-order residual (through the permutation), the LM iterates and the final state of 2 x 3 LM
    iterations agree bitwise -- fp64 and fp32, weighted (dedup form) and unweighted records, config 2 and 3."""
    import ptzba
    import synthetic
    p = synthetic.make_problem(config, seed=0)
    frame, landmark, xy, w = p.frame, p.landmark, p.xy, None
    if weighted:
        frame, landmark, xy, w, _ = synthetic.dedup_records(frame, landmark, xy)
    rng = np.random.default_rng(1)
    x_full = np.concatenate([np.asarray(p.init_ptz).reshape(-1), np.asarray(p.init_rays).reshape(-1)])
    x_full = x_full + rng.normal(0, 1e-3, x_full.shape)
    out = []
    for front in (2 ** 62, 0):  # host, device
        h = ptzba.BAHandle(0)
        h.set_setup_front(front)
        h.set_problem(p.n_pose, p.n_landmark, frame, landmark, xy, p.u, p.v, weight=w, precision=precision,
                      loss=ptzba.LOSS_HUBER, f_scale=1.0)
        assert h.setup_timing()  # (phases recorded either way)
        r = h.residual(x_full)
        h.set_state(p.init_ptz, p.init_rays)
        h.save_state()
        rs = [h.solve_resident(restore=True, ftol=1e-12, xtol=1e-14, max_iter=3) for _ in range(2)]
        out.append((r, h.get_state(), [(x.cost, x.njev, x.nfev, x.status) for x in rs], h.info()))
        h.close()
    (ra, sa, la, ia), (rb, sb, lb, ib) = out
    assert ia == ib
    assert np.array_equal(ra, rb)
    assert la == lb
    assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])


@pytest.mark.parametrize("config", ["config1", "config2"])
@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("loss", [0, 1])
def test_initial_cost_is_finite_and_matches_oracle(gpu_available, config, precision, loss):
    """a round-5 working-tree build of K1 (never committed) produced a NaN cost at x0
    in fp32 (config 2, linear loss: initial_cost=nan, njev=0, reported as a damping-limit stop).  Every precision x loss
    combination's x0 linearisation must give the oracle's cost (fp64 1e-10, fp32 2e-6 relative), and the LM must hand
    back the same initial cost."""
    import ptzba
    import synthetic
    from oracle import ptz_oracle as orc
    p = synthetic.make_problem(config, seed=0)
    x_full = np.concatenate([np.asarray(p.init_ptz).reshape(-1), np.asarray(p.init_rays).reshape(-1)])
    want = orc.ba_cost(x_full, p.n_pose, p.u, p.v, p.frame.astype(np.int64), p.landmark.astype(np.int64), p.xy,
                       loss="huber" if loss else "linear", f_scale=1.0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, loss=loss, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    got = float(h.read_scalars()[0])
    tol = 1e-10 if precision == 0 else 2e-6
    assert np.isfinite(got) and abs(got - want) <= tol * want, (got, want)
    h.set_state(p.init_ptz, p.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=5).run()
    assert np.isfinite(res.initial_cost) and abs(res.initial_cost - want) <= tol * want
    assert res.njev >= 1 and res.status in (0, 2, 3)
    h.close()


@pytest.mark.parametrize("device_loop", [True, False])
def test_non_finite_initial_residual_raises_like_scipy(gpu_available, device_loop):
    """A non-finite x0 (here one ray's theta) makes the residual non-finite: scipy's least_squares raises
    ValueError("Residuals are not finite in the initial point."); the drop-in LM raises the same instead of reporting a
    damping-limit stop.  (Non-finite observations are already refused by set_problem.)"""
    import ptzba
    import synthetic
    p = synthetic.make_problem("config1", seed=0)
    rays = np.array(p.init_rays, np.float64)
    rays[int(p.landmark[7]), 0] = np.nan
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=1)
    h.set_state(p.init_ptz, rays)
    with pytest.raises(ValueError, match="not finite in the initial point"):
        ptzba.LMSolver(h, ftol=1e-4, device_loop=device_loop).run()
    h.close()
