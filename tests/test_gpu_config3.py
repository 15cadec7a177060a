"""GPU parity at the headline size (BASELINE configs[2]: 500 keyframes x 20k rays, 14.6M pair-form
records) and at shapes the small fixtures never reach.

The reference cannot run at config 3 (dense FD Jacobian ~9.7 PB), so parity here rests on
the oracle (oracle/ptz_oracle.py, pinned to reference runs by test_oracle_golden.py) evaluated on the
same records, and on size-independent properties:
  * fp64 residual vector at x0 == oracle `compute_residual_records` (the vectorised restatement of
    bundle_adjustment._compute_residual, :25-106) on all 29.2M residuals, atol 1e-8 px;
  * fp32 LM + Huber (the bench configuration) and fp64 LM + Huber converge to the same poses:
    pan / tilt / f RMSE <= 1e-4 (north-star gate);
  * at the fp64 linear-loss optimum the oracle's analytic gradient J^T r (per-record 2x5 Jacobian,
    SURVEY Appendix A) is <= 1e-6 of its value at x0 (first-order optimality of the reference cost).
  * at the pinned oracle's tight optimum (tests/golden/config3_optimum.npz) the GPU's fp32-Huber and fp64-linear
    solves agree to pan / tilt / f RMSE <= 1e-4 -- BASELINE's "RMSE vs reference" at the headline.
Also: landmarks seen in more than K1's 128-segment window (window-crossing path of K1), and the one-shot
C entry ptzba_solve against the Python-driven LM."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def config3():
    import synthetic
    return synthetic.make_problem("config3", seed=0)


def _oracle_gradient(p, ptz, rays, loss="linear", f_scale=1.0):
    """Gradient of the pair-form cost at (ptz, rays): [n_pose, 3] pose part, [M, 2] ray part.  linear: J^T r;
    huber: scipy's convention (cost 0.5 f^2 sum rho((r_i / f)^2) over SCALAR residuals, rho' = 1 inside the
    unit and 1/sqrt(z) beyond), i.e. J^T (rho'(z) * r) with z per residual component."""
    from oracle import ptz_oracle as orc
    fr = p.frame.astype(np.int64)
    lm = p.landmark.astype(np.int64)
    x_full = np.concatenate([np.asarray(ptz).reshape(-1), np.asarray(rays).reshape(-1)])
    gp = np.zeros((p.n_pose, 3))
    gr = np.zeros((p.n_landmark, 2))
    chunk = 2_000_000  # bounded host memory for the [R, 2, 5] Jacobian
    for a in range(0, len(fr), chunk):
        b = min(len(fr), a + chunk)
        r = orc.compute_residual_records(x_full, p.n_pose, p.u, p.v, fr[a:b], lm[a:b], p.xy[a:b]).reshape(-1, 2)
        J = orc.record_jacobian(p.u, p.v, np.asarray(ptz)[fr[a:b]], np.asarray(rays)[lm[a:b]])
        if loss == "huber":
            z = (r / f_scale) ** 2
            r = r * np.where(z <= 1.0, 1.0, 1.0 / np.sqrt(np.maximum(z, 1.0)))
        g = np.einsum("rkc,rk->rc", J, r)
        np.add.at(gp, fr[a:b], g[:, :3])
        np.add.at(gr, lm[a:b], g[:, 3:])
    gp[0] = 0.0  # frame 0 is the fixed gauge (bundle_adjustment.py:197)
    return gp, gr


def test_config3_residual_fp64_matches_oracle(gpu_available, config3):
    import ptzba
    from oracle import ptz_oracle as orc
    p = config3
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
    assert h.info()["n_obs"] == len(p.frame) > 14_000_000
    x_full = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    r = h.residual(x_full)
    h.close()
    r_ref = orc.compute_residual_records(x_full, p.n_pose, p.u, p.v, p.frame.astype(np.int64),
                                         p.landmark.astype(np.int64), p.xy)
    assert r.shape == r_ref.shape == (2 * len(p.frame),)
    np.testing.assert_allclose(r, r_ref, rtol=0, atol=1e-8)


def test_config3_fp32_huber_equals_fp64_huber(gpu_available, config3):
    """The headline configuration (fp32 records, Huber) converges to the fp64 optimum: RMSE <= 1e-4."""
    import ptzba
    import synthetic
    p = config3
    out = []
    for prec, tol in ((ptzba.FP32, 1e-10), (ptzba.FP64, 1e-12)):
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec,
                      loss=ptzba.LOSS_HUBER, f_scale=1.0)
        h.set_state(p.init_ptz, p.init_rays)
        res = ptzba.LMSolver(h, ftol=tol, xtol=1e-12, max_iter=60).run()
        ptz, rays = h.get_state()
        h.close()
        # fp32: ftol=1e-10 is below the fp32 cost's round-off (~1e-7 relative), so the last trials may find no
        # resolvable decrease at the optimum (damping limit, status 5); the cost and poses are gated below
        ok = (1, 2, 3, ptzba.STATUS_DAMPING) if prec == ptzba.FP32 else (1, 2, 3)
        assert res.status in ok and res.cost < res.initial_cost, res
        out.append((res, ptz, rays))
    (r32, p32, y32), (r64, p64, y64) = out
    rmse = synthetic.pose_rmse(p32, p64)
    assert np.all(rmse <= 1e-4), rmse
    assert abs(r32.cost - r64.cost) <= 1e-6 * r64.cost
    # the solve recovers the generating poses to the noise level (0.5 px keypoint noise)
    gt = synthetic.pose_rmse(p64, p.gt_ptz)
    assert gt[0] < 0.01 and gt[1] < 0.01 and gt[2] < 1.0, gt


def test_config3_fp64_optimum_is_stationary_for_oracle_cost(gpu_available, config3):
    """First-order optimality of the reference cost at the GPU's fp64 linear-loss optimum, judged by the
    oracle's own analytic gradient: |J^T r|_inf at x* <= 1e-6 |J^T r|_inf at x0 (poses and rays)."""
    import ptzba
    p = config3
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
    h.set_state(p.init_ptz, p.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-15, xtol=1e-15, max_iter=80).run()
    ptz, rays = h.get_state()
    h.close()
    gp0, gr0 = _oracle_gradient(p, p.init_ptz, p.init_rays)
    gp, gr = _oracle_gradient(p, ptz, rays)
    # per parameter kind (deg vs px units differ): pan, tilt, f, theta, phi
    for k in range(3):
        assert np.abs(gp[:, k]).max() <= 1e-6 * np.abs(gp0[:, k]).max(), (k, np.abs(gp[:, k]).max(), res)
    for k in range(2):
        assert np.abs(gr[:, k]).max() <= 1e-6 * np.abs(gr0[:, k]).max(), (3 + k, np.abs(gr[:, k]).max(), res)


def test_config3_fp32_huber_optimum_is_stationary_for_oracle_cost(gpu_available, config3):
    """The HEADLINE arithmetic pinned to the oracle: at the optimum of the fp32 records + Huber solve (the bench
    configuration, matrix-core K2), the oracle's fp64 Huber gradient of the reference residual (scipy's rho'
    weights on the per-record 2x5 Jacobian, bundle_adjustment.py:25-106 with least_squares(loss='huber')) is
    <= 1e-5 of its value at x0, per parameter kind.  (fp32 records and the fp16-split Schur products bound how
    far below that the fp32 solve can get; the fp64 linear-loss test above gates 1e-6.)"""
    import ptzba
    p = config3
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-12, xtol=1e-14, max_iter=60).run()
    ptz, rays = h.get_state()
    h.close()
    gp0, gr0 = _oracle_gradient(p, p.init_ptz, p.init_rays, "huber")
    gp, gr = _oracle_gradient(p, ptz, rays, "huber")
    ratios = [np.abs(gp[:, k]).max() / np.abs(gp0[:, k]).max() for k in range(3)] + \
             [np.abs(gr[:, k]).max() / np.abs(gr0[:, k]).max() for k in range(2)]
    print(f"fp32-huber stationarity |g*|/|g0| per kind (pan, tilt, f, theta, phi): {ratios}, {res}")
    assert max(ratios) <= 1e-5, (ratios, res)


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("weighted", [False, True])
def test_landmarks_longer_than_k1_window(gpu_available, precision, weighted):
    """Landmarks seen in up to 256 frames (> K1_SEGW = 128 segments): K1 walks each landmark in several
    128-segment windows and masks the neighbouring windows' records inside shared 4-record groups.
    One undamped step equals the oracle's sparse normal-equation solution (as
    test_single_gauss_newton_step_is_exact), pair form and de-duplicated weighted form."""
    import scipy.sparse.linalg as spla
    import ptzba
    import synthetic
    from oracle import ptz_oracle as orc
    p = synthetic.make_small_problem(260, 80, 50.0, 52.0, seed=5)  # every frame observed
    fr, lm, xy, w = p.frame, p.landmark, p.xy, None
    if weighted:
        fr, lm, xy, w, _ = synthetic.dedup_records(fr, lm, xy)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, fr, lm, xy, p.u, p.v, weight=w, precision=precision)
    assert h.info()["max_seg_per_landmark"] > 128
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    h.build_reduced(0.0)
    h.solve_reduced()
    assert h.read_scalars()[5] == 0
    h.accept(True)
    ptz1, rays1 = h.get_state()
    h.close()
    dx_gpu = np.concatenate([(ptz1 - p.init_ptz)[1:].reshape(-1), (rays1 - p.init_rays).reshape(-1)])
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    f64, l64 = fr.astype(np.int64), lm.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], f64, l64).tocsc()
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, f64, l64, xy)
    if w is not None:
        sw = np.repeat(np.sqrt(w), 2)
        J = (J.T.multiply(sw)).T.tocsc()
        r = r * sw
    dx = spla.spsolve((J.T @ J).tocsc(), -(J.T @ r))
    tol = 1e-7 if precision == 0 else 2e-3
    err = np.abs(dx_gpu - dx).max() / np.abs(dx).max()
    assert err < tol, err


@pytest.mark.parametrize("config,precision,loss", [("config1", 0, 0), ("config2", 1, 1)])
def test_one_shot_solve_equals_lm_solver(gpu_available, config, precision, loss):
    """ptzba_solve (the C-driven LM, include/ptzba.h) takes the same decisions as ptzba.LMSolver's
    device loop: same iterations, status and state; inputs are carried in and results out through the
    caller's buffers."""
    import ptzba
    import synthetic
    p = synthetic.make_problem(config, seed=4)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, loss=loss)
    h.set_state(p.init_ptz, p.init_rays)
    ref = ptzba.LMSolver(h, ftol=1e-8, xtol=1e-12, max_iter=40).run()
    ptz_ref, rays_ref = h.get_state()
    ptz, rays, res = h.solve(p.init_ptz, p.init_rays, ftol=1e-8, xtol=1e-12, max_iter=40)
    h.close()
    assert (res.njev, res.nfev, res.status) == (ref.njev, ref.nfev, ref.status), (res, ref)
    assert res.cost == ref.cost and res.initial_cost == ref.initial_cost
    assert np.array_equal(ptz, ptz_ref) and np.array_equal(rays, rays_ref)


def test_config3_two_level_dissection_matches_one_level(gpu_available, config3, monkeypatch):
    """The default order at config 3 is the two-level nested dissection (26 elimination levels, four
    back-substitution chains: api.hip nested_order2); it must give the same LM iterates as the one-level order
    [A | B reversed | C] (PTZBA_ND_DEPTH=1): fp64 linear loss, 4 iterations, poses within 1e-9 deg / 1e-7 px,
    rays within 1e-9 deg, same iteration count and cost to 1e-12 relative."""
    import ptzba
    p = config3
    out = {}
    for depth in ("1", "2"):
        monkeypatch.setenv("PTZBA_ND_DEPTH", depth)
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
        info = h.solver_info()
        assert info["nd_depth"] == int(depth), info
        h.set_state(p.init_ptz, p.init_rays)
        # damped start (rounds 1-4's default): with Gauss-Newton steps the 4th trial sits at round-off, where its
        # acceptance depends on the summation order the two orders differ in
        res = ptzba.LMSolver(h, ftol=1e-15, xtol=1e-15, max_iter=4, lambda0=1e-4).run()
        out[depth] = (h.get_state(), res, info)
        h.close()
    (ptz1, rays1), r1, i1 = out["1"]
    (ptz2, rays2), r2, i2 = out["2"]
    assert i1["levels"] == 30 and i2["levels"] == 26, (i1, i2)
    assert r1.njev == r2.njev and r1.nfev == r2.nfev
    assert abs(r1.cost - r2.cost) <= 1e-12 * r1.cost
    np.testing.assert_allclose(ptz2[:, :2], ptz1[:, :2], rtol=0, atol=1e-9)
    np.testing.assert_allclose(ptz2[:, 2], ptz1[:, 2], rtol=0, atol=1e-7)
    np.testing.assert_allclose(rays2, rays1, rtol=0, atol=1e-9)


def _config3_optimum(p):
    """tests/golden/config3_optimum.npz (make_golden.py gen_config3): the pinned oracle's tight optimum of the
    reference cost at the headline size, checked to belong to these records."""
    from conftest import golden
    d = golden("config3_optimum.npz")
    assert int(d["n_records"]) == len(p.frame) and int(d["frame_sum"]) == int(p.frame.astype(np.int64).sum())
    assert int(d["landmark_sum"]) == int(p.landmark.astype(np.int64).sum())
    assert abs(float(d["xy_sum"]) - float(p.xy.sum())) <= 1e-9 * abs(float(d["xy_sum"]))
    return d


@pytest.mark.parametrize("arith", ["fp32_huber", "fp64_linear"])
def test_config3_optimum_matches_oracle_fixture(gpu_available, config3, arith):
    """BASELINE's "pan-tilt-focal RMSE vs reference" at the headline (500 KF x 20k rays): the GPU solve against the
    tight optimum of the oracle restatement of the reference residual (bundle_adjustment.py:25-106, :200-202 with
    frame 0 as the gauge), tests/golden/config3_optimum.npz.  fp32_huber is the bench's arithmetic (fp32 records,
    matrix-core K2, scipy's loss='huber') vs the fixture's Huber optimum; fp64_linear is the reference's own
    arithmetic vs its linear-loss optimum.  Gate (north star): pan / tilt / f RMSE <= 1e-4 (deg, deg, px) for the
    converged solve; rays RMSE <= 1e-4 deg; cost within 1e-7 relative.  The solve stopped by the reference's own rule
    (ftol = 1e-4, what bench.py times) meets the same pose gate since round 5 (Gauss-Newton start, huber curvature
    switch: ptzba.LAMBDA0 / HUBER_CURVATURE), its rays within 1e-3 deg."""
    import ptzba
    import synthetic
    p = config3
    d = _config3_optimum(p)
    prec, loss, key = ((ptzba.FP32, ptzba.LOSS_HUBER, "_huber") if arith == "fp32_huber"
                       else (ptzba.FP64, ptzba.LOSS_LINEAR, ""))
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec, loss=loss, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    h.save_state()
    r_ref = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100).run()  # the reference's termination
    ptz_ref, rays_ref = h.get_state()
    h.restore_state()
    res = ptzba.LMSolver(h, ftol=1e-12, xtol=1e-14, max_iter=60).run()
    ptz, rays = h.get_state()
    h.close()
    pt, rt, ct = d["ptz_tight" + key], d["rays_tight" + key], float(d["tight_cost" + key])
    rmse = synthetic.pose_rmse(ptz, pt)
    rmse_ref = synthetic.pose_rmse(ptz_ref, pt)
    ray_rmse = float(np.sqrt(np.mean((rays - rt) ** 2)))
    ray_rmse_ref = float(np.sqrt(np.mean((rays_ref - rt) ** 2)))
    print(f"{arith}: pose RMSE vs oracle optimum {rmse} (ftol=1e-4 solve: {rmse_ref}, rays {ray_rmse_ref:.3e} deg, "
          f"{r_ref.njev} its), rays {ray_rmse:.3e} deg, cost {res.cost:.10f} vs {ct:.10f}")
    assert np.all(rmse <= 1e-4), rmse
    # the solve stopped by the reference's own rule (ftol = 1e-4: ~4 iterations at this size)
    assert np.all(rmse_ref <= 1e-4), rmse_ref
    assert ray_rmse_ref <= 1e-3, ray_rmse_ref
    assert ray_rmse <= 1e-4
    assert abs(res.cost - ct) <= 1e-7 * ct


@pytest.mark.parametrize("knob", ["PTZBA_BS_PERSIST=1"])
def test_config3_schedule_knobs_bitwise_equal(gpu_available, config3, monkeypatch, knob):
    """Schedule-only variants of the factorisation / back-substitution give bit-identical LM iterates at config 3 (the
    same arithmetic in the same order): PTZBA_BS_PERSIST=1 -- every back-substitution step in ONE launch with
    per-column update counters (k_chol_backsolve_pst).  (Round 6 removed the PTZBA_CHOL_COH=0 plain-access knob: the
    level launches' coherent tile traffic is the only SPD form.)  4 LM iterations in the headline arithmetic, twice (the persistent
    back-solve's counters advance by one epoch per launch)."""
    import ptzba
    p = config3
    name, val = knob.split("=")
    out = []
    for v in ("0", val):
        monkeypatch.setenv(name, v)
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                      loss=ptzba.LOSS_HUBER, f_scale=1.0)
        h.set_state(p.init_ptz, p.init_rays)
        h.save_state()
        rs = [h.solve_resident(restore=True, ftol=1e-12, xtol=1e-14, max_iter=4) for _ in range(2)]
        out.append((h.get_state(), [(r.cost, r.njev, r.nfev) for r in rs]))
        h.close()
    (a_ptz, a_rays), a_res = out[0]
    (b_ptz, b_rays), b_res = out[1]
    assert a_res == b_res
    assert np.array_equal(a_ptz, b_ptz) and np.array_equal(a_rays, b_rays)
