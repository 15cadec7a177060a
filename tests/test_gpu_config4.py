"""GPU tests of BASELINE configs[3] (5000 keyframes x 200k rays in 10 tilt rows; 410M pair-form records)
and of the multi-row keyframe grid it is built from.

On a row-major keyframe grid a landmark seen by two tilt rows spans a whole row of frame indices, so
the solver paths config 3 never reaches are exercised here: Schur chunk lists with per-landmark frame
gaps, a coupling band of ~57 tiles (nested dissection on a 2-D coupled grid), and the back substitutions
for update lists larger than LDS (blocked right-looking, the default there, and left-looking).  Parity is the same as for the small configs: one
undamped step equals the oracle's sparse normal-equation solution (bundle_adjustment.py:25-106 via
oracle/ptz_oracle.py); at full size, the fp64 residual vector against the oracle on a sample of records,
the cost K1 reduces against the residual vector, and a monotone LM descent (bundle_adjustment.py:200-202).
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gn_step(p, precision, ordering):
    import ptzba
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, ordering=ordering)
    info = h.solver_info()
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    h.build_reduced(0.0)
    h.solve_reduced()
    assert h.read_scalars()[5] == 0
    h.accept(True)
    ptz1, rays1 = h.get_state()
    h.close()
    return np.concatenate([(ptz1 - p.init_ptz)[1:].reshape(-1), (rays1 - p.init_rays).reshape(-1)]), info


@pytest.fixture(scope="module")
def grid():
    import synthetic
    # 3 tilt rows x 40 keyframes: landmarks seen by two rows leave gaps of ~20-40 frames in their range
    return synthetic.make_grid_problem(120, 6000, -20.0, 20.0, (-10.0, 0.0, 10.0), seed=3)


@pytest.mark.parametrize("backsolve", ["lookahead", "ll", "blk"])
@pytest.mark.parametrize("ordering", [0, 1, 2])
def test_grid_gauss_newton_step_is_exact(gpu_available, grid, monkeypatch, backsolve, ordering):
    import scipy.sparse.linalg as spla
    from oracle import ptz_oracle as orc
    p = grid
    monkeypatch.setenv("PTZBA_BACKSOLVE", {"lookahead": "la", "ll": "ll", "blk": "blk"}[backsolve])
    dx_gpu, info = _gn_step(p, 0, ordering)
    assert info["backsolve"] == {"lookahead": "lookahead", "ll": "left-looking", "blk": "blocked"}[backsolve]
    if ordering != 1:  # 1: the solver's choice (natural, one or two dissection levels)
        assert info["ordering"] == ("nested" if ordering == 2 else "natural")
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm).tocsc()
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    dx = spla.spsolve((J.T @ J).tocsc(), -(J.T @ r))
    err = np.abs(dx_gpu - dx).max() / np.abs(dx).max()
    assert err < 1e-7, err


@pytest.mark.parametrize("blocks", ["1", "0"])
@pytest.mark.parametrize("ordering", [0, 1, 2])
def test_grid_delayed_trailing_updates_exact(gpu_available, grid, monkeypatch, ordering, blocks):
    """The factorisation with delayed trailing updates (PTZBA_CHOL_DELAY=2: trailing tasks every other level,
    up to four update panels per task; config 4's default), with the trailing tiles in 2 x 2 block tasks (the
    default) or one task per tile (PTZBA_CHOL_BLOCKS=0), gives the same exact Gauss-Newton step."""
    import scipy.sparse.linalg as spla
    from oracle import ptz_oracle as orc
    p = grid
    monkeypatch.setenv("PTZBA_CHOL_DELAY", "2")
    monkeypatch.setenv("PTZBA_CHOL_BLOCKS", blocks)
    dx_gpu, info = _gn_step(p, 0, ordering)
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm).tocsc()
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    dx = spla.spsolve((J.T @ J).tocsc(), -(J.T @ r))
    err = np.abs(dx_gpu - dx).max() / np.abs(dx).max()
    assert err < 1e-7, err


@pytest.mark.parametrize("ordering", [0, 2])
def test_grid_trailing_blocks_bitwise_equal_per_tile_tasks(gpu_available, grid, monkeypatch, ordering):
    """2 x 2 trailing-block tasks apply the union of their tiles' update panels in the same order as one task per
    tile (the extra panels multiply zero tiles): the Gauss-Newton step is bitwise the same."""
    monkeypatch.setenv("PTZBA_CHOL_DELAY", "2")
    monkeypatch.setenv("PTZBA_CHOL_BLOCKS", "1")
    dx_blk, _ = _gn_step(grid, 1, ordering)
    monkeypatch.setenv("PTZBA_CHOL_BLOCKS", "0")
    dx_tile, _ = _gn_step(grid, 1, ordering)
    assert np.array_equal(dx_blk, dx_tile)


@pytest.fixture(scope="module")
def config4():
    import synthetic
    t0 = time.time()
    p = synthetic.make_problem("config4", seed=0)
    print(f"config4 generated in {time.time() - t0:.1f} s: {p.n_pose} KF, {p.n_landmark} landmarks, "
          f"{len(p.frame)} records, {p.n_pairs} pairs", flush=True)
    return p


@pytest.mark.timeout(900)
def test_config4_residual_fp64_matches_oracle(gpu_available, config4):
    """fp64 residual vector of the full config-4 problem at x0: every residual the GPU returns for a
    random sample of 2M records equals the oracle's (atol 1e-8 px), and 1/2 |r|^2 over all 820M residuals
    equals the initial cost K1 reduces."""
    import ptzba
    from oracle import ptz_oracle as orc
    p = config4
    t0 = time.time()
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
    info, sinfo = h.info(), h.solver_info()
    print(f"set_problem fp64 {time.time() - t0:.1f} s; {info}; {sinfo}", flush=True)
    assert info["n_obs"] == len(p.frame) > 300_000_000
    assert sinfo["backsolve"] == "blocked"
    x_full = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    r = h.residual(x_full)
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    cost_k1 = h.read_scalars()[0]
    h.close()
    rng = np.random.default_rng(0)
    idx = np.sort(rng.choice(len(p.frame), 2_000_000, replace=False))
    r_ref = orc.compute_residual_records(x_full, p.n_pose, p.u, p.v, p.frame[idx].astype(np.int64),
                                         p.landmark[idx].astype(np.int64), p.xy[idx]).reshape(-1, 2)
    np.testing.assert_allclose(r.reshape(-1, 2)[idx], r_ref, rtol=0, atol=1e-8)
    cost = 0.5 * float(np.dot(r, r))
    assert abs(cost - cost_k1) <= 1e-9 * cost, (cost, cost_k1)


@pytest.mark.timeout(900)
def test_config4_lm_three_iterations(gpu_available, config4):
    """set_problem + 3 LM iterations at full size in the headline arithmetic (fp32 records, Huber): every
    iteration is accepted or retried by the reference's rules and the cost decreases monotonically from
    the one fp64 K1 computes; the solve is structurally the blocked back-substitution / nested path."""
    import ptzba
    p = config4
    t0 = time.time()
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    print(f"set_problem fp32 {time.time() - t0:.1f} s; {h.info()}; {h.solver_info()}", flush=True)
    h.set_state(p.init_ptz, p.init_rays)
    h.reset_kernel_times(True, groups=0xF)
    costs = []
    t1 = time.time()
    for _ in range(3):
        res = ptzba.LMSolver(h, ftol=1e-12, xtol=1e-14, max_iter=1).run()
        costs.append((res.initial_cost, res.cost, res.njev))
    h.sync()
    dt = time.time() - t1
    kt = h.kernel_times()
    h.close()
    print(f"config4 3 LM iterations in {dt:.2f} s; costs {costs}; kernel ms {kt}", flush=True)
    for c0, c1, nj in costs:
        assert nj == 1 and c1 < c0
    assert costs[1][0] == costs[0][1] and costs[2][0] == costs[1][1]
    assert costs[2][1] < 0.5 * costs[0][0]


def _sampled_gradient(p, ptz, rays, frames, landmarks, loss="huber"):
    """Oracle gradient of the pair-form cost (scipy's huber rho' weights, bundle_adjustment.py:25-106 residual,
    SURVEY Appendix A Jacobian) restricted to a sample: the pose gradient of `frames` (from all their records) and
    the ray gradient of `landmarks` (from all theirs) -- exact for those parameters, at a fraction of the cost."""
    from oracle import ptz_oracle as orc
    x_full = np.concatenate([np.asarray(ptz).reshape(-1), np.asarray(rays).reshape(-1)])
    out = []
    for kind, sel in (("frame", np.isin(p.frame, frames)), ("landmark", np.isin(p.landmark, landmarks))):
        fr = p.frame[sel].astype(np.int64)
        lm = p.landmark[sel].astype(np.int64)
        r = orc.compute_residual_records(x_full, p.n_pose, p.u, p.v, fr, lm, p.xy[sel]).reshape(-1, 2)
        if loss == "huber":
            r = r * np.where(r * r <= 1.0, 1.0, 1.0 / np.sqrt(np.maximum(r * r, 1.0)))
        J = orc.record_jacobian(p.u, p.v, np.asarray(ptz)[fr], np.asarray(rays)[lm])
        g = np.einsum("rkc,rk->rc", J, r)
        if kind == "frame":
            G = np.zeros((p.n_pose, 3))
            np.add.at(G, fr, g[:, :3])
            out.append(np.abs(G[frames]).max(0))
        else:
            G = np.zeros((p.n_landmark, 2))
            np.add.at(G, lm, g[:, 3:])
            out.append(np.abs(G[landmarks]).max(0))
    return np.concatenate(out)


@pytest.mark.timeout(900)
def test_config4_optimum_is_stationary_on_samples(gpu_available, config4):
    """Config 4's optimum in the headline arithmetic (fp32 records, matrix-core K2, Huber), pinned to the oracle
    the way config 3's is (test_gpu_config3.py): solved to a tight tolerance, the oracle's gradient of the reference
    cost is <= 1e-5 of its value at x0 for every parameter kind -- evaluated exactly on a sample (the poses of 12
    keyframes from every tilt row, from all their records, and the rays of 3000 landmarks, from all theirs),
    since the oracle's full 410M-record gradient would take minutes."""
    import ptzba
    p = config4
    rng = np.random.default_rng(11)
    frames = np.sort(rng.choice(np.arange(1, p.n_pose), 12, replace=False))
    landmarks = np.sort(rng.choice(p.n_landmark, 3000, replace=False))
    g0 = _sampled_gradient(p, p.init_ptz, p.init_rays, frames, landmarks)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-12, xtol=1e-14, max_iter=40).run()
    ptz, rays = h.get_state()
    h.close()
    g = _sampled_gradient(p, ptz, rays, frames, landmarks)
    ratio = g / g0
    print(f"config4 fp32-huber: {res}; sampled |g*|/|g0| (pan, tilt, f, theta, phi) {ratio}", flush=True)
    # DAMPING (5): at this tolerance the fp32 cost stops resolving a decrease before ftol does -- at a point whose
    # gradient is already ~1e-8 of x0's (measured), which is what this test gates
    assert res.status in (1, 2, 3, 5) and res.cost < res.initial_cost, res
    assert np.all(ratio <= 1e-5), ratio
