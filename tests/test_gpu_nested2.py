"""GPU parity of the two-level nested-dissection order (api.hip nested_order2: A1 | C1 | A2 | C2 | A3 | C3 | A4,
four leaves factored side by side, four back-substitution chains over the separator tree) on a problem small
enough for the oracle's sparse solve: one undamped Gauss-Newton step equals the sparse normal-equation
solution of the reference residual (bundle_adjustment.py:25-106 via oracle/ptz_oracle.py) with every
back-substitution form and with delayed trailing updates (incl. 2 x 2 trailing blocks)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide():
    import synthetic
    # 200 keyframes over 200 deg of pan (every frame observed): a short coupling window, the solver picks two
    # dissection levels
    return synthetic.make_small_problem(200, 6000, -100.0, 100.0, seed=1)


@pytest.fixture(scope="module")
def sparse_step(wide):
    import scipy.sparse.linalg as spla
    from oracle import ptz_oracle as orc
    p = wide
    x0 = np.concatenate([p.init_ptz[1:].reshape(-1), p.init_rays.reshape(-1)])
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    J = orc.ba_jacobian(x0, p.n_pose, p.n_landmark, p.u, p.v, p.init_ptz[0], fr, lm).tocsc()
    r = orc.compute_residual_records(np.concatenate([p.init_ptz[0], x0]), p.n_pose, p.u, p.v, fr, lm, p.xy)
    return spla.spsolve((J.T @ J).tocsc(), -(J.T @ r))


@pytest.mark.parametrize("backsolve", ["lookahead", "ll", "blk"])
@pytest.mark.parametrize("delay", ["1", "2"])
def test_two_level_order_gauss_newton_step_is_exact(gpu_available, wide, sparse_step, monkeypatch, backsolve, delay):
    import ptzba
    p = wide
    monkeypatch.setenv("PTZBA_BACKSOLVE", {"lookahead": "la", "ll": "ll", "blk": "blk"}[backsolve])
    monkeypatch.setenv("PTZBA_CHOL_DELAY", delay)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
    info = h.solver_info()
    # (a delayed-update plan of this order needs more than four panels per task: the planner then takes DT = 1)
    assert info["nd_depth"] == 2 and info["ordering"] == "nested", info
    assert info["backsolve"] == {"lookahead": "lookahead", "ll": "left-looking", "blk": "blocked"}[backsolve]
    h.set_state(p.init_ptz, p.init_rays)
    h.linearize()
    h.build_reduced(0.0)
    h.solve_reduced()
    assert h.read_scalars()[5] == 0
    h.accept(True)
    ptz1, rays1 = h.get_state()
    h.close()
    dx_gpu = np.concatenate([(ptz1 - p.init_ptz)[1:].reshape(-1), (rays1 - p.init_rays).reshape(-1)])
    err = np.abs(dx_gpu - sparse_step).max() / np.abs(sparse_step).max()
    assert err < 1e-7, err


def test_two_level_order_lm_matches_one_level(gpu_available, wide, monkeypatch):
    """Device-driven LM under the two-level order and under the one-level order (PTZBA_ND_DEPTH=1): the same
    iterates (fp64, 4 iterations: poses within 1e-9 deg / 1e-7 px, same trial count, cost to 1e-12)."""
    import ptzba
    p = wide
    out = []
    for depth in ("2", "1"):
        monkeypatch.setenv("PTZBA_ND_DEPTH", depth)
        h = ptzba.BAHandle(0)
        h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP64)
        assert h.solver_info()["nd_depth"] == int(depth)
        h.set_state(p.init_ptz, p.init_rays)
        res = ptzba.LMSolver(h, ftol=1e-15, xtol=1e-15, max_iter=4, lambda0=1e-4).run()  # damped: see test_gpu_config3
        out.append((h.get_state()[0], res))
        h.close()
    (a, ra), (b, rb) = out
    assert ra.njev == rb.njev and ra.nfev == rb.nfev
    assert abs(ra.cost - rb.cost) <= 1e-12 * ra.cost
    np.testing.assert_allclose(a[:, :2], b[:, :2], rtol=0, atol=1e-9)
    np.testing.assert_allclose(a[:, 2], b[:, 2], rtol=0, atol=1e-7)
