"""Pin the CPU oracle (oracle/ptz_oracle.py) to the reference's own outputs.

Every fixture under tests/golden/ was produced by RUNNING the reference in the build container
(tests/golden/make_golden.py, SURVEY §8c recipe).  Integer bookkeeping is compared bit-exactly;
floating point within the stated tolerances (fp64 rounding only)."""
import random

import numpy as np
import pytest

from conftest import golden
from oracle import ptz_oracle as orc


def test_from_ray_to_image_kat():
    d = golden("kat_projection.npz")
    x, y = orc.from_ray_to_image(float(d["u"]), float(d["v"]), d["f"], d["cam_pan"], d["cam_tilt"], d["theta"], d["phi"])
    np.testing.assert_allclose(x, d["xy"][:, 0], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(y, d["xy"][:, 1], rtol=1e-12, atol=1e-9)


def test_closed_form_equals_q_form_with_abs_q2():
    """x = u + f q0/q2, y = v + f q1/|q2| (incl. rays behind the camera, q2 < 0)."""
    import synthetic
    d = golden("kat_projection.npz")
    x, y, q2 = synthetic._project(float(d["u"]), float(d["v"]), d["f"], d["cam_pan"], d["cam_tilt"], d["theta"], d["phi"])
    assert np.sum(q2 < 0) > 100  # the behind-camera subset is exercised
    np.testing.assert_allclose(x, d["xy"][:, 0], rtol=1e-10, atol=1e-7)
    np.testing.assert_allclose(y, d["xy"][:, 1], rtol=1e-10, atol=1e-7)


def test_from_image_to_ray_kat():
    d = golden("kat_projection.npz")
    th, ph = orc.from_image_to_ray(float(d["u"]), float(d["v"]), d["bp_f"], d["bp_pan"], d["bp_tilt"], d["bp_x"], d["bp_y"])
    np.testing.assert_allclose(th, d["bp_ray"][:, 0], rtol=0, atol=1e-10)
    np.testing.assert_allclose(ph, d["bp_ray"][:, 1], rtol=0, atol=1e-10)


def test_ptz_camera_kat():
    d = golden("kat_projection.npz")
    u, v = float(d["u"]), float(d["v"])
    for row in d["cam_rows"]:
        has_d, cp, ct, f, th, ph, px, py, ix, iy, bth, bph = row
        disp = d["displacement"] if has_d else None
        xy = orc.project_rays(u, v, f, cp, ct, [[th, ph]], disp)[0]
        assert abs(xy[0] - px) < 1e-8 and abs(xy[1] - py) < 1e-8
        r = orc.back_project_to_rays(u, v, f, cp, ct, [[ix, iy]], disp)[0]
        assert abs(r[0] - bth) < 1e-10 and abs(r[1] - bph) < 1e-10


def _lists_from_flat(n, mi, mj, k1, k2, lm):
    src = [[[] for _ in range(n)] for _ in range(n)]
    dst = [[[] for _ in range(n)] for _ in range(n)]
    lmk = [[[] for _ in range(n)] for _ in range(n)]
    for a, b, c, e, l in zip(mi, mj, k1, k2, lm):
        src[a][b].append(int(c))
        dst[a][b].append(int(e))
        lmk[a][b].append(int(l))
    return src, dst, lmk


def _points(d):
    off = d["points_off"]
    return [d["points"][off[i]:off[i + 1]] for i in range(len(off) - 1)]


@pytest.mark.parametrize("name", ["ba_4x60", "ba_6x120", "ba_10x200"])
def test_residual_vectors(name):
    d = golden(name + ".npz")
    n, m = int(d["n_pose"]), int(d["n_landmark"])
    src, dst, lmk = _lists_from_flat(n, d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"])
    pts = _points(d)
    for x, r_ref in zip(d["xs"], d["rs"]):
        r = orc.compute_residual(x, n, m, int(d["n_residual"]), pts, src, dst, lmk, float(d["u"]), float(d["v"]),
                                 d["ref_pose"])
        np.testing.assert_allclose(r, r_ref, rtol=0, atol=1e-9 * max(1.0, np.abs(r_ref).max() / 1e3))


@pytest.mark.parametrize("name", ["ba_4x60", "ba_6x120", "ba_10x200"])
def test_x0_init_last_writer_wins(name):
    d = golden(name + ".npz")
    n, m = int(d["n_pose"]), int(d["n_landmark"])
    x0 = orc.init_x0(d["init_ptz"], m, _points(d), d["m_i"], d["m_j"], d["m_k1"], d["m_lm"], float(d["u"]), float(d["v"]))
    np.testing.assert_allclose(x0[3:], d["x0"], rtol=0, atol=1e-10)


@pytest.mark.parametrize("name", ["ba_4x60", "ba_6x120", "ba_10x200"])
def test_keyframe_assembly_order(name):
    """set() de-dup order of (local, global) pairs decides feature order (bundle_adjustment.py:236-241)."""
    d = golden(name + ".npz")
    n = int(d["n_pose"])
    src, dst, lmk = _lists_from_flat(n, d["m_i"], d["m_j"], d["m_k1"], d["m_k2"], d["m_lm"])
    out = orc.assemble_keyframe_pairs(n, src, dst, lmk)
    off = d["kf_off"]
    for i, (loc, glb) in enumerate(out):
        np.testing.assert_array_equal(np.asarray(loc, np.int64), d["kf_local"][off[i]:off[i + 1]])
        np.testing.assert_array_equal(glb.astype(np.int64), d["kf_lmk"][off[i]:off[i + 1]])


def _graph_pairs_reference_order(d):
    """Replay build_matching_graph's pair loop on the recorded raw matches: i<j, mask, >20 rule,
    random.shuffle cap to 200 with the recorded global `random` seed (image_process.py:568-607)."""
    raw = {}
    off = 0
    for i, j, c in zip(d["raw_pi"], d["raw_pj"], d["raw_cnt"]):
        raw[(int(i), int(j))] = (list(d["raw_a"][off:off + c]), list(d["raw_b"][off:off + c]))
        off += c
    n = len(d["mask"])
    random.seed(int(d["seed"]))
    pairs = []
    for i in range(n):
        for j in range(i + 1, n):
            if d["mask"][i][j] == 0:
                continue
            a, b = raw[(i, j)]
            if len(a) > 20:
                if len(a) > 200:
                    rl = list(range(len(a)))
                    random.shuffle(rl)
                    rl = rl[:200]
                    a = [a[k] for k in rl]
                    b = [b[k] for k in rl]
                pairs.append((i, j, [int(x) for x in a], [int(x) for x in b]))
    return n, pairs


def test_matching_graph_bookkeeping_oracle():
    d = golden("matching_graph.npz")
    n, pairs = _graph_pairs_reference_order(d)
    src, dst, lmk, n_landmark, warn = orc.build_landmark_index(n, pairs)
    assert n_landmark == int(d["n_landmark"])
    assert warn > 0  # the fixture contains inconsistent matches
    mi, mj, k1, k2, lm = orc.flatten_matches(src, dst, lmk)
    for a, k in zip((mi, mj, k1, k2, lm), ("m_i", "m_j", "m_k1", "m_k2", "m_lm")):
        np.testing.assert_array_equal(a, d[k])


def test_h_jacobian_oracle():
    for name in ("ekf_R50.npz", "ekf_R300.npz"):
        d = golden(name)
        H = orc.compute_h_jacobian(float(d["u"]), float(d["v"]), float(d["pan0"]), float(d["tilt0"]), float(d["f0"]),
                                   d["H_rays"])
        np.testing.assert_allclose(H, d["H"], rtol=0, atol=1e-6)


def _ekf_state(d):
    R = len(d["rays0"])
    cov0 = np.diag(d["cov_base_diag"]).astype(np.float64)
    cov0[2, 2] = float(d["f_var"])
    cov0 = cov0 + d["cov_B"] @ d["cov_B"].T
    return dict(u=float(d["u"]), v=float(d["v"]), pan=float(d["pan0"]), tilt=float(d["tilt0"]), f=float(d["f0"]),
                displacement=None, rays=d["rays0"].copy(), state_cov=cov0), R


@pytest.mark.parametrize("name", ["ekf_R50.npz", "ekf_R300.npz"])
def test_ekf_update_oracle(name):
    d = golden(name)
    s, R = _ekf_state(d)
    out = orc.ekf_update(s, d["obs"], d["obs_idx"], int(d["height"]), int(d["width"]))
    assert abs(out["pan"] - float(d["pan1"])) < 1e-9
    assert abs(out["tilt"] - float(d["tilt1"])) < 1e-9
    assert abs(out["f"] - float(d["f1"])) < 1e-6
    np.testing.assert_allclose(out["velocity"], d["velocity"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(out["rays"], d["rays1"], rtol=0, atol=1e-9)
    cov = out["state_cov"]
    np.testing.assert_allclose(cov[:3, :3], d["cov1_pose"], rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(np.diag(cov), d["cov1_diag"], rtol=1e-7, atol=1e-12)
    pk = d["cov1_pick"]
    np.testing.assert_allclose(cov[pk[:, 0], pk[:, 1]], d["cov1_pick_val"], rtol=1e-6, atol=1e-12)
    assert int(np.sum(cov != _ekf_state(d)[0]["state_cov"])) == int(d["n_changed"])


def test_config2_reference_residual_sample():
    import synthetic
    d = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    assert len(p.frame) == int(d["n_records"]) and int(p.frame.sum()) == int(d["frame_sum"])
    r = orc.compute_residual_records(d["x0"], p.n_pose, p.u, p.v, p.frame.astype(np.int64), p.landmark.astype(np.int64),
                                     p.xy)
    np.testing.assert_allclose(r[d["r_ref_sample_idx"]], d["r_ref_sample"], rtol=0, atol=1e-9)
    assert abs(float(np.sum(r * r)) - float(d["r_ref_sumsq"])) <= 1e-10 * float(d["r_ref_sumsq"])


def test_config3_optimum_fixture():
    """Headline fixture (make_golden.py gen_config3): the records regenerate bit for bit, the oracle residual at x0
    equals a sample of the REFERENCE's own _compute_residual (bundle_adjustment.py:25-106, run on all 29.2M values
    when the fixture was made) and its sum of squares, and both stored optima are stationary points of the reference
    cost (max |gradient| per parameter kind <= 1e-7 of its value at x0) with the stored costs."""
    import synthetic
    d = golden("config3_optimum.npz")
    p = synthetic.make_problem("config3", seed=0)
    fr, lm = p.frame.astype(np.int64), p.landmark.astype(np.int64)
    assert len(fr) == int(d["n_records"]) and int(fr.sum()) == int(d["frame_sum"]) and int(lm.sum()) == int(d["landmark_sum"])
    x0 = np.concatenate([p.init_ptz.reshape(-1), p.init_rays.reshape(-1)])
    assert float(x0.sum()) == float(d["x0_sum"])
    idx = d["r_ref_sample_idx"]
    rec = np.unique(idx // 2)
    r = orc.compute_residual_records(x0, p.n_pose, p.u, p.v, fr[rec], lm[rec], p.xy[rec])
    r_all = np.full(2 * len(fr), np.nan)
    r_all[np.repeat(2 * rec, 2) + np.tile([0, 1], len(rec))] = r
    np.testing.assert_allclose(r_all[idx], d["r_ref_sample"], rtol=0, atol=1e-9)
    assert np.all(d["grad_tight"] <= 1e-7 * d["grad_x0"]), (d["grad_tight"], d["grad_x0"])
    assert np.all(d["grad_tight_huber"] <= 1e-7 * d["grad_x0_huber"]), (d["grad_tight_huber"], d["grad_x0_huber"])
    for key, loss in (("", "linear"), ("_huber", "huber")):
        c = orc.ba_cost_chunked(d["ptz_tight" + key], d["rays_tight" + key], p.u, p.v, fr, lm, p.xy, loss=loss)
        assert abs(c - float(d["tight_cost" + key])) <= 1e-12 * c


def test_schur_tight_solve_reproduces_config2_fixture():
    """The landmark-eliminating tight solver behind the config-3 fixture (orc.schur_tight_solve) reproduces the
    config-2 optimum that scipy trf + a sparse Gauss-Newton polish produced (config2_optimum.npz)."""
    import synthetic
    d = golden("config2_optimum.npz")
    p = synthetic.make_problem("config2", seed=0)
    ptz, rays, info = orc.schur_tight_solve(p.init_ptz, p.init_rays, p.u, p.v, p.frame, p.landmark, p.xy)
    xt = d["x_tight"]
    n = p.n_pose
    np.testing.assert_allclose(ptz[1:].reshape(-1), xt[:3 * (n - 1)], rtol=0, atol=1e-9)
    np.testing.assert_allclose(rays.reshape(-1), xt[3 * (n - 1):], rtol=0, atol=1e-9)
    assert abs(info["cost"] - float(d["tight_cost"])) <= 1e-10 * info["cost"]


def test_synthetic_generator_matches_reference_rules():
    """problem_from_pairs reproduces the first-seen landmark ids and last-writer ray init."""
    import synthetic
    scene = synthetic.make_scene(8, 300, 50, 60, seed=3)
    pairs = synthetic.scene_pairs(scene, seed=3)
    prob = synthetic.problem_from_pairs(scene, pairs)
    src, dst, lmk, n_landmark, warn = orc.build_landmark_index(len(scene.kp_xy), pairs)
    assert n_landmark == prob.n_landmark and warn == 0
    mi, mj, k1, k2, lm = orc.flatten_matches(src, dst, lmk)
    np.testing.assert_array_equal(lm, prob.landmark[0::2])
    x0 = orc.init_x0(scene.init_ptz, n_landmark, scene.kp_xy, mi, mj, k1, lm, scene.u, scene.v)
    np.testing.assert_allclose(x0[3 * len(scene.kp_xy):].reshape(-1, 2), prob.init_rays, rtol=0, atol=1e-10)
    frame, landmark, xy = orc.pair_records(scene.kp_xy, mi, mj, k1, k2, lm)
    np.testing.assert_array_equal(frame, prob.frame)
    np.testing.assert_allclose(xy, prob.xy)


def test_reloc_oracle_pinned_to_reference():
    """relocalization.py:22-40 restated: the reference's own least_squares optimum and cost."""
    d = golden("reloc.npz")
    u, v = float(d["u"]), float(d["v"])
    r = orc.reloc_residual(d["x_tight"], d["rays"], d["points"], u, v)
    assert abs(0.5 * float(r @ r) - float(d["cost_tight"])) <= 1e-9 * float(d["cost_tight"])
    x, c = orc.refine_pose(d["pose0"], d["rays"], d["points"], u, v, ftol=1e-15, xtol=1e-15, gtol=1e-15)
    assert np.all(np.abs(x - d["x_tight"]) <= [1e-9, 1e-9, 1e-7])
