#!/usr/bin/env python3
"""Where does the LM stop at the reference's termination (ftol=1e-4, bundle_adjustment.py:200-202), per damping
schedule?  For config 3 (fp32 + Huber, fp64 + linear) and config 2, each lambda0 in the list: iterations, trials,
cost above the pinned optimum and pan / tilt / f RMSE against it (tests/golden/config{2,3}_optimum.npz), plus the
shipped ftol=1e-4 results of the reference (x_ls in tests/golden/ba_*.npz).  Measurement tool, not a test."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import ptzba  # noqa: E402
import synthetic  # noqa: E402

LAMS = [float(x) for x in os.environ.get("LAMS", "1e-4,1e-6,1e-8,1e-12").split(",")]


def rmse_rays(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


def study_config(cfg, precision, loss):
    p = synthetic.make_problem(cfg, seed=0)
    z = np.load(os.path.join(ROOT, "tests", "golden", f"{cfg}_optimum.npz"))
    key = "_huber" if loss == ptzba.LOSS_HUBER else ""
    if cfg == "config3":
        pt, rt, ct = z["ptz_tight" + key], z["rays_tight" + key], float(z["tight_cost" + key])
    else:
        xt = z["x_tight" + key]
        pt = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
        rt = xt[3 * (p.n_pose - 1):].reshape(-1, 2)
        ct = float(z["tight_cost" + key])
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=precision, loss=loss,
                  f_scale=1.0)
    out = []
    for lam in LAMS:
        h.set_state(p.init_ptz, p.init_rays)
        r = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100, lambda0=lam, device_loop=False).run()
        ptz, rays = h.get_state()
        row = dict(hcurv=os.environ.get("PTZBA_HUBER_CURV", "1"), config=cfg, precision="fp32" if precision == ptzba.FP32 else "fp64",
                   loss="huber" if key else "linear", lambda0=lam, njev=r.njev, nfev=r.nfev, status=r.status,
                   cost_rel=(r.cost - ct) / ct, rmse=[float(x) for x in synthetic.pose_rmse(ptz, pt)],
                   rays_rmse=rmse_rays(rays, rt),
                   history=[(int(i), float(c), float(l), int(t)) for i, c, l, t in r.history])
        print(json.dumps(row), flush=True)
        out.append(row)
    h.close()
    return out


def study_fixture(name):
    from test_gpu_ba import _problem_from_golden
    d = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    n, m, frame, landmark, xy, u, v = _problem_from_golden(d)
    x0 = np.concatenate([d["ref_pose"], d["x0"]])
    for lam in LAMS:
        ptz, rays, res = ptzba.solve(n, m, frame, landmark, xy, u, v, x0[:3 * n].reshape(n, 3), x0[3 * n:].reshape(m, 2),
                                     precision=ptzba.FP64, ftol=1e-4, xtol=1e-8, max_iter=100, lambda0=lam)
        x = np.concatenate([ptz.reshape(-1)[3:], rays.reshape(-1)])
        dl = np.abs(x - d["x_ls"])
        dt = np.abs(x - d["x_tight"])
        print(json.dumps(dict(fixture=name, lambda0=lam, njev=res.njev, ref_njev=int(d["ls_njev"]),
                              cost=res.cost, ref_cost=float(d["ls_cost"]),
                              max_vs_x_ls_angle=float(np.concatenate([dl[:3 * (n - 1)].reshape(-1, 3)[:, :2].ravel(), dl[3 * (n - 1):]]).max()),
                              max_vs_x_ls_f=float(dl[:3 * (n - 1)].reshape(-1, 3)[:, 2].max()),
                              max_vs_tight_angle=float(np.concatenate([dt[:3 * (n - 1)].reshape(-1, 3)[:, :2].ravel(), dt[3 * (n - 1):]]).max()),
                              max_vs_tight_f=float(dt[:3 * (n - 1)].reshape(-1, 3)[:, 2].max()))), flush=True)


if __name__ == "__main__" and not {"switch", "defaults"} & set(sys.argv[1:]):
    which = sys.argv[1:] or ["fixtures", "config2", "config3"]
    if "fixtures" in which:
        for nm in ("ba_6x120", "ba_10x200"):
            study_fixture(nm)
    lin = "huber-only" not in which
    if "config2" in which:
        if lin:
            study_config("config2", ptzba.FP64, ptzba.LOSS_LINEAR)
        study_config("config2", ptzba.FP32, ptzba.LOSS_HUBER)
    if "config3" in which:
        study_config("config3", ptzba.FP32, ptzba.LOSS_HUBER)
        if lin:
            study_config("config3", ptzba.FP64, ptzba.LOSS_LINEAR)


def host_lm_switch(h, ftol, xtol, lam0, switch_after, hc_new, relin, max_iter=100, min_lambda=1e-12):
    """ptzba.LMSolver._run_host's rules with a curvature switch: after accepted iteration `switch_after` later
    linearisations use hc_new (relin: re-linearise the current point at once)."""
    h.set_huber_curvature(1.0)
    h.linearize()
    s = h.read_scalars()
    cost = s[0]
    lam, nu, it, status, hist = lam0, 2.0, 0, 0, []
    while it < max_iter:
        accepted, retries = False, 0
        while not accepted and retries < 30:
            h.build_reduced(lam)
            h.solve_reduced()
            s = h.read_scalars()
            new_cost, pred, dx2, x2, info = s[1], s[2], s[3], s[4], s[5]
            ok = info == 0 and np.isfinite(new_cost) and np.isfinite(pred)
            actual = cost - new_cost
            rho = actual / pred if (ok and pred > 0) else -1.0
            if ok and rho > 0:
                accepted = True
                h.accept(True)
                lam = max(min_lambda, lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3))
            else:
                h.accept(False)
                lam = max(lam * nu, 1e-9)
                nu *= 2.0
                retries += 1
        if not accepted:
            status = -1
            break
        it += 1
        old, cost = cost, new_cost
        hist.append((it, float(cost), float(rho), retries))
        if it == switch_after:
            h.set_huber_curvature(max(hc_new, 1e-9))
            if relin:
                h.linearize()
        if actual < ftol * old and rho > 0.25:
            status = 2
            break
        if np.sqrt(dx2) < xtol * (xtol + np.sqrt(x2)):
            status = 3
            break
    h.set_huber_curvature(1.0)
    return it, status, cost, hist


def study_switch(cfg):
    p = synthetic.make_problem(cfg, seed=0)
    z = np.load(os.path.join(ROOT, "tests", "golden", f"{cfg}_optimum.npz"))
    if cfg == "config3":
        pt, rt, ct = z["ptz_tight_huber"], z["rays_tight_huber"], float(z["tight_cost_huber"])
    else:
        xt = z["x_tight_huber"]
        pt = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
        rt = xt[3 * (p.n_pose - 1):].reshape(-1, 2)
        ct = float(z["tight_cost_huber"])
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    for sw in (1, 2, 100):
        for hc in ((0.1, 0.01, 0.0) if sw < 100 else (1.0,)):
            for relin in ((0, 1) if sw < 100 else (0,)):
                h.set_state(p.init_ptz, p.init_rays)
                it, st, cost, hist = host_lm_switch(h, 1e-4, 1e-8, 1e-12, sw, hc, relin)
                ptz, rays = h.get_state()
                print(json.dumps(dict(config=cfg, switch_after=sw, hc=hc, relin=relin, njev=it, status=st,
                                      cost_rel=(cost - ct) / ct, rmse=[float(x) for x in synthetic.pose_rmse(ptz, pt)],
                                      rays_rmse=rmse_rays(rays, rt), history=hist)), flush=True)
    h.close()


if __name__ == "__main__" and "switch" in sys.argv[1:]:
    for c in ("config2", "config3"):
        study_switch(c)


def study_defaults():
    """The shipped defaults (ptzba.LAMBDA0 / HUBER_CURVATURE / CURVATURE_SWITCH) through both LM loops."""
    for cfg in ("config2", "config3"):
        p = synthetic.make_problem(cfg, seed=0)
        z = np.load(os.path.join(ROOT, "tests", "golden", f"{cfg}_optimum.npz"))
        for prec, loss in ((ptzba.FP32, ptzba.LOSS_HUBER), (ptzba.FP64, ptzba.LOSS_LINEAR), (ptzba.FP64, ptzba.LOSS_HUBER)):
            key = "_huber" if loss == ptzba.LOSS_HUBER else ""
            if cfg == "config3":
                pt, rt, ct = z["ptz_tight" + key], z["rays_tight" + key], float(z["tight_cost" + key])
            else:
                xt = z["x_tight" + key]
                pt = np.concatenate([p.init_ptz[0], xt[:3 * (p.n_pose - 1)]]).reshape(-1, 3)
                rt = xt[3 * (p.n_pose - 1):].reshape(-1, 2)
                ct = float(z["tight_cost" + key])
            h = ptzba.BAHandle(0)
            h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=prec, loss=loss)
            for dl in (True, False):
                h.set_state(p.init_ptz, p.init_rays)
                r = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100, device_loop=dl).run()
                ptz, rays = h.get_state()
                print(json.dumps(dict(config=cfg, precision=int(prec), loss=int(loss), device_loop=dl, njev=r.njev,
                                      nfev=r.nfev, status=r.status, cost_rel=(r.cost - ct) / ct,
                                      rmse=[float(x) for x in synthetic.pose_rmse(ptz, pt)],
                                      rays_rmse=rmse_rays(rays, rt))), flush=True)
            h.close()


if __name__ == "__main__" and "defaults" in sys.argv[1:]:
    study_defaults()
    for nm in ("ba_6x120", "ba_10x200"):
        LAMS[:] = [ptzba.LAMBDA0]
        study_fixture(nm)
