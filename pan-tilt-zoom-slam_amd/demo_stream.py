"""
Streaming PTZ SLAM driver (BASELINE configs[4]): the demo_soccer.py loop (demo_soccer.py:17-55) on a
synthetic 1080p court stream -- per frame `PtzSlam.tracking` (LK flow + homography RANSAC stand-in, EKF
update on the GPU, ray removal / addition), `relocalize` + `init_system` when tracking is lost, and
`add_keyframe` (keyframe bundle adjustment on the GPU) when the map asks for a new keyframe.

The keyframe map is the reference's `Map` (every keyframe adjusted, scene_map.py:53-117) or, with
--window N, a sliding window over the last N keyframes (the rule of RandomForestMap.bundle_adjustment_
processing, scene_map.py:198-244, with the window the config asks for: 30).  --keyframe-every K adds a
keyframe every K frames on top of the reference's overlap rule (ptz_slam.py:458), so long windows fill up.

  python demo_stream.py [--frames 300] [--window 30] [--keyframe-every 10] [--json]

Prints one JSON line: end-to-end frames/s, per-frame tracking latency, keyframe BA latency, pose error
against the ground truth, and the time spent inside the front-end stand-in (synthetic.StreamFrontEnd:
not part of the SLAM path; the fps without it is reported too).
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def run_stream(slam, scene, n_frames, camera0, keyframe_every=None, on_frame=None):
    """The demo_soccer.py:17-55 loop over frames 0..n_frames-1 of `scene` with an initialised `slam`
    object (this build's PtzSlam or the reference's).  Returns per-frame records and timings."""
    img = scene.image(0)
    slam.init_system(img, camera0)
    slam.add_keyframe(img, camera0, 0, enable_rf=False)
    rec = dict(ptz=[list(camera0.get_ptz())], velocity=[[0.0, 0.0, 0.0]], n_rays=[len(slam.rays)],
               n_kp=[len(slam.previous_keypoints)], keyframe=[1], lost=[0], t_track=[0.0], t_kf=[0.0])
    for i in range(1, n_frames):
        img = scene.image(i)
        t0 = time.perf_counter()
        slam.tracking(next_img=img, bad_tracking_percentage=80)
        t1 = time.perf_counter()
        added = lost = 0
        if slam.tracking_lost:
            cam = slam.relocalize(img, slam.current_camera, enable_rf=False)
            slam.init_system(img, cam)
            lost = 1
        elif slam.new_keyframe or (keyframe_every and i % keyframe_every == 0):
            slam.add_keyframe(img, slam.current_camera, i, enable_rf=False)
            slam.new_keyframe = False
            added = 1
            lr = sys.modules.get("bundle_adjustment")
            if lr is not None and getattr(lr, "LAST_RESULT", None):
                rec.setdefault("kf_timing", []).append(dict(lr.LAST_RESULT.get("timing", {})))
                res = lr.LAST_RESULT.get("result")
                rec.setdefault("kf_lm", []).append(
                    (int(getattr(res, "njev", 0)), int(getattr(res, "nfev", 0)), int(getattr(res, "status", 0)),
                     int(lr.LAST_RESULT.get("n_residual", 0))))
        t2 = time.perf_counter()
        cam = slam.cameras[i] if i < len(slam.cameras) else slam.current_camera
        rec["ptz"].append([cam.pan, cam.tilt, cam.focal_length])
        rec["velocity"].append([float(x) for x in np.asarray(slam.velocity).reshape(-1)[:3]])
        rec["n_rays"].append(len(slam.rays))
        rec["n_kp"].append(len(slam.previous_keypoints))
        rec["keyframe"].append(added)
        rec["lost"].append(lost)
        rec["t_track"].append(t1 - t0)
        rec["t_kf"].append(t2 - t1)
        if on_frame:
            on_frame(i, slam)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--window", type=int, default=30, help="keyframes per sliding-window BA (0: all, as Map)")
    ap.add_argument("--keyframe-every", type=int, default=5)
    ap.add_argument("--pan-range", type=float, default=40.0)
    ap.add_argument("--frontend", choices=("gpu", "standin"), default="gpu",
                    help="gpu: rendered 1080p frames through the GPU front-end (SIFT, LK, RANSAC); "
                         "standin: StreamFrontEnd's ground-truth correspondences")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--gc", choices=("default", "freeze", "scheduled"), default="scheduled",
                    help="freeze: gc.freeze() before the loop -- the ~10^5 objects of the imports (torch, scipy) leave the "
                         "cyclic collector's generations, so its full collections in the loop take ~4 ms instead of "
                         "14-19 ms (profiles/r05j_*); scheduled (default): freeze, and the full (generation-2) "
                         "collections run between frames every --gc-every frames instead of wherever the allocation "
                         "counters trip them -- with freeze alone one lands inside keyframe 51's detection in every run "
                         "(r05j / BENCH_r05: detect 4.7-9.8 ms against ~1 ms); their time stays in the end-to-end wall; "
                         "default: Python's own setting")
    ap.add_argument("--gc-every", type=int, default=100,
                    help="scheduled: frames between the full collections (freeze alone ran ~3 per 300 frames)")
    ap.add_argument("--setup-front", type=int, default=None,
                    help="records from which the keyframe BA's set_problem builds on the device (ptzba.SETUP_FRONT_MIN; "
                         "default: the library's 64K, i.e. the device front for a window's ~170K records; 4194304 restores round 5)")
    a = ap.parse_args()
    import gc
    gc_stats = {}  # generation -> [collections, total ms, max ms] during the loop (Python's cyclic collector)
    gc_t = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t[0] = time.perf_counter()
        else:
            dt = 1e3 * (time.perf_counter() - gc_t[0])
            st = gc_stats.setdefault(info["generation"], [0, 0.0, 0.0])
            st[0] += 1
            st[1] += dt
            st[2] = max(st[2], dt)
    import ptzba
    import synthetic
    from ptz_slam import PtzSlam
    if a.setup_front is not None:
        ptzba.SETUP_FRONT_MIN = a.setup_front
    from scene_map import Map
    scene = synthetic.StreamScene(a.frames, seed=a.seed, pan_lo=-a.pan_range / 2, pan_hi=a.pan_range / 2)
    t_render = 0.0
    if a.frontend == "standin":
        fe = synthetic.StreamFrontEnd(scene).install()
        source = scene
    else:
        fe = None
        t0 = time.perf_counter()
        source = synthetic.RenderedStream(scene, seed=a.seed)
        for i in range(a.frames):  # frames are decoded before the loop (the reference reads them from disk)
            source.image(i)
        t_render = time.perf_counter() - t0
    slam = PtzSlam()
    slam.keyframe_map = Map("sift", max_ba_frame=a.window or None)
    on_frame = None
    gc_thresholds = gc.get_threshold()
    if a.gc in ("freeze", "scheduled"):
        gc.collect()
        gc.freeze()
    if a.gc == "scheduled":
        # generations 0 / 1 stay automatic (sub-ms); generation 2 only where on_frame runs it: between frames, after the
        # frame's tracking / keyframe timers, inside the end-to-end wall clock
        gc.set_threshold(gc_thresholds[0], gc_thresholds[1], 1 << 30)

        def on_frame(i, _slam):
            if i % max(1, a.gc_every) == 0:
                gc.collect(2)
    gc.callbacks.append(_gc_cb)
    quiet = contextlib.nullcontext() if a.verbose else contextlib.redirect_stdout(io.StringIO())
    t0 = time.perf_counter()
    with quiet:
        rec = run_stream(slam, source, a.frames, scene.camera(0), keyframe_every=a.keyframe_every, on_frame=on_frame)
    wall = time.perf_counter() - t0
    gc.callbacks.remove(_gc_cb)
    gc.set_threshold(*gc_thresholds)
    est = np.asarray(rec["ptz"])
    err = est - scene.cams[:len(est)]
    tt = np.asarray(rec["t_track"][1:])
    tk = np.asarray([t for t, k in zip(rec["t_kf"], rec["keyframe"]) if k][1:] or [0.0])
    fe_time = fe.time if fe else 0.0
    out = {
        "workload": f"config5: streaming PTZ tracking, {a.frames} frames 1920x1080, keyframe BA window "
                    f"{a.window or 'all'}, keyframe every {a.keyframe_every} frames + overlap rule",
        "frontend": ("GPU SIFT / pyramidal LK / homography RANSAC on rendered frames" if fe is None else
                     "stand-in: ground-truth correspondences (synthetic.StreamFrontEnd)"),
        "frames": a.frames, "fps_end_to_end": a.frames / wall, "wall_s": wall, "render_s_outside_loop": t_render,
        "frontend_standin_s": fe_time, "fps_excluding_frontend_standin": a.frames / max(wall - fe_time, 1e-9),
        "tracking_ms": {"mean": 1e3 * float(tt.mean()), "p50": 1e3 * float(np.median(tt)),
                        "p99": 1e3 * float(np.percentile(tt, 99))},
        "keyframes": int(sum(rec["keyframe"])), "keyframe_ba_ms": {"mean": 1e3 * float(tk.mean()),
                                                                  "p50": 1e3 * float(np.median(tk)),
                                                                  "max": 1e3 * float(tk.max()),
                                                                  "argmax_keyframe": int(np.argmax(tk)) + 1},
        "final_keyframes_in_map": len(slam.keyframe_map.keyframe_list), "rays_final": rec["n_rays"][-1],
        "lost_frames": int(sum(rec["lost"])),
        "pose_rmse_vs_truth": {"pan_deg": float(np.sqrt(np.mean(err[:, 0] ** 2))),
                               "tilt_deg": float(np.sqrt(np.mean(err[:, 1] ** 2))),
                               "f_px": float(np.sqrt(np.mean(err[:, 2] ** 2)))},
        "device": ptzba.lib().ptzba_version().decode(),
        "gc": a.gc + (f" (full collections every {a.gc_every} frames, between frames)" if a.gc == "scheduled" else ""),
        "gc_pauses_ms": {str(g): {"count": v[0], "total": v[1], "max": v[2]} for g, v in sorted(gc_stats.items())},
    }
    kt = rec.get("kf_timing", [])[1:]
    if kt:  # where a keyframe's BA call spends its time (bundle_adjustment.LAST_RESULT["timing"], mean ms)
        keys = sorted({k for d in kt for k in d})
        out["keyframe_ba_breakdown_ms"] = {k: 1e3 * float(np.mean([d.get(k, 0.0) for d in kt])) for k in keys}
        kall = rec.get("kf_timing", [])  # one per in-loop keyframe, as tk
        if len(kall) == len(tk):  # the slowest keyframe call's own breakdown
            out["keyframe_ba_slowest_breakdown_ms"] = {k: 1e3 * float(kall[int(np.argmax(tk))].get(k, 0.0)) for k in keys}
    lm = rec.get("kf_lm", [])
    if lm and len(lm) == len(tk):  # the LM of each keyframe call: iterations (njev), evaluations (nfev), status
        a_lm = np.asarray(lm)
        out["keyframe_lm"] = {"njev_mean": float(a_lm[:, 0].mean()), "njev_max": int(a_lm[:, 0].max()),
                              "nfev_mean": float(a_lm[:, 1].mean()), "nfev_max": int(a_lm[:, 1].max()),
                              "slowest": {"njev": int(a_lm[int(np.argmax(tk)), 0]), "nfev": int(a_lm[int(np.argmax(tk)), 1]),
                                          "status": int(a_lm[int(np.argmax(tk)), 2]),
                                          "residuals": int(a_lm[int(np.argmax(tk)), 3])},
                              "per_keyframe": [list(map(int, r)) for r in lm]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
