#!/usr/bin/env python3
"""Host-side cost of one sliding-window keyframe BA call (config 5) without a GPU: a 30-keyframe window whose
detections and raw matches are already cached (the steady state of scene_map's window), so build_graph's
bookkeeping, the cap replay, landmark ids, record packing and keyframe assembly are what is timed -- the parts of
keyframe_ba_breakdown_ms that are not GPU work.

  python tools/keyframe_host_bench.py [--frames 30] [--kp 1500] [--matches 260] [--reps 20]
"""
import argparse
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pan-tilt-zoom-slam_amd"))

import bundle_adjustment  # noqa: E402
import correspondence  # noqa: E402
import image_process  # noqa: E402
import ptzba  # noqa: E402
from key_frame import KeyFrame  # noqa: E402


class KP:
    __slots__ = ("pt",)

    def __init__(self, x, y):
        self.pt = (x, y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--kp", type=int, default=1500)
    ap.add_argument("--matches", type=int, default=260)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    n = a.frames
    dets = {}
    for f in range(n + a.reps):
        xy = rng.uniform(0, 1080, (a.kp, 2))
        dets[f] = ([KP(float(x), float(y)) for x, y in xy], rng.integers(0, 255, (a.kp, 128)).astype(np.float32), xy)
    raw = {}

    def fake_detect(im, method):
        return dets[int(im[0])][:2]

    def fake_match(kp1, des1, kp2, des2, method):
        key = (id(kp1), id(kp2))
        if key not in raw:
            m = int(rng.integers(a.matches // 2, 2 * a.matches))
            raw[key] = (rng.choice(a.kp, m, replace=False).tolist(), None, rng.choice(a.kp, m, replace=False).tolist(), None)
        r = raw[key]
        return None, r[0], None, r[2]

    image_process._detect = fake_detect
    image_process._match = fake_match
    image_process.match_sift_features = None  # (not the GPU batch matcher: cached raw matches)
    cache = correspondence.CorrespondenceCache()
    images = {f: np.array([f]) for f in dets}
    random.seed(1)
    tt = {}

    def tick(k, t0):
        tt.setdefault(k, []).append(time.perf_counter() - t0)
        return time.perf_counter()

    for rep in range(a.reps + 1):
        keys = list(range(rep, rep + n))
        cache.retain(keys)
        mask = [[1] * n for _ in range(n)]
        # warm the cache for every pair of the window but the newest keyframe's (they are matched per call)
        t0 = time.perf_counter()
        g = correspondence.build_graph([images[k] for k in keys], mask, "sift", cache=cache, keys=keys)
        t0 = tick("build_graph", t0)
        fr, lm, xy, src = g.records()
        t0 = tick("records", t0)
        lists = bundle_adjustment._KeyframeLists(g)
        kfs = []
        for i in range(n):
            kf = KeyFrame(images[keys[i]], keys[i], np.zeros(3), np.eye(3), 640, 360, 0.0, 0.0, 1000.0)
            kf.set_features_lazy(g.keypoints[i], g.descriptors[i], lists, i)
            kfs.append(kf)
        t0 = tick("keyframes", t0)
        kfs[-1].landmark_index
        t0 = tick("keyframe_lists (on first use)", t0)
        for k, v in g.timing.items():
            tt.setdefault(k, []).append(v)
        if rep == 0:
            tt.clear()
    print("window %d frames, %d pairs, %d matches, %d landmarks, %d records" %
          (n, len(g.pair_i), g.n_matches, g.n_landmark, len(fr)))
    for k, v in tt.items():
        print("%-30s %7.3f ms (min %.3f)" % (k, 1e3 * float(np.median(v)), 1e3 * float(np.min(v))))


if __name__ == "__main__":
    main()
