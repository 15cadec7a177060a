"""Host-side BA data preparation at a BASELINE config: the native correspondence builder
against the reference's Python bookkeeping on the same match graph (CPU only).

  python tools/bench_builder.py [--kf 500 --rays 20000]

Legs:
  native-cold   correspondence.build_graph (front-end hooks + native cap shuffle + ids), records,
                keyframe features/assembly
  native-cached the same with every detection / pair match served by a CorrespondenceCache
                (what the second and later keyframes of an incremental map pay)
  python-ref    the reference's algorithms for the same steps in the interpreter: random.shuffle cap
                (image_process.py:592-597), per-pair record loops (bundle_adjustment.py:67-99 order) and
                set() keyframe de-dup (:214-248); the front-end hook cost is the same and excluded."""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))

import numpy as np  # noqa: E402

import correspondence  # noqa: E402
import synthetic  # noqa: E402
from util import overlap_pan_angle  # noqa: E402


def native(g):
    t = time.time()
    g.records()
    off, loc, glo = g.keyframe_features()
    for i in range(g.n_frames):
        loc_i = loc[off[i]:off[i + 1]]
        list(map(g.keypoints[i].__getitem__, loc_i.tolist()))
        np.asarray(g.descriptors[i]).take(loc_i, axis=0)
    return time.time() - t


def python_ref(g, raw_lens):
    t0 = time.time()
    random.seed(0)
    for n in raw_lens:
        lst = list(range(int(n)))
        random.shuffle(lst)
        lst[:200]
    t_shuffle = time.time() - t0
    src, dst, lmk = g.lists()
    pts = g.points()
    t1 = time.time()
    n = g.n_frames
    rec = []
    for i in range(n):
        for j in range(n):
            for a, b, l in zip(src[i][j], dst[i][j], lmk[i][j]):
                rec.append((i, pts[i][a], l))
                rec.append((j, pts[j][b], l))
    t_rec = time.time() - t1
    t2 = time.time()
    for i in range(n):
        pairs = []
        for j in range(n):
            for a, l in zip(src[i][j], lmk[i][j]):
                pairs.append((a, l))
        for j in range(n):
            for b, l in zip(dst[j][i], lmk[j][i]):
                pairs.append((b, l))
        pairs = set(pairs)
        loc = [p[0] for p in pairs]
        [g.keypoints[i][k] for k in loc]
        np.asarray(g.descriptors[i]).take(loc, axis=0)
    t_kf = time.time() - t2
    return t_shuffle, t_rec, t_kf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kf", type=int, default=500)
    ap.add_argument("--rays", type=int, default=20000)
    ap.add_argument("--skip-python", action="store_true")
    a = ap.parse_args()
    sc = synthetic.make_scene(a.kf, a.rays, -60, 60, seed=0)
    fe = synthetic.SyntheticFrontEnd(sc).install()
    n, ip = len(sc.init_ptz), sc.init_ptz
    mask = [[1 if overlap_pan_angle(ip[i][2], ip[i][0], ip[j][2], ip[j][0], 1280) > 5 else 0 for j in range(n)]
            for i in range(n)]
    cache = correspondence.CorrespondenceCache()
    out = {"config": f"{a.kf}x{a.rays}"}
    for leg in ("native_cold", "native_cached"):
        random.seed(0)
        t = time.time()
        g = correspondence.build_graph(list(range(n)), mask, "sift", cache=cache, keys=list(range(n)))
        tg = time.time() - t
        tp = native(g)
        out[leg] = {"graph_s": round(tg, 3), "pack_s": round(tp, 3), "total_s": round(tg + tp, 3)}
    out["matches"] = int(g.n_matches)
    out["landmarks"] = int(g.n_landmark)
    raw_lens = [len(v[0]) for v in cache.matches.values() if len(v[0]) > 200]
    out["capped_pairs"] = len(raw_lens)
    if not a.skip_python:
        ts, tr, tk = python_ref(g, raw_lens)
        out["python_ref"] = {"shuffle_s": round(ts, 3), "records_s": round(tr, 3), "keyframes_s": round(tk, 3),
                             "total_s": round(ts + tr + tk, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
