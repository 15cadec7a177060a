"""
Correspondence -> packed-observation builder.

The reference builds the BA problem in Python loops and rebuilds it from scratch on every keyframe:
`Map.add_keyframe_with_ba` (scene_map.py:53-117) calls `bundle_adjustment`, which re-detects features
in every keyframe and re-matches every overlapping pair (bundle_adjustment.py:135-146 ->
image_process.build_matching_graph, image_process.py:509-667) before packing the residual
(bundle_adjustment.py:167-197) and the keyframes (:214-248).  At the headline size that host work is
about a minute against a ~40 ms GPU solve.

This module keeps the reference's outputs bit for bit and changes how they are produced:

  * `MatchGraph` holds the matching graph as flat CSR arrays (pairs in (i, j) order, matches
    concatenated) instead of N x N lists of lists; `lists()` gives the reference's view on demand.
  * The 200-match cap replays `random.shuffle` of the global `random` generator natively
    (ptzba.py_shuffle_prefix): same permutations, same generator state afterwards.  The shuffles are
    replayed after matching rather than interleaved with it, which is identical as long as the matcher
    hooks do not draw from the global `random` (OpenCV's matchers do not).
  * Landmark ids (first-seen rule), pair-form records with the x0 source record of each landmark, and
    the keyframes' set()-ordered feature lists are computed natively (libptzba builder.cpp).
  * `CorrespondenceCache` remembers detections per image and raw (pre-cap) matches per image pair, so
    an incremental map (`scene_map.Map`) or a sliding window (`RandomForestMap`) only detects the new
    image and matches the pairs it adds.  Detection and matching are deterministic in the reference
    (SIFT + brute-force ratio test), so cached results are the results a re-run would produce; the cap
    shuffle is still replayed for every capped pair, in the reference's order, keeping the global
    `random` stream and therefore every id identical to the reference's full rebuild.

The two interpreter-defined orderings (shuffle, set iteration) are checked against the running
interpreter once per process (`_self_check`); if they ever disagree the interpreter itself is used.
"""
import random

import time

import numpy as np

import image_process
import ptzba

MIN_MATCH_NUM = 20    # image_process.py:580: a pair is kept with MORE than this many matches
MAX_MATCH_NUM = 200   # image_process.py:581: longer match lists are shuffled and cut to this

_NATIVE_ORDER = None


def _self_check():
    """Native shuffle / set-order emulation == this interpreter (cheap; once per process)."""
    global _NATIVE_ORDER
    if _NATIVE_ORDER is None:
        ok = True
        r1, r2 = random.Random(20240917), random.Random(20240917)
        lens = [2, 3, 257, 1500]
        ref = []
        for n in lens:
            lst = list(range(n))
            r1.shuffle(lst)
            ref += lst[:MAX_MATCH_NUM]
        ok &= np.array_equal(ptzba.py_shuffle_prefix(lens, MAX_MATCH_NUM, r2), ref) and r1.random() == r2.random()
        rng = np.random.default_rng(7)
        a = rng.integers(0, 40000, 70000)
        b = rng.integers(0, 90000, 70000)
        oa, ob = ptzba.set_order_pairs(a, b)
        want = list(set(zip(a.tolist(), b.tolist())))
        ok &= len(want) == len(oa) and want == list(zip(oa.tolist(), ob.tolist()))
        _NATIVE_ORDER = bool(ok)
        if not ok:
            print("correspondence: native shuffle/set emulation differs from this interpreter; using Python")
    return _NATIVE_ORDER


def _shuffle_prefixes(lens):
    if _self_check():
        return ptzba.py_shuffle_prefix(lens, MAX_MATCH_NUM)
    out = []
    for n in lens:
        lst = list(range(int(n)))
        random.shuffle(lst)
        out += lst[:MAX_MATCH_NUM]
    return np.asarray(out, np.int64)


def _same_image(a, b):
    if a is b:
        return True
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return isinstance(a, np.ndarray) and isinstance(b, np.ndarray) and a.shape == b.shape and np.array_equal(a, b)
    try:
        return bool(a == b)
    except Exception:
        return False


class CorrespondenceCache:
    """Detections per image key and raw (pre-cap) matches per ordered key pair, reused across BA calls.
    Keys are the keyframes' image indices (KeyFrame.img_index); a key whose image changed is re-detected
    and its pairs re-matched."""

    _next_dev_id = 1  # device descriptor-set ids, unique per process (ptzba.desc_put keys)

    def __init__(self):
        self.detections = {}   # key -> (image, keypoints, descriptors, xy [K, 2])
        self.matches = {}      # (key_i, key_j, method) -> (idx1 int32, idx2 int32)
        self.dev = {}          # (key, method) -> (device descriptor-set id, rows): descriptors kept on the GPU
        self.n_detect = 0
        self.n_match = 0
        self.n_detect_hit = 0
        self.n_match_hit = 0

    def dev_set(self, key, feature_method, descriptors):
        """Id of this detection's descriptors uploaded to the device (once per detection) for the batched GPU
        matcher (ptzba.match_knn2_sets): a sliding window re-matches its new keyframe against every older one."""
        k = (key, feature_method)
        hit = self.dev.get(k)
        if hit is None:
            d = ptzba.desc_put_new(CorrespondenceCache._next_dev_id, descriptors)
            hit = (CorrespondenceCache._next_dev_id, d)
            CorrespondenceCache._next_dev_id += 1
            self.dev[k] = hit
        return hit

    def _drop_dev(self, keep):
        gone = [k for k in self.dev if not keep(k)]
        if gone:
            ids = [self.dev.pop(k)[0] for k in gone]
            try:
                ptzba.desc_drop(ids)
            except Exception:
                pass

    def __del__(self):
        try:
            self._drop_dev(lambda k: False)
        except Exception:
            pass

    def detect(self, key, image, feature_method):
        hit = self.detections.get((key, feature_method))
        if hit is not None and _same_image(hit[0], image):
            self.n_detect_hit += 1
            return hit[1:]
        if hit is not None:
            self.forget(key)
        kps, des = image_process._detect(image, feature_method)
        self.n_detect += 1
        xy = image_process.keypoint_xy(kps)
        self.detections[(key, feature_method)] = (image, kps, des, xy)
        return kps, des, xy

    def prepare(self, key, image, feature_method, device=0):
        """A map's first keyframe (no BA yet): its detection, which the first BA call would make, and the one-time
        costs of that call -- the interpreter self-check of the native bookkeeping and the shared BA handle
        (ptzba.warm_up) -- so no keyframe BA call carries process warm-up."""
        _self_check()
        self.detect(key, image, feature_method)
        ptzba.warm_up(device)

    def match(self, key_i, key_j, det_i, det_j, feature_method):
        k = (key_i, key_j, feature_method)
        hit = self.matches.get(k)
        if hit is not None:
            self.n_match_hit += 1
            return hit
        m = _match_raw(det_i, det_j, feature_method)
        self.n_match += 1
        self.matches[k] = m
        return m

    def peek(self, key_i, key_j, feature_method):
        return self.matches.get((key_i, key_j, feature_method))

    def store(self, key_i, key_j, feature_method, m):
        self.n_match += 1
        self.matches[(key_i, key_j, feature_method)] = m

    def forget(self, key):
        self.detections = {k: v for k, v in self.detections.items() if k[0] != key}
        self.matches = {k: v for k, v in self.matches.items() if k[0] != key and k[1] != key}
        self._drop_dev(lambda k: k[0] != key)

    def retain(self, keys):
        """Drop everything about images not in `keys` (sliding windows keep memory bounded)."""
        keep = set(keys)
        self.detections = {k: v for k, v in self.detections.items() if k[0] in keep}
        self.matches = {k: v for k, v in self.matches.items() if k[0] in keep and k[1] in keep}
        self._drop_dev(lambda k: k[0] in keep)


def _match_raw(det_i, det_j, feature_method):
    _, index1, _, index2 = image_process._match(det_i[0], det_i[1], det_j[0], det_j[1], feature_method)
    assert len(index1) == len(index2)
    return (np.asarray(index1, dtype=np.int32).reshape(-1), np.asarray(index2, dtype=np.int32).reshape(-1))


class MatchGraph:
    """The matching graph of image_process.build_matching_graph as flat arrays.

    pair_i/pair_j/pair_off: kept pairs in the reference's loop order (i < j) and their match ranges;
    k1/k2: matched keypoint indices (capped), lm: landmark id of each match; kp_off/kp_xy: keypoints."""

    def __init__(self, keypoints, descriptors, kp_xy_list, pair_i, pair_j, pair_off, k1, k2):
        self.n_frames = len(keypoints)
        self.keypoints = keypoints
        self.descriptors = descriptors
        self.kp_count = np.array([len(x) for x in kp_xy_list], np.int64)
        self.kp_off = np.concatenate([[0], np.cumsum(self.kp_count)]).astype(np.int64)
        self.kp_xy = np.concatenate(kp_xy_list).reshape(-1, 2) if kp_xy_list else np.zeros((0, 2))
        self.pair_i = np.asarray(pair_i, np.int32)
        self.pair_j = np.asarray(pair_j, np.int32)
        self.pair_off = np.asarray(pair_off, np.int64)
        self.k1 = np.asarray(k1, np.int64)
        self.k2 = np.asarray(k2, np.int64)
        cnt = np.diff(self.pair_off)
        self.m_i = np.repeat(self.pair_i, cnt)
        self.m_j = np.repeat(self.pair_j, cnt)
        self.lm, self.n_landmark, self.n_inconsistent = ptzba.build_landmarks_flat(
            self.kp_count, self.pair_i, self.pair_j, cnt, self.k1, self.k2)

    @property
    def n_matches(self):
        return len(self.k1)

    def points(self):
        return [self.kp_xy[self.kp_off[f]:self.kp_off[f + 1]] for f in range(self.n_frames)]

    def lists(self):
        """(src_pt_index, dst_pt_index, landmark_index) as the reference's N x N lists of int lists."""
        n = self.n_frames
        src = [[[] for _ in range(n)] for _ in range(n)]
        dst = [[[] for _ in range(n)] for _ in range(n)]
        lmk = [[[] for _ in range(n)] for _ in range(n)]
        for p in range(len(self.pair_i)):
            i, j = int(self.pair_i[p]), int(self.pair_j[p])
            a, b = self.pair_off[p], self.pair_off[p + 1]
            src[i][j] = self.k1[a:b].tolist()
            dst[i][j] = self.k2[a:b].tolist()
            lmk[i][j] = self.lm[a:b].tolist()
        return src, dst, lmk

    def records(self):
        """Pair-form records in _compute_residual order + x0 source record per landmark."""
        return ptzba.pack_records(self.n_frames, self.m_i, self.m_j, self.k1, self.k2, self.lm, self.kp_off,
                                  self.kp_xy, self.n_landmark)

    def keyframe_features(self):
        """CSR (off, local, global) of each keyframe's features in the reference's set() order."""
        if _self_check():
            return ptzba.keyframe_features(self.n_frames, self.m_i, self.m_j, self.k1, self.k2, self.lm)
        off, loc, glo = [0], [], []
        order = np.argsort(self.m_j, kind="stable")
        for f in range(self.n_frames):
            s = self.m_i == f
            d = order[self.m_j[order] == f]
            pairs = list(zip(self.k1[s].tolist(), self.lm[s].tolist())) + list(zip(self.k2[d].tolist(),
                                                                                  self.lm[d].tolist()))
            u = list(set(pairs))
            loc += [p[0] for p in u]
            glo += [p[1] for p in u]
            off.append(len(loc))
        return np.array(off, np.int64), np.array(loc, np.int64), np.array(glo, np.int64)


def build_graph(images, image_match_mask=(), feature_method="sift", verbose=False, cache=None, keys=None):
    """image_process.build_matching_graph (image_process.py:509-667) producing a MatchGraph.
    `cache` (CorrespondenceCache) + `keys` (one hashable id per image, e.g. KeyFrame.img_index) reuse
    detections and raw matches from earlier calls."""
    assert feature_method in ("sift", "orb", "latch")
    n = len(images)
    if len(image_match_mask) != 0:
        assert len(image_match_mask) == n
        for m in image_match_mask:
            assert len(m) == n
    elif verbose:
        print("Warning: image match mask is NOT used, may have false positive matches!")
    if cache is not None:
        if keys is None or len(keys) != n or len(set(keys)) != n:
            cache = None  # keys must identify the images uniquely
    t_det = time.perf_counter()
    dets = []
    for f, im in enumerate(images):
        if cache is not None:
            dets.append(cache.detect(keys[f], im, feature_method))
        else:
            kps, des = image_process._detect(im, feature_method)
            dets.append((kps, des, image_process.keypoint_xy(kps)))
    t_match = time.perf_counter()
    todo = [(i, j) for i in range(n) for j in range(i + 1, n)
            if not (len(image_match_mask) != 0 and image_match_mask[i][j] == 0)]
    # GPU SIFT matcher: every pair still to match in one batched call (kNN-2 per train image over the concatenated
    # queries, one RANSAC launch for all pairs) -- per pair exactly match_sift_features' result
    pre = {}
    if feature_method == "sift" and image_process.match_sift_features is image_process.GPU_MATCH_SIFT:
        if cache is None:
            need = todo
        else:
            peek = cache.matches.get
            need = [(i, j) for i, j in todo if peek((keys[i], keys[j], feature_method)) is None]
        if len(need) > 1:
            # (xy arrays: no .pt loops; with a cache the descriptors stay on the device across calls)
            dev = None if cache is None else [(cache.dev_set(keys[i], feature_method, dets[i][1]),
                                               cache.dev_set(keys[j], feature_method, dets[j][1])) for i, j in need]
            res = image_process.match_sift_features_batch(
                [(dets[i][2], dets[i][1], dets[j][2], dets[j][1]) for i, j in need], dev_sets=dev)
            for (i, j), (a, b) in zip(need, res):
                m = (np.asarray(a, dtype=np.int32).reshape(-1), np.asarray(b, dtype=np.int32).reshape(-1))
                pre[(i, j)] = m
                if cache is not None:
                    cache.store(keys[i], keys[j], feature_method, m)
    pi, pj, raw = [], [], []
    mget = cache.matches.get if cache is not None else None  # (the cache's hits read in place: ~435 pairs per call)
    hits = 0
    for ij in todo:
        m = pre.get(ij)
        if m is None:
            i, j = ij
            if cache is None:
                m = _match_raw(dets[i], dets[j], feature_method)
            else:
                m = mget((keys[i], keys[j], feature_method))
                if m is None:
                    m = cache.match(keys[i], keys[j], dets[i], dets[j], feature_method)
                else:
                    hits += 1
        if len(m[0]) > MIN_MATCH_NUM:
            pi.append(ij[0])
            pj.append(ij[1])
            raw.append(m)
        elif verbose:
            print("no enough matches between image: %d and %d" % ij)
    if cache is not None:
        cache.n_match_hit += hits
    t_cap = time.perf_counter()
    # 200-match cap: the reference's random.shuffle sequence, replayed in pair order; every pair's kept matches are
    # gathered in one indexing pass over the concatenated raw lists (uncapped pairs whole, capped pairs at their
    # shuffled prefix positions)
    raw_len = np.array([len(a) for a, _ in raw], np.int64)
    cnt = np.minimum(raw_len, MAX_MATCH_NUM)
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
    if raw:
        raw_off = np.concatenate([[0], np.cumsum(raw_len)[:-1]]).astype(np.int64)
        pos = np.arange(off[-1], dtype=np.int64) - np.repeat(off[:-1], cnt)  # position within the pair
        capped = raw_len > MAX_MATCH_NUM
        if capped.any():
            pos[np.repeat(capped, cnt)] = _shuffle_prefixes(raw_len[capped])
        src = np.repeat(raw_off, cnt) + pos
        k1 = np.concatenate([a for a, _ in raw])[src]
        k2 = np.concatenate([b for _, b in raw])[src]
    else:
        k1 = k2 = np.zeros(0, np.int64)
    if verbose:
        for p in range(len(pi)):
            print("%d matches between image: %d and %d" % (cnt[p], pi[p], pj[p]))
    g = MatchGraph([d[0] for d in dets], [d[1] for d in dets], [d[2] for d in dets], pi, pj, off, k1, k2)
    g.timing = {"detect_s": t_match - t_det, "match_s": t_cap - t_match, "cap_graph_s": time.perf_counter() - t_cap}
    if g.n_inconsistent and verbose:
        print("Warning: %d in-consistent matching results" % g.n_inconsistent)
    if verbose:
        print("number of landmark is %d" % g.n_landmark)
    return g
