"""Host model of the reduced-system plan (api.hip make_plan): tile pattern with symbolic fill, elimination
levels and back-substitution chain lengths for a given frame order.  Used to pick the nested-dissection
depth without a GPU.

  python tools/nd_model.py [config3]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "pan-tilt-zoom-slam_amd"))
import synthetic  # noqa: E402

NB = 32


def coupling_window(prob):
    """frame_win_hi[f]: the last frame coupled to f (a landmark seen by f is seen up to it)."""
    n = prob.n_pose
    fr, lm = prob.frame.astype(np.int64), prob.landmark.astype(np.int64)
    last = np.full(prob.n_landmark, -1, np.int64)
    np.maximum.at(last, lm, fr)
    win = np.arange(n, dtype=np.int64)
    np.maximum.at(win, fr, last[lm])
    return win


def pad(x):
    return (x + NB - 1) // NB * NB


def plan(pos, n_aug, win, nf, max_cols=2):
    T = n_aug // NB + 1
    nz = np.zeros((T, T), bool)
    n = len(win)
    for f1 in range(nf, n):
        for f2 in range(f1, min(n - 1, win[f1]) + 1):
            p1, p2 = pos[f1], pos[f2]
            for a in (p1, p1 + 2):
                for b in (p2, p2 + 2):
                    i, j = b // NB, a // NB
                    if i < j:
                        i, j = j, i
                    nz[i, j] = True
    ta = n_aug // NB
    nz[ta, : ta + 1] = True
    np.fill_diagonal(nz, True)
    for k in range(T):
        R = np.nonzero(nz[k + 1:, k])[0] + k + 1
        if len(R):
            sub = nz[np.ix_(R, R)]
            nz[np.ix_(R, R)] = sub | np.tril(np.ones_like(sub))
    level = np.zeros(T, int)
    count = []
    for k in range(T):
        L = 0
        for p in np.nonzero(nz[k, :k])[0]:
            L = max(L, level[p] + 1)
        while L < len(count) and count[L] >= max_cols:
            L += 1
        if L >= len(count):
            count += [0] * (L + 1 - len(count))
        count[L] += 1
        level[k] = L
    return nz, level, len(count)


def nested1(n, nf, win):
    pmax = np.maximum.accumulate(np.concatenate([[-1], win]))
    best = None
    for m in range(nf + 1, n):
        cend = max(m, pmax[m] + 1)
        if cend >= n:
            break
        ta, tb, tc = pad(3 * (m - nf)) // NB, pad(3 * (n - cend)) // NB, pad(3 * (cend - m)) // NB
        chain = max(ta, tb) + tc + 1
        if best is None or chain < best[0]:
            best = (chain, m, cend)
    return best


def order_from_parts(n, parts):
    """parts: list of frame lists in system order, each padded to whole tiles."""
    pos = np.full(n, -1, np.int64)
    row = 0
    for fl in parts:
        for k, f in enumerate(fl):
            pos[f] = row + 3 * k
        row += pad(3 * len(fl))
    return pos, row


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    prob = synthetic.make_problem(cfg)
    win = coupling_window(prob)
    n, nf = prob.n_pose, 1
    span = win - np.arange(n)
    print(f"{cfg}: n_pose {n}, coupling window mean {span.mean():.1f} max {span.max()}")
    pos, n_aug = order_from_parts(n, [list(range(nf, n))])
    _, _, L = plan(pos, n_aug, win, nf)
    print("natural: levels", L)
    chain, m, cend = nested1(n, nf, win)
    parts = [list(range(nf, m)), list(range(n - 1, cend - 1, -1)), list(range(m, cend))]
    pos, n_aug = order_from_parts(n, parts)
    _, _, L = plan(pos, n_aug, win, nf)
    print(f"nested-1: A [{nf},{m}) C [{m},{cend}) B [{cend},{n}) n_aug {n_aug} levels {L}")
    # two-level dissection: top separator in the middle, each half split again
    pmax = np.maximum.accumulate(np.concatenate([[-1], win]))

    def split(lo, hi):  # separator [m, cend) inside [lo, hi) minimising the longer side
        best = None
        for m in range(lo + 1, hi):
            cend = max(m, pmax[m] + 1)
            if cend >= hi:
                break
            d = max(m - lo, hi - cend)
            if best is None or d < best[0]:
                best = (d, m, cend)
        return best

    def balanced(lo, hi):  # (m1, c1) most balanced split of [lo, hi), running max of win from lo
        best, run = None, -1
        for m1 in range(lo + 1, hi):
            run = max(run, win[m1 - 1])
            c1 = max(m1, run + 1)
            if c1 >= hi:
                break
            d = abs((m1 - lo) - (hi - c1))
            if best is None or d < best[0]:
                best = (d, m1, c1)
        return None if best is None else best[1:]

    def tiles(a, b):
        return pad(3 * (b - a)) // NB

    best = None
    for m in range(nf + 2, n - 1):
        cend = max(m, pmax[m] + 1)
        if cend >= n - 1:
            break
        sl, sr = balanced(nf, m), balanced(cend, n)
        if sl is None or sr is None:
            continue
        (m1, c1), (m3, c3) = sl, sr
        est = max(max(tiles(nf, m1), tiles(c1, m)) + tiles(m1, c1),
                  max(tiles(cend, m3), tiles(c3, n)) + tiles(m3, c3)) + tiles(m, cend) + 1
        if best is None or est < best[0]:
            best = (est, m, cend, m1, c1, m3, c3)
    est, m, cend, m1, c1, m3, c3 = best
    parts = [list(range(nf, m1)), list(range(c1, m)), list(range(cend, m3)), list(range(n - 1, c3 - 1, -1)),
             list(range(m1, c1)), list(range(m3, c3)), list(range(m, cend))]
    pos, n_aug = order_from_parts(n, parts)
    nz, level, L = plan(pos, n_aug, win, nf, max_cols=4)
    print(f"nested-2 searched: estimate {est}, parts {[len(p) for p in parts]} n_aug {n_aug} levels {L}")
    for mc in (2, 4):
        _, m, cend = split(nf, n)
        left, right = (nf, m), (cend, n)
        sl, sr = split(*left), split(*right)
        if sl is None or sr is None:
            print("no two-level split")
            return
        _, m1, c1 = sl
        _, m3, c3 = sr
        parts = [list(range(nf, m1)), list(range(c1, m)), list(range(m1, c1)),
                 list(range(cend, m3)), list(range(c3, n)), list(range(m3, c3)), list(range(m, cend))]
        pos, n_aug = order_from_parts(n, parts)
        nz, level, L = plan(pos, n_aug, win, nf, max_cols=mc)
        sizes = [len(p) for p in parts]
        print(f"nested-2 (max {mc} cols/level): parts {sizes} n_aug {n_aug} levels {L}")


if __name__ == "__main__":
    main()
