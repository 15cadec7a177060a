"""The factorisation plans libptzba builds (ptzba_plan_export, host only), replayed task by task on the CPU
(tests/chol_plan_exec.py restates k_chol_step's tile tasks in numpy) on an SPD matrix with the reduced camera
system's coupling structure, must reproduce numpy's Cholesky factor: the one- and two-level nested orders, the
delayed trailing updates and their 2 x 2 trailing blocks.  Plan logic only: the device arithmetic is checked by
the GPU tests (test_gpu_nested2.py, test_gpu_config4.py)."""
import os

import numpy as np
import pytest

from conftest import ROOT

import chol_plan_exec as cpe
import ptzba


def band_window(n, w):
    return np.minimum(np.arange(n) + w, n - 1).astype(np.int32)


CASES = {
    "config3": lambda: np.load(os.path.join(ROOT, "tests", "golden", "config3_window.npy")),
    "band300": lambda: band_window(300, 24),
}


@pytest.mark.parametrize("env", [{}, {"PTZBA_ND_DEPTH": "1"}, {"PTZBA_CHOL_DELAY": "2"},
                                 {"PTZBA_CHOL_DELAY": "2", "PTZBA_CHOL_BLOCKS": "0"},
                                 {"PTZBA_CHOL_DELAY": "2", "PTZBA_ND_DEPTH": "1"}])
@pytest.mark.parametrize("case", sorted(CASES))
def test_plan_replays_to_the_cholesky_factor(monkeypatch, case, env):
    for k in ("PTZBA_ND_DEPTH", "PTZBA_CHOL_DELAY", "PTZBA_CHOL_BLOCKS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    win = CASES[case]()
    pos, tasks, off, n_aug, _ = ptzba.plan_export(win, 1)
    ld = (n_aug + 1 + 31) // 32 * 32
    S = cpe.test_matrix(pos, win, n_aug, ld)
    Lf, _ = cpe.replay(S, tasks, off)
    Lref = np.linalg.cholesky(S)
    assert np.abs(Lf - Lref).max() <= 1e-12 * np.abs(Lref).max()
    if env == {"PTZBA_CHOL_DELAY": "2", "PTZBA_ND_DEPTH": "1"}:
        assert ((tasks[:, 0] & 3) == 3).any()  # the delayed plan uses 2 x 2 trailing blocks
    if env.get("PTZBA_CHOL_BLOCKS") == "0":
        assert not ((tasks[:, 0] & 3) == 3).any()


def _tree_problem(win0, seed=0):
    """Synthetic landmarks over a coupling window: per frame f three landmarks on f plus 1-3 frames of (f, win[f]],
    the first of them reaching win[f] itself, so the records' own window is the given one (nondecreasing)."""
    rng = np.random.default_rng(seed)
    n = len(win0)
    fr, lm = [], []
    n_lm = 0
    for f in range(n):
        hi = int(win0[f])
        for q in range(3):
            F = {f}
            if hi > f:
                if q == 0:
                    F.add(hi)
                F |= {int(x) for x in rng.integers(f + 1, hi + 1, size=int(rng.integers(1, 4)))}
            fr += sorted(F)
            lm += [n_lm] * len(F)
            n_lm += 1
    return np.array(fr, np.int32), np.array(lm, np.int32), n_lm


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("env", [{}, {"PTZBA_CHOL_DELAY": "2"}, {"PTZBA_CHOL_DELAY": "2", "PTZBA_CHOL_BLOCKS": "0"}])
def test_rank_tree_plans_replay_to_the_cholesky_factor(monkeypatch, world, env):
    """Every rank's rank-tree plan (ptzba_dist_plan_export, host only), replayed on the CPU with the protocol's
    exchanges in between (a shared leaf's tiles summed over its group before its phase, an inner separator's over
    its group, the root's over all ranks; padding / augmented-diagonal set up per phase as k_chol_prepare does), on
    per-rank partial systems built from landmarks dealt by ptzba_partition_landmarks: each rank's factor over its
    columns (and the forward-substituted augmented row) equals numpy's Cholesky factor of the summed system -- the
    exactly-once split of the later phases' updates, the flush levels, delayed trailing updates and 2 x 2 blocks
    included.  Config 3's coupling window (two dissection levels: own subtrees at 2, X_SUB at 3 / 4, shared leaves
    at 8)."""
    for k in ("PTZBA_ND_DEPTH", "PTZBA_CHOL_DELAY", "PTZBA_CHOL_BLOCKS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    win0 = CASES["config3"]()
    frame, landmark, n_lm = _tree_problem(win0)
    n = len(win0)
    win = ptzba.frame_coupling_window(n, frame, landmark)
    owner, mode, _ = ptzba.partition_landmarks(n, n_lm, frame, landmark, world)
    assert mode == 1
    plans = [ptzba.dist_plan_export(win, world, r) for r in range(world)]
    pos, n_aug = plans[0][0], plans[0][3]
    assert all(np.array_equal(p[0], pos) for p in plans)
    ld = (n_aug + 1 + 31) // 32 * 32
    T = ld // cpe.NB
    taug = n_aug // cpe.NB
    rng = np.random.default_rng(1)
    S = [np.zeros((ld, ld)) for _ in range(world)]
    boosted = np.zeros(n, bool)
    for l in range(n_lm):
        F = [int(f) for f in frame[landmark == l] if f >= 1]
        if not F:
            continue
        rows = np.concatenate([pos[f] + np.arange(3) for f in F])
        G = rng.standard_normal((len(rows), 2))
        r = int(owner[l])
        S[r][np.ix_(rows, rows)] += G @ G.T
        S[r][n_aug, rows] += 0.1 * rng.standard_normal(len(rows))
        for f in F:  # diagonal dominance, each frame's once, by a rank that holds it
            if not boosted[f]:
                S[r][pos[f]:pos[f] + 3, pos[f]:pos[f] + 3] += 4.0 * len(F) * np.eye(3)
                boosted[f] = True
    pad = np.ones(ld, bool)
    for f in range(1, n):
        pad[pos[f]:pos[f] + 3] = False
    pad[n_aug:] = False
    full = sum(S)
    full = np.tril(full) + np.tril(full, -1).T
    full[pad, pad] = 1.0
    full[n_aug, n_aug] = 1e12
    full[n_aug + 1:, n_aug + 1:] = np.eye(ld - n_aug - 1)
    Lref = np.linalg.cholesky(full)
    A = [np.tril(s) for s in S]
    Ld = [dict() for _ in range(world)]
    NB = cpe.NB

    def tiles_sum(stage_kind):
        # sum each group's exchanged tiles (the ranks of one group list the same tiles in the same order)
        groups = {}
        for r, (_, _, _, _, phases, xts) in enumerate(plans):
            for q, ph in enumerate(phases):
                if ph[2] == stage_kind and (q > 0 or ph[4] > 1):
                    groups.setdefault((ph[3], ph[4]), []).append((r, xts[q]))
        for (r0, nr), members in groups.items():
            assert len(members) == nr
            xt = members[0][1]
            assert all(np.array_equal(m[1], xt) for m in members)
            sls = [(slice(ti * NB, (ti + 1) * NB), slice(tj * NB, (tj + 1) * NB)) for ti, tj in xt]
            if stage_kind == ptzba.X_PART:  # b over the shared leaf's rows travels as a vector range (the
                # library writes it into the augmented row at the first phase's prepare): the augmented row here
                cols = sorted({int(tj) for _, tj in xt})
                sls += [(slice(n_aug, n_aug + 1), slice(tj * NB, (tj + 1) * NB)) for tj in cols]
            for sl in sls:
                tot = sum(A[r][sl] for r, _ in members)
                for r, _ in members:
                    A[r][sl] = tot

    def run(r, q):
        _, tasks, off, _, phases, _ = plans[r]
        lv0, lv1, kind = phases[q][:3]
        # prepare: identity padding on this phase's rows; the root phase sets the augmented diagonal
        rows = [i for i in range(n_aug) if pad[i] and phase_of_col[r][i // NB] == q]
        for i in rows:
            A[r][i, i] = 1.0
        if kind == ptzba.X_SEP:
            A[r][n_aug, n_aug] = 1e12
            for i in range(n_aug + 1, ld):
                A[r][i, i] = 1.0
        cpe.replay_levels(A[r], Ld[r], tasks, off, lv0, lv1)

    phase_of_col = []
    for r in range(world):
        cp = -np.ones(T, int)
        _, tasks, off, _, phases, _ = plans[r]
        for q, ph in enumerate(phases):
            for L in range(ph[0], ph[1]):
                for t in tasks[off[L]:off[L + 1]]:
                    if (int(t[0]) & 3) == 0 and int(t[1]) == int(t[2]):
                        cp[int(t[2])] = q
        phase_of_col.append(cp)
    tiles_sum(ptzba.X_PART)
    for r in range(world):
        run(r, 0)
    tiles_sum(ptzba.X_SUB)
    for r in range(world):
        for q, ph in enumerate(plans[r][4]):
            if ph[2] == ptzba.X_SUB:
                run(r, q)
    tiles_sum(ptzba.X_SEP)
    for r in range(world):
        run(r, len(plans[r][4]) - 1)
    scale = np.abs(Lref[:n_aug, :n_aug]).max()
    for r in range(world):
        Lf, _ = cpe.assemble(A[r], Ld[r])
        cols = np.flatnonzero(phase_of_col[r] >= 0)
        for tj in cols:
            if tj >= taug:
                continue
            for ti in range(tj, T):
                sl = (slice(ti * NB, min((ti + 1) * NB, ld)), slice(tj * NB, (tj + 1) * NB))
                if ti == taug:
                    sl = (slice(n_aug, n_aug + 1), sl[1])  # the augmented row (y), not the diagonal's padding
                got, ref = Lf[sl], Lref[sl]
                if ti > tj and phase_of_col[r][ti] < 0:
                    continue
                assert np.abs(got - ref).max() <= 1e-9 * max(scale, np.abs(ref).max()), (world, r, ti, tj)
