"""CPU replay of libptzba's level-scheduled tile Cholesky (chol_kernels.hip k_chol_step) on a plan exported by
ptzba_plan_export: test infrastructure that checks a factorisation PLAN (order, fill, levels, update panels,
delayed trailing updates, 2 x 2 trailing blocks) against numpy's Cholesky of the same matrix, without a GPU.

Task semantics (one int4 record, chol_kernels.hip):
  type 0  panel (i, k):  D = A_kk - sum_u L_k,p_u L_k,p_u^T;  T = A_ik - sum_{u in tmask} L_i,p_u L_k,p_u^T;
                         L_kk = chol(D) (i == k: to Ldiag, A_kk untouched), else A_ik <- T L_kk^-T
  type 1  trailing (i, j): A_ij -= sum_u L_i,p_u L_j,p_u^T
  type 2  inverse of a diagonal factor tile (no effect on the factor)
  type 3  2 x 2 trailing block: tiles (i + a, j + b) of the mask, each as type 1 with the block's panels
(Round 4's supercolumn tasks and their continuation records were removed in round 6 with chol_super.)
"""
import numpy as np

NB = 32


def decode(t):
    x, y, z, w = (int(v) & 0xFFFFFFFF for v in t)
    typ = x & 3
    ups = [(w & 0x3FFF) - 1, ((w >> 14) & 0x3FFF) - 1, ((x >> 2) & 0x3FFF) - 1, ((x >> 16) & 0x3FFF) - 1]
    tmask = ((w >> 28) & 3) | ((x >> 30) << 2)
    return typ, y, z, ups, tmask


def test_matrix(pos, win, n_aug, ld, n_fixed=1, seed=0):
    """SPD matrix with the reduced camera system's structure: 3x3 blocks for coupled frame pairs at the system
    positions, identity padding rows, an augmented right-hand-side row with a dominant diagonal."""
    rng = np.random.default_rng(seed)
    n = len(pos)
    S = np.zeros((ld, ld))
    for f1 in range(n_fixed, n):
        for f2 in range(f1, int(win[f1]) + 1):
            p1, p2 = pos[f1], pos[f2]
            blk = rng.standard_normal((3, 3))
            S[p2:p2 + 3, p1:p1 + 3] += blk
            if p1 != p2:
                S[p1:p1 + 3, p2:p2 + 3] += blk.T
            else:
                S[p1:p1 + 3, p1:p1 + 3] = 0.5 * (S[p1:p1 + 3, p1:p1 + 3] + S[p1:p1 + 3, p1:p1 + 3].T)
    rows = np.zeros(ld, bool)
    for f in range(n_fixed, n):
        rows[pos[f]:pos[f] + 3] = True
    S[np.arange(ld), np.arange(ld)] = np.where(rows, np.abs(S).sum(1) + 1.0, 1.0)
    b = rng.standard_normal(n_aug) * rows[:n_aug]
    S[n_aug, :n_aug] = b
    S[:n_aug, n_aug] = b
    S[n_aug, n_aug] = np.abs(b).sum() * 1e3 + 1.0
    return S


def replay(S, tasks, level_off):
    """Run the task list level by level on a copy of S (lower tiles); returns the assembled lower factor."""
    ld = S.shape[0]
    T = ld // NB
    A = np.tril(S).copy()
    Ldiag = {}
    replay_levels(A, Ldiag, tasks, level_off, 0, len(level_off) - 1)
    return assemble(A, Ldiag)


def assemble(A, Ldiag):
    T = A.shape[0] // NB
    Lf = np.zeros_like(A)
    for a in range(T):
        for b in range(a):
            Lf[a * NB:(a + 1) * NB, b * NB:(b + 1) * NB] = A[a * NB:(a + 1) * NB, b * NB:(b + 1) * NB]
        if a in Ldiag:
            Lf[a * NB:(a + 1) * NB, a * NB:(a + 1) * NB] = Ldiag[a]
    return Lf, Ldiag


def replay_levels(A, Ldiag, tasks, level_off, L0, L1):
    """Levels [L0, L1) of a task list on A (lower tiles, in place); diagonal factor tiles go to Ldiag."""

    def tile(a, b):
        return A[a * NB:(a + 1) * NB, b * NB:(b + 1) * NB]

    def sym(a):
        return np.tril(a) + np.tril(a, -1).T

    for L in range(L0, L1):
        writes = []  # a level's results land after all its tasks read (the tasks of one launch run concurrently)
        for q in range(level_off[L], level_off[L + 1]):
            typ, i, j, ups, tmask = decode(tasks[q])
            if typ == 2:
                continue
            if typ in (1, 3):
                outs = [(i, j)] if typ == 1 else [(i + (m >> 1), j + (m & 1)) for m in range(4) if (tmask >> m) & 1]
                for (ti, tj) in outs:
                    C = tile(ti, tj)
                    for p in ups:
                        if p >= 0:
                            C -= tile(ti, p) @ tile(tj, p).T
                continue
            k = j
            D = np.tril(tile(k, k)) + np.tril(tile(k, k), -1).T
            Tt = tile(i, k).copy() if i != k else None
            for u, p in enumerate(ups):
                if p < 0:
                    continue
                D = D - tile(k, p) @ tile(k, p).T
                if Tt is not None and (tmask >> u) & 1:
                    Tt -= tile(i, p) @ tile(k, p).T
            Lkk = np.linalg.cholesky(D)
            if i == k:
                Ldiag[k] = Lkk
            else:
                tile(i, k)[:] = np.linalg.solve(Lkk, Tt.T).T
        for (a, b), v in writes:
            tile(a, b)[:] = v
