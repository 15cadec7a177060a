"""Test infrastructure: a numpy implementation of the libptzba handle protocol (ptzba.BAHandle:
linearize / build_reduced / solve_reduced / read_scalars / accept / exchange) built on the oracle's
residual and analytic Jacobian, so the multi-rank host logic (ptzba.LMSolver with an all-reduce hook,
bench.shard_by_landmark) can run on CPU ranks over gloo.  It mirrors the library's split of the
scalars: `scal` holds rank-local (landmark / record) partials that are summed across ranks, `loc`
holds pose partials that every rank computes identically from the summed reduced system
(api.hip ptzba_read_scalars, ba_kernels.hip k_backsub / k_pose_trial).  Linear loss, fp64.
Never used by the product."""
import numpy as np

from oracle import ptz_oracle as orc


class NumpyBAHandle:
    def __init__(self):
        self.n_fixed = 1

    def set_problem(self, n_pose, n_landmark, frame, landmark, xy, u, v):
        self.n_pose, self.n_lm = int(n_pose), int(n_landmark)
        self.frame = np.asarray(frame, np.int64)
        self.landmark = np.asarray(landmark, np.int64)
        self.xy = np.asarray(xy, np.float64).reshape(-1, 2)
        self.u, self.v = float(u), float(v)
        self.nf = self.n_pose - self.n_fixed
        ns = 3 * self.nf
        self.sys = np.zeros(ns * ns + 3 * ns)
        self.scal = np.zeros(8)
        self.loc = np.zeros(8)
        self.info = 0

    def set_state(self, ptz, rays):
        self.ptz = np.array(ptz, np.float64).reshape(-1, 3)
        self.rays = np.array(rays, np.float64).reshape(-1, 2)
        self.D_pose = np.zeros(3 * self.n_pose)
        self.D_ray = np.zeros(2 * self.n_lm)

    def get_state(self):
        return self.ptz.copy(), self.rays.copy()

    # -------------------------------------------------------------------------------------------
    def _lin(self, ptz, rays):
        x_full = np.concatenate([ptz.reshape(-1), rays.reshape(-1)])
        r = orc.compute_residual_records(x_full, self.n_pose, self.u, self.v, self.frame, self.landmark,
                                         self.xy).reshape(-1, 2)
        J = orc.record_jacobian(self.u, self.v, ptz[self.frame], rays[self.landmark])
        Jp, Jr = J[:, :, :3], J[:, :, 3:]
        U = np.zeros((self.n_pose, 3, 3))
        gp = np.zeros((self.n_pose, 3))
        V = np.zeros((self.n_lm, 2, 2))
        gl = np.zeros((self.n_lm, 2))
        W = np.zeros((self.n_pose, self.n_lm, 3, 2))
        np.add.at(U, self.frame, np.einsum('rki,rkj->rij', Jp, Jp))
        np.add.at(gp, self.frame, np.einsum('rki,rk->ri', Jp, r))
        np.add.at(V, self.landmark, np.einsum('rki,rkj->rij', Jr, Jr))
        np.add.at(gl, self.landmark, np.einsum('rki,rk->ri', Jr, r))
        np.add.at(W, (self.frame, self.landmark), np.einsum('rki,rkj->rij', Jp, Jr))
        present = np.zeros(self.n_lm, bool)
        present[self.landmark] = True
        return dict(cost=0.5 * float(np.sum(r * r)), U=U, gp=gp, V=V, gl=gl, W=W, present=present)

    def linearize(self):
        self.cur = self._lin(self.ptz, self.rays)
        self.scal[:] = 0
        self.scal[0] = self.cur['cost']

    def build_reduced(self, lam):
        L = self.cur
        self.lam = float(lam)
        nf, fx = self.nf, self.n_fixed
        dV = np.stack([L['V'][:, 0, 0], L['V'][:, 1, 1]], 1).reshape(-1)
        self.D_ray = np.where(L['present'].repeat(2), np.maximum(self.D_ray, np.maximum(dV, 1e-12)), self.D_ray)
        Vd = L['V'] + self.lam * np.einsum('lk,kj->lkj', self.D_ray.reshape(-1, 2), np.eye(2))
        Vinv = np.zeros_like(Vd)
        Vinv[L['present']] = np.linalg.inv(Vd[L['present']])
        self.Vinv = Vinv
        Wf = L['W'][fx:]                                   # [nf, nl, 3, 2]
        Y = np.einsum('flij,ljk->flik', Wf, Vinv)          # W V^-1
        S = np.zeros((nf, 3, nf, 3))
        for f in range(nf):
            S[f, :, f, :] += L['U'][fx + f]
        # S -= sum_lk Y[f,l,i,k] W[g,l,j,k], as one BLAS product (a plain einsum loops for seconds at 160 frames)
        nl = Y.shape[1]
        Ym = Y.transpose(0, 2, 1, 3).reshape(nf * 3, nl * 2)
        Wm = Wf.transpose(0, 2, 1, 3).reshape(nf * 3, nl * 2)
        S -= (Ym @ Wm.T).reshape(nf, 3, nf, 3)
        b = -L['gp'][fx:] + np.einsum('flik,lk->fi', Y, L['gl'])
        ns = 3 * nf
        self.sys[:ns * ns] = S.reshape(ns, ns).reshape(-1)
        self.sys[ns * ns:ns * ns + ns] = b.reshape(-1)
        self.sys[ns * ns + ns:ns * ns + 2 * ns] = L['gp'][fx:].reshape(-1)
        self.sys[ns * ns + 2 * ns:] = np.stack([L['U'][fx:, k, k] for k in range(3)], 1).reshape(-1)

    def solve_reduced(self):
        L = self.cur
        ns = 3 * self.nf
        S = self.sys[:ns * ns].reshape(ns, ns).copy()
        b = self.sys[ns * ns:ns * ns + ns]
        gpose = self.sys[ns * ns + ns:ns * ns + 2 * ns]
        dU = self.sys[ns * ns + 2 * ns:]
        fx3 = 3 * self.n_fixed
        self.D_pose[fx3:] = np.maximum(self.D_pose[fx3:], dU)
        S[np.diag_indices(ns)] += self.lam * self.D_pose[fx3:]
        try:
            Lc = np.linalg.cholesky(S)
            dp = np.linalg.solve(Lc.T, np.linalg.solve(Lc, b))
            self.info = 0
        except np.linalg.LinAlgError:
            dp = np.zeros(ns)
            self.info = 1
        self.ptz_trial = self.ptz.copy()
        self.ptz_trial[self.n_fixed:] += dp.reshape(-1, 3)
        t = L['gl'] + np.einsum('flij,fi->lj', L['W'][self.n_fixed:], dp.reshape(-1, 3))
        dl = -np.einsum('lij,lj->li', self.Vinv, t)
        dl[~L['present']] = 0
        self.rays_trial = self.rays + dl
        self.trial = self._lin(self.ptz_trial, self.rays_trial)
        pres = L['present']
        Dr = self.D_ray.reshape(-1, 2)
        self.scal[:] = 0
        self.scal[1] = self.trial['cost']
        self.scal[2] = float(np.sum((-0.5 * np.sum(L['gl'] * dl, 1) + 0.5 * self.lam * np.sum(Dr * dl * dl, 1))[pres]))
        self.scal[3] = float(np.sum((dl * dl)[pres]))
        self.scal[4] = float(np.sum((self.rays * self.rays)[pres]))
        self.loc[:] = 0
        self.loc[0] = float(-0.5 * gpose @ dp + 0.5 * self.lam * np.sum(self.D_pose[fx3:] * dp * dp))
        self.loc[1] = float(dp @ dp)
        self.loc[2] = float(np.sum(self.ptz * self.ptz))
        self.loc[3] = float(np.max(np.abs(gpose))) if ns else 0.0
        self.scal[0] = self.cur['cost']

    def read_scalars(self):
        s, l = self.scal, self.loc
        return np.array([s[0], s[1], s[2] + l[0], s[3] + l[1], s[4] + l[2], float(self.info), l[3], 0.0])

    def accept(self, ok):
        if ok:
            self.ptz, self.rays = self.ptz_trial, self.rays_trial
            self.cur = self.trial
            self.scal[0] = self.cur['cost']

    def exchange(self):
        return self.sys, self.scal

    def sync(self):
        pass


class NumpyPartHandle(NumpyBAHandle):
    """The PART-OWNED multi-GPU protocol of libptzba (include/ptzba.h, api.hip make_plan_part / solve_impl) in
    numpy: this rank holds the landmarks ptzba_partition_landmarks gave it (they see its part P = A or B and
    the separator C only); it factors P, forms P's Schur update of C locally, and sums only the separator
    block over the ranks (X_SEP; a group's non-leaders send zeros), after summing P's interior inside its
    rank group when the group has more than one rank (X_PART).  Pose partials are counted once over all ranks
    (P's frames by the group leader, C's and the fixed frames by rank 0) and summed with the landmark partials
    and the factorisation status (X_SCAL, 16 values).  `hook(kind, array)` sums in place over the kind's ranks.
    The handle runs its exchanges itself (internal_exchange), like a GPU handle with a comm or hook."""
    internal_exchange = True

    def set_dist(self, world, rank, split, hook):
        m, cend, _ = split
        g0 = (world + 1) // 2
        self.part = 0 if rank < g0 else 1
        self.group_size = g0 if self.part == 0 else world - g0
        self.leader = rank in (0, g0)
        self.rank = rank
        self.hook = hook
        fx = self.n_fixed
        free = np.arange(fx, self.n_pose)
        self.P = free[(free < m) if self.part == 0 else (free >= cend)] - fx
        self.C = free[(free >= m) & (free < cend)] - fx
        owned = np.zeros(self.n_pose, bool)
        owned[self.P + fx] = True
        owned[self.C + fx] = True
        self.owned = owned
        cnt = np.zeros(self.n_pose, bool)
        if self.leader:
            cnt[self.P + fx] = True
        if rank == 0:
            cnt[self.C + fx] = True
            cnt[:fx] = True
        self.counted = cnt
        assert np.all(owned[self.frame[self.frame >= fx]]), "a record sees a frame outside this rank's part"

    def linearize(self):
        super().linearize()
        self.loc[:] = 0
        red = np.concatenate([self.scal, self.loc])  # only the cost is used here
        self.hook("scal", red)
        self.scal[:], self.loc[:] = red[:8], red[8:]

    def build_reduced(self, lam):
        super().build_reduced(lam)
        if self.group_size > 1:
            self.hook("part", self.sys)

    def solve_reduced(self):
        L = self.cur
        ns = 3 * self.nf
        fx, fx3 = self.n_fixed, 3 * self.n_fixed
        S = self.sys[:ns * ns].reshape(ns, ns).copy()
        b = self.sys[ns * ns:ns * ns + ns].copy()
        gpose = self.sys[ns * ns + ns:ns * ns + 2 * ns].copy()
        dU = self.sys[ns * ns + 2 * ns:].copy()
        rows = lambda fr: (3 * fr[:, None] + np.arange(3)).reshape(-1)  # noqa: E731
        p, c = rows(self.P), rows(self.C)
        D = self.D_pose[fx3:]
        D[p] = np.maximum(D[p], dU[p])
        info = 0
        try:
            Lpp = np.linalg.cholesky(S[np.ix_(p, p)] + np.diag(self.lam * D[p]))
            Lcp = np.linalg.solve(Lpp, S[np.ix_(c, p)].T).T
            yp = np.linalg.solve(Lpp, b[p])
        except np.linalg.LinAlgError:
            info = 1
            Lpp = np.eye(len(p)); Lcp = np.zeros((len(c), len(p))); yp = np.zeros(len(p))
        Scc = S[np.ix_(c, c)] - Lcp @ Lcp.T
        bc = b[c] - Lcp @ yp
        sep = np.concatenate([Scc.reshape(-1), bc, gpose[c], dU[c]])
        if not self.leader:
            sep[:] = 0.0
        self.hook("sep", sep)
        k = len(c)
        Scc, bc = sep[:k * k].reshape(k, k), sep[k * k:k * k + k]
        gpose[c], dU[c] = sep[k * k + k:k * k + 2 * k], sep[k * k + 2 * k:]
        D[c] = np.maximum(D[c], dU[c])
        dp = np.zeros(ns)
        try:
            Lcc = np.linalg.cholesky(Scc + np.diag(self.lam * D[c]))
            dp[c] = np.linalg.solve(Lcc.T, np.linalg.solve(Lcc, bc))
        except np.linalg.LinAlgError:
            info = 1
        dp[p] = np.linalg.solve(Lpp.T, yp - Lcp.T @ dp[c])
        self.info = info
        self._finish_trial(dp, gpose, D, info)

    def _finish_trial(self, dp, gpose, D, info):
        L = self.cur
        fx = self.n_fixed
        self.ptz_trial = self.ptz.copy()
        self.ptz_trial[fx:] += dp.reshape(-1, 3)
        t = L['gl'] + np.einsum('flij,fi->lj', L['W'][fx:], dp.reshape(-1, 3))
        dl = -np.einsum('lij,lj->li', self.Vinv, t)
        dl[~L['present']] = 0
        self.rays_trial = self.rays + dl
        self.trial = self._lin(self.ptz_trial, self.rays_trial)
        pres = L['present']
        Dr = self.D_ray.reshape(-1, 2)
        self.scal[:] = 0
        self.scal[0] = self.cur['cost']
        self.scal[1] = self.trial['cost']
        self.scal[2] = float(np.sum((-0.5 * np.sum(L['gl'] * dl, 1) + 0.5 * self.lam * np.sum(Dr * dl * dl, 1))[pres]))
        self.scal[3] = float(np.sum((dl * dl)[pres]))
        self.scal[4] = float(np.sum((self.rays * self.rays)[pres]))
        cr = self.counted[fx:].repeat(3)  # counted free rows
        self.loc[:] = 0
        self.loc[0] = float(np.sum((-0.5 * gpose * dp + 0.5 * self.lam * D * dp * dp)[cr]))
        self.loc[1] = float(np.sum((dp * dp)[cr]))
        self.loc[2] = float(np.sum((self.ptz * self.ptz)[self.counted]))
        self.loc[3] = float(np.max(np.abs(gpose[cr]))) if cr.any() else 0.0
        self.loc[4] = float(info)
        red = np.concatenate([self.scal, self.loc])
        self.hook("scal", red)
        self.scal[:], self.loc[:] = red[:8], red[8:]

    def read_scalars(self):
        s, l = self.scal, self.loc
        return np.array([s[0], s[1], s[2] + l[0], s[3] + l[1], s[4] + l[2], l[4], l[3], 0.0])

    def accept(self, ok):
        if ok:
            self.ptz, self.rays = self.ptz_trial, self.rays_trial
            self.cur = self.trial
            self.scal[0] = self.cur['cost']


class NumpyTreeHandle(NumpyPartHandle):
    """The RANK-TREE protocol of libptzba (round 4: include/ptzba.h, api.hip make_plan_tree / solve_impl) in numpy.
    The rank's phases come from the library's own plan (ptzba.dist_rank_phases: its base -- own subtree or shared
    leaf -- then each ancestor separator up to the root, with each node's rank group).  Before a phase its columns
    (the phase block, the later phases' rows against it, b, g and diag U over its rows) are summed over the phase's
    group -- a shared leaf's before the first phase ('part'), an inner separator's ('sub'), the root's ('sep') --
    then the phase is damped and eliminated, and its Schur update of the later phases is applied by ONE group member
    per entry (frame pair (f_i + f_j) mod group size; b by (f_i + n_pose) mod size): the exactly-once rule, here per
    frame block where the library splits per 32-row tile.  Back-substitution runs the phases from the root down.
    `hook(kind, array, (r0, nr))` sums in place over ranks [r0, r0 + nr)."""

    def set_dist(self, world, rank, phases, hook):
        fx = self.n_fixed
        self.rank, self.world, self.hook = rank, world, hook
        self.phases = []
        owned = np.zeros(self.n_pose, bool)
        cnt = np.zeros(self.n_pose, bool)
        for kind, r0, nr, f0, f1 in phases:
            fr = np.arange(max(f0, fx), f1)
            owned[fr] = True
            if rank == r0:
                cnt[fr] = True  # a phase's frames are counted by its group's first rank
            self.phases.append((kind, r0, nr, fr - fx))
        if rank == 0:
            cnt[:fx] = True
        self.owned, self.counted = owned, cnt
        self.group_size = 1  # (no whole-system group sum in build_reduced: the phases sum their columns)
        assert np.all(owned[self.frame[self.frame >= fx]]), "a record sees a frame outside this rank's phases"

    def linearize(self):
        super().linearize()

    def _sum(self, kind, arr, grp):
        self.hook(kind, arr, grp)

    def solve_reduced(self):
        import ptzba
        ns = 3 * self.nf
        fx, fx3 = self.n_fixed, 3 * self.n_fixed
        S = self.sys[:ns * ns].reshape(ns, ns).copy()
        b = self.sys[ns * ns:ns * ns + ns].copy()
        gpose = self.sys[ns * ns + ns:ns * ns + 2 * ns].copy()
        dU = self.sys[ns * ns + 2 * ns:].copy()
        rows = lambda fr: (3 * fr[:, None] + np.arange(3)).reshape(-1)  # noqa: E731
        P = [rows(ph[3]) for ph in self.phases]
        D = self.D_pose[fx3:]
        info = 0
        elim = []
        for q, (kind, r0, nr, _) in enumerate(self.phases):
            p = P[q]
            R = np.concatenate(P[q + 1:]) if q + 1 < len(P) else np.zeros(0, np.int64)
            if q > 0 or nr > 1:  # the phase's columns summed over its group
                k, m = len(p), len(R)
                buf = np.concatenate([S[np.ix_(p, p)].reshape(-1), S[np.ix_(R, p)].reshape(-1), b[p], gpose[p], dU[p]])
                self._sum(ptzba.X_NAMES[kind], buf, (r0, nr))
                S[np.ix_(p, p)] = buf[:k * k].reshape(k, k)
                S[np.ix_(R, p)] = buf[k * k:k * k + m * k].reshape(m, k)
                S[np.ix_(p, R)] = S[np.ix_(R, p)].T
                o = k * k + m * k
                b[p], gpose[p], dU[p] = buf[o:o + k], buf[o + k:o + 2 * k], buf[o + 2 * k:]
            D[p] = np.maximum(D[p], dU[p])
            try:
                Lq = np.linalg.cholesky(S[np.ix_(p, p)] + np.diag(self.lam * D[p]))
                X = np.linalg.solve(Lq, S[np.ix_(R, p)].T).T
                y = np.linalg.solve(Lq, b[p])
            except np.linalg.LinAlgError:
                info = 1
                Lq, X, y = np.eye(len(p)), np.zeros((len(R), len(p))), np.zeros(len(p))
            me = self.rank - r0
            fR = R // 3 + fx
            own = (fR[:, None] + fR[None, :]) % nr == me
            ownb = (fR + self.n_pose) % nr == me
            S[np.ix_(R, R)] -= np.where(own, X @ X.T, 0.0)
            b[R] -= np.where(ownb, X @ y, 0.0)
            elim.append((p, R, Lq, X, y))
        dp = np.zeros(ns)
        for p, R, Lq, X, y in reversed(elim):
            dp[p] = np.linalg.solve(Lq.T, y - X.T @ dp[R])
        self.info = info
        self._finish_trial(dp, gpose, D, info)
