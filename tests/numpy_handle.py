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
        S -= np.einsum('flik,gljk->figj', Y, Wf)
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
