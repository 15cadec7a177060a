"""Multi-rank host path on CPU ranks over gloo, world_size 2.

bench.py's N>1 protocol: records sharded by landmark block (bench.shard_by_landmark), poses replicated,
ptzba.LMSolver with an all-reduce hook that sums the reduced camera system ('sys') and the rank-local
scalars ('scal') in place.  The handle here is tests/numpy_handle.py (the library's handle protocol
in numpy — there is no GPU in this container); the GPU handle exposes the same two buffers through
ptzba_exchange.  A 2-rank solve must reproduce the 1-rank solve of the whole problem."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


# a Marquardt start (rounds 1-4's default): the ranks' solves sum in a different order than the single-rank
# solve, and with Gauss-Newton steps (ptzba.LAMBDA0) the tight ftol test fires at round-off, where the iteration
# count is not reproducible across summation orders; damped steps keep the last reductions above it
DAMPED = 1e-4

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(prob, frame, landmark, xy, allreduce=None, iters=12):
    import ptzba
    from numpy_handle import NumpyBAHandle
    h = NumpyBAHandle()
    h.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v)
    h.set_state(prob.init_ptz, prob.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-9, xtol=1e-12, max_iter=iters, allreduce=allreduce, lambda0=DAMPED).run()
    ptz, rays = h.get_state()
    return res, ptz, rays


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import bench
    import synthetic
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = synthetic.make_problem("config1", seed=0)
    sel = bench.shard_by_landmark(prob.landmark, prob.n_landmark, rank, world)
    from numpy_handle import NumpyBAHandle  # noqa: F401  (import check before the solve)
    holder = {}

    def allreduce(kind):
        h = holder["h"]
        sys_, scal = h.exchange()
        dist.all_reduce(torch.from_numpy(sys_ if kind == "sys" else scal))

    import ptzba
    h = NumpyBAHandle()
    holder["h"] = h
    h.set_problem(prob.n_pose, prob.n_landmark, prob.frame[sel], prob.landmark[sel], prob.xy[sel], prob.u, prob.v)
    h.set_state(prob.init_ptz, prob.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-9, xtol=1e-12, max_iter=12, allreduce=allreduce, lambda0=DAMPED).run()
    ptz, rays = h.get_state()
    owned = np.zeros(prob.n_landmark, bool)
    owned[prob.landmark[sel]] = True
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), ptz=ptz, rays=rays, owned=owned, cost=res.cost,
             njev=res.njev, n_rec=int(sel.sum()))
    dist.barrier()
    dist.destroy_process_group()


def test_landmark_shards_partition_records():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    import bench
    import synthetic
    p = synthetic.make_problem("config1", seed=0)
    for world in (2, 3, 8):
        masks = [bench.shard_by_landmark(p.landmark, p.n_landmark, r, world) for r in range(world)]
        tot = np.sum(masks, axis=0)
        assert np.all(tot == 1)  # every record on exactly one rank
        for m in masks:  # a landmark never straddles ranks
            assert not np.intersect1d(np.unique(p.landmark[m]), np.unique(p.landmark[~m])).size


def test_two_rank_solve_matches_single_rank(tmp_path):
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    import synthetic
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    prob = synthetic.make_problem("config1", seed=0)
    res1, ptz1, rays1 = _solve(prob, prob.frame, prob.landmark, prob.xy)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    assert sum(int(o["n_rec"]) for o in outs) == len(prob.frame)
    for o in outs:
        # poses are replicated and identical to the 1-rank solve
        np.testing.assert_allclose(o["ptz"], ptz1, rtol=0, atol=1e-9)
        # each rank's own landmarks match
        np.testing.assert_allclose(o["rays"][o["owned"]], rays1[o["owned"]], rtol=0, atol=1e-9)
        assert abs(float(o["cost"]) - res1.cost) <= 1e-9 * res1.cost
        assert int(o["njev"]) == res1.njev
    # and the solve reached the (tight) least-squares optimum of the whole problem
    from oracle import ptz_oracle as orc
    x_full = np.concatenate([ptz1.reshape(-1), rays1.reshape(-1)])
    J = orc.ba_jacobian(x_full[3:], prob.n_pose, prob.n_landmark, prob.u, prob.v, ptz1[0],
                        prob.frame.astype(np.int64), prob.landmark.astype(np.int64))
    r = orc.compute_residual_records(x_full, prob.n_pose, prob.u, prob.v, prob.frame.astype(np.int64),
                                     prob.landmark.astype(np.int64), prob.xy)
    g = J.T @ r
    assert res1.status == 2 and np.abs(g).max() < 1e-4 * np.abs(J).max()


def _bench_line(out):
    import json
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def test_bench_gpus_launches_ranks():
    """`bench.py --gpus 2` outside a launcher starts 2 ranks (torch.distributed.run child process) that
    rendezvous over gloo; --dry-run stops after the rendezvous (no GPU in this container)."""
    import subprocess
    env = dict(os.environ, PTZBA_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"


def test_bench_rejects_world_size_mismatch():
    """A launcher world size that differs from --gpus is an error (exit 3), never a silent N=1 run."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def _part_worker(rank, world, port, out_dir):
    """One rank of a PART-OWNED solve (include/ptzba.h): landmarks from ptzba_partition_landmarks, the part's
    interior summed in its rank group ('part', only with > 1 rank per group), the separator block over all
    ranks ('sep'), the partial scalars ('scal') -- numpy emulation of the library's protocol over gloo."""
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ptzba
    import synthetic
    from numpy_handle import NumpyPartHandle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g0 = (world + 1) // 2
    groups = [dist.new_group(list(range(g0))), dist.new_group(list(range(g0, world)))]
    mine = groups[0 if rank < g0 else 1]
    prob = synthetic.make_problem("config2", seed=0)
    owner, mode, split = ptzba.partition_landmarks(prob.n_pose, prob.n_landmark, prob.frame, prob.landmark, world)
    assert mode == 1, "config 2 splits"
    sel = owner[prob.landmark] == rank

    def hook(kind, arr):
        dist.all_reduce(torch.from_numpy(arr), group=mine if kind == "part" else None)

    h = NumpyPartHandle()
    h.set_problem(prob.n_pose, prob.n_landmark, prob.frame[sel], prob.landmark[sel], prob.xy[sel], prob.u, prob.v)
    h.set_dist(world, rank, split, hook)
    h.set_state(prob.init_ptz, prob.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-9, xtol=1e-12, max_iter=8, lambda0=DAMPED).run()
    ptz, rays = h.get_state()
    own_lm = np.zeros(prob.n_landmark, bool)
    own_lm[prob.landmark[sel]] = True
    np.savez(os.path.join(out_dir, f"part{world}_rank{rank}.npz"), ptz=ptz, rays=rays, owned=h.owned, own_lm=own_lm,
             cost=res.cost, njev=res.njev, n_rec=int(sel.sum()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_part_owned_solve_matches_single_rank(tmp_path, world):
    """The part-owned multi-GPU protocol (each rank factors its part A or B plus the separator C; only C is
    summed over all ranks, the part's interior inside its rank group when the group has > 1 rank) reproduces
    the 1-rank solve of the whole problem (config 2: A = frames 1-9, C = 10-42, B = 43-49): same iterations
    and cost, every owned pose and every rank's rays within 1e-8; every frame is owned by some rank."""
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    import synthetic
    mp.start_processes(_part_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    prob = synthetic.make_problem("config2", seed=0)
    res1, ptz1, rays1 = _solve(prob, prob.frame, prob.landmark, prob.xy, iters=8)
    outs = [np.load(os.path.join(tmp_path, f"part{world}_rank{r}.npz")) for r in range(world)]
    assert sum(int(o["n_rec"]) for o in outs) == len(prob.frame)
    covered = np.zeros(prob.n_pose, bool)
    for o in outs:
        own = o["owned"]
        covered |= own
        np.testing.assert_allclose(o["ptz"][own], ptz1[own], rtol=0, atol=1e-8)
        np.testing.assert_allclose(o["rays"][o["own_lm"]], rays1[o["own_lm"]], rtol=0, atol=1e-8)
        assert abs(float(o["cost"]) - res1.cost) <= 1e-10 * res1.cost
        assert int(o["njev"]) == res1.njev
    assert covered[1:].all()


def _tree_problem():
    import synthetic
    return synthetic.make_small_problem(160, 1000, -100.0, 100.0, seed=1)  # 160 KF: a two-level rank tree


def _tree_worker(rank, world, port, out_dir):
    """One rank of the RANK-TREE solve (include/ptzba.h, round 4): landmarks from ptzba_partition_landmarks, the
    rank's phases from the library's plan (ptzba.dist_rank_phases), each phase's columns summed over its node's
    rank group before it, the exactly-once split of the later phases' updates -- numpy emulation over gloo."""
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ptzba
    from numpy_handle import NumpyTreeHandle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = _tree_problem()
    win = ptzba.frame_coupling_window(prob.n_pose, prob.frame, prob.landmark)
    owner, mode, _ = ptzba.partition_landmarks(prob.n_pose, prob.n_landmark, prob.frame, prob.landmark, world)
    assert mode == 1
    # every tree group, created on every rank in the same order (the phases of all ranks name them)
    all_groups = sorted({(r0, nr) for r in range(world) for _, r0, nr, _, _ in ptzba.dist_rank_phases(win, world, r)
                         if 1 < nr < world})
    groups = {g: dist.new_group(list(range(g[0], g[0] + g[1]))) for g in all_groups}
    phases = ptzba.dist_rank_phases(win, world, rank)
    sel = owner[prob.landmark] == rank
    kinds = []

    def hook(kind, arr, grp=None):
        kinds.append(kind)
        g = None if grp is None or grp[1] == world else groups[grp]
        dist.all_reduce(torch.from_numpy(arr), group=g)

    h = NumpyTreeHandle()
    h.set_problem(prob.n_pose, prob.n_landmark, prob.frame[sel], prob.landmark[sel], prob.xy[sel], prob.u, prob.v)
    h.set_dist(world, rank, phases, hook)
    h.set_state(prob.init_ptz, prob.init_rays)
    res = ptzba.LMSolver(h, ftol=1e-9, xtol=1e-12, max_iter=6, lambda0=DAMPED).run()
    ptz, rays = h.get_state()
    own_lm = np.zeros(prob.n_landmark, bool)
    own_lm[prob.landmark[sel]] = True
    np.savez(os.path.join(out_dir, f"tree{world}_rank{rank}.npz"), ptz=ptz, rays=rays, owned=h.owned, own_lm=own_lm,
             cost=res.cost, njev=res.njev, n_rec=int(sel.sum()), kinds=np.array(sorted(set(kinds))),
             phases=np.array(phases, np.int64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 6])
def test_rank_tree_solve_matches_single_rank(tmp_path, world):
    """The rank-tree protocol (round 4) on a 160-keyframe chain whose order has two dissection levels: at 2 ranks
    each owns a half (own subtree) and only the root separator is summed; at 4 each owns a leaf and the inner
    separators are summed over pairs ('sub'); at 6 the first leaf of each half is shared by two ranks ('part').  With
    the later phases' updates split over the group members (exactly once), the result equals the 1-rank solve:
    same iterations and cost, every owned pose and every rank's rays within 1e-8, every frame owned."""
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    mp.start_processes(_tree_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    prob = _tree_problem()
    res1, ptz1, rays1 = _solve(prob, prob.frame, prob.landmark, prob.xy, iters=6)
    outs = [np.load(os.path.join(tmp_path, f"tree{world}_rank{r}.npz")) for r in range(world)]
    assert sum(int(o["n_rec"]) for o in outs) == len(prob.frame)
    covered = np.zeros(prob.n_pose, bool)
    kinds = set()
    for o in outs:
        own = o["owned"]
        covered |= own
        kinds |= set(o["kinds"].tolist())
        np.testing.assert_allclose(o["ptz"][own], ptz1[own], rtol=0, atol=1e-8)
        np.testing.assert_allclose(o["rays"][o["own_lm"]], rays1[o["own_lm"]], rtol=0, atol=1e-8)
        assert abs(float(o["cost"]) - res1.cost) <= 1e-10 * res1.cost
        assert int(o["njev"]) == res1.njev
    assert covered[1:].all()
    want = {"sep", "scal"} | ({"sub"} if world >= 3 else set()) | ({"part"} if world >= 6 else set())
    assert kinds == want, kinds
