"""Sharded solve through libptzba on the GPU: two ranks on one device over gloo, records
sharded by landmark block (bench.shard_by_landmark), the library's packed exchange buffer and partial
scalars all-reduced by ptzba.LMSolver's hook -- the protocol bench.py --gpus N runs over RCCL.  The 2-rank
solve must reproduce the 1-rank solve of the whole problem: same iterations, poses and each rank's own
rays within 1e-8 (the reduced system is summed from two partials instead of one: rounding only)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
pytestmark = pytest.mark.gpu

CFG = dict(precision="fp64", loss="linear", ftol=1e-10, max_iter=8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solve(h, prob, allreduce=None):
    import ptzba
    h.set_state(prob.init_ptz, prob.init_rays)
    res = ptzba.LMSolver(h, ftol=CFG["ftol"], xtol=1e-14, max_iter=CFG["max_iter"], allreduce=allreduce).run()
    ptz, rays = h.get_state()
    return res, ptz, rays


def _handle(prob, frame, landmark, xy, win_hi, device=0):
    import ptzba
    h = ptzba.BAHandle(device)
    h.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v, precision=ptzba.FP64,
                  loss=ptzba.LOSS_LINEAR, frame_win_hi=win_hi)
    return h


def _worker(rank, world, port, out_dir, config):
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import bench
    import ptzba
    import synthetic
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = synthetic.make_problem(config, seed=0)
    win_hi = ptzba.frame_coupling_window(prob.n_pose, prob.frame, prob.landmark)
    sel = bench.shard_by_landmark(prob.landmark, prob.n_landmark, rank, world)
    h = _handle(prob, prob.frame[sel], prob.landmark[sel], prob.xy[sel], win_hi)
    h.set_stream(torch.cuda.current_stream().cuda_stream)
    xb_ptr, xb_n = h.exchange_packed()
    _, _, scal_ptr = h.exchange()
    t_sys = torch.as_tensor(bench._DevArray(xb_ptr, xb_n), device="cuda:0")
    t_scal = torch.as_tensor(bench._DevArray(scal_ptr, ptzba.NSCALARS), device="cuda:0")

    def allreduce(kind):
        if kind == "sys":
            h.pack()
            dist.all_reduce(t_sys)
            h.unpack()
        else:
            dist.all_reduce(t_scal)

    res, ptz, rays = _solve(h, prob, allreduce)
    owned = np.zeros(prob.n_landmark, bool)
    owned[prob.landmark[sel]] = True
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), ptz=ptz, rays=rays, owned=owned, cost=res.cost,
             njev=res.njev, n_rec=int(sel.sum()), xb_n=xb_n)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["config1", "config2"])
def test_two_rank_gpu_solve_matches_single_rank(gpu_available, tmp_path, config):
    import ptzba
    import synthetic
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), config), nprocs=world, join=True,
                       start_method="spawn")
    prob = synthetic.make_problem(config, seed=0)
    win_hi = ptzba.frame_coupling_window(prob.n_pose, prob.frame, prob.landmark)
    res1, ptz1, rays1 = _solve(_handle(prob, prob.frame, prob.landmark, prob.xy, win_hi), prob)
    outs = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(world)]
    assert sum(int(o["n_rec"]) for o in outs) == len(prob.frame)
    assert res1.njev >= 2
    for o in outs:
        assert int(o["njev"]) == res1.njev
        np.testing.assert_allclose(o["ptz"], ptz1, rtol=0, atol=1e-8)
        np.testing.assert_allclose(o["rays"][o["owned"]], rays1[o["owned"]], rtol=0, atol=1e-8)
        assert abs(float(o["cost"]) - res1.cost) <= 1e-9 * res1.cost
    # the two ranks took bit-identical pose steps (same summed system, same decisions)
    assert np.array_equal(outs[0]["ptz"], outs[1]["ptz"])
