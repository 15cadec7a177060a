#!/usr/bin/env python3
"""Per-rank device time of an N-way sharded solve, measured on ONE MI355X.

For each N, rank r's share of the problem (ptzba_partition_landmarks: part-owned when the frame chain splits) is
set up alone on the device with a no-op exchange hook, and K trials of the LM step (build_reduced + solve_reduced
at a fixed damping: K2, the part's factorisation phase, the separator phase, back-substitution, trial, trial
linearisation) are timed with HIP events per kernel group.  The numbers are the rank's own device work per trial;
the collectives are NOT included (an 8-GPU node is not available to this build) -- their payloads are printed so
the step time at N can be modelled as  rank time + sum over exchanges of (latency + bytes / bandwidth).
The values the no-op exchange leaves in the system are partial sums, so the factorisation may report a non-positive
pivot: the kernels run the same work either way (timing only, no numerics are used).

  python tools/dist_model.py [--config config3] [--worlds 1,2,4,8] [--trials 40]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="config3")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--trials", type=int, default=40)
    ap.add_argument("--ranks", default="first", choices=["first", "all"])
    ap.add_argument("--mode", default="part", choices=["part", "replicated"],
                    help="replicated: contiguous landmark shards (bench.shard_by_landmark), every rank factors the whole "
                         "summed system (one X_SYS all-reduce of the packed system per trial)")
    a = ap.parse_args()
    import torch
    import ptzba
    import synthetic
    torch.cuda.set_device(0)
    prob = synthetic.make_problem(a.config, seed=0)
    win = ptzba.frame_coupling_window(prob.n_pose, prob.frame, prob.landmark)
    out = []
    for world in [int(x) for x in a.worlds.split(",")]:
        if world == 1:
            ranks, owner, mode, split = [0], None, 0, None
        elif a.mode == "replicated":
            ranks, owner, mode, split = [0], None, 0, None  # every shard runs the same full factorisation
        else:
            owner, mode, split = ptzba.partition_landmarks(prob.n_pose, prob.n_landmark, prob.frame, prob.landmark, world)
            ranks = list(range(world))
            if a.ranks == "first":  # one rank per base of the rank tree (ranks sharing a leaf run the same plan)
                bases = [ptzba.dist_plan_summary(win, world, r)["base"] for r in ranks]
                ranks = [r for r in ranks if r == 0 or bases[r] != bases[r - 1]]
        for rank in ranks:
            repl = world > 1 and a.mode == "replicated"
            if repl:
                import bench
                sel = bench.shard_by_landmark(prob.landmark, prob.n_landmark, rank, world)
            else:
                sel = np.ones(len(prob.frame), bool) if owner is None else owner[prob.landmark] == rank
            h = ptzba.BAHandle(0)
            h.set_problem(prob.n_pose, prob.n_landmark, prob.frame[sel], prob.landmark[sel], prob.xy[sel], prob.u,
                          prob.v, precision=ptzba.FP32, loss=ptzba.LOSS_HUBER, frame_win_hi=win,
                          dist_world=world if (world > 1 and not repl) else 0, dist_rank=rank)
            if repl:  # the packed system and the scalars, all-reduced over all ranks per trial
                xi = {"mode": "replicated", "exchanges": [[ptzba.X_SYS, 0, world, int(h.exchange_packed()[1])],
                                                          [ptzba.X_SCAL, 0, world, int(ptzba.NSCALARS)]]}
            else:
                xi = h.dist_info() if world > 1 else None
            if xi is not None and not repl:
                xi["exchanges"] = h.dist_exchanges()
            if world > 1:
                h.set_exchange_hook(lambda kind, ptr, count, stream: None)
            h.set_state(prob.init_ptz, prob.init_rays)
            h.linearize()
            for _ in range(3):
                h.build_reduced(1e-3)
                h.solve_reduced()
            h.sync()
            h.reset_kernel_times(True, groups=0xF)
            t0 = time.perf_counter()
            for _ in range(a.trials):
                h.build_reduced(1e-3)
                h.solve_reduced()
            h.sync()
            wall = (time.perf_counter() - t0) / a.trials
            kt = h.kernel_times()
            rec = dict(config=a.config, world=world, rank=rank, n_records=int(sel.sum()), wall_ms_per_trial=1e3 * wall,
                       kernel_ms={k: round(v[0], 4) for k, v in kt.items()}, solver=h.solver_info(), exchange=xi)
            h.close()
            print(json.dumps(rec), flush=True)
            out.append(rec)
    return out


if __name__ == "__main__":
    main()
