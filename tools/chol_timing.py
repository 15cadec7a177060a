"""Per-level phase timing of the tile Cholesky (a -DCS_TIMING build of libptzba, passed as PTZBA_LIB):
one reduced-system build + solve at config3, clock64 stamps of block 0 of every level launch:
[stage tiles, panel updates, potrf+trsm wave, (to next level start)], and (round 6) the pivot sweep's cycle
accounting: eight stamps per 4-pivot block of wave 0 (chol_kernels.hip CSB) and the helpers' publication times.
  PTZBA_LIB=.../libptzba_cst.so python tools/chol_timing.py [--json out.json]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

cfg = os.environ.get("CT_CONFIG", "config3")
p = synthetic.make_problem(cfg, seed=0)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
              loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays)
ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=2).run()
L = ptzba.lib()
L.ptzba_debug_cs_stamps.argtypes = [ctypes.c_void_p]
NSTAMP = 64 * 6 + 64 * 10 + 64 * 64 + 64 * 24 + 64 * 4
res = []
for rep in range(5):
    buf = np.zeros(NSTAMP, dtype=np.int64)
    h.linearize()
    h.build_reduced(1e-3)
    h.sync()
    assert L.ptzba_debug_cs_stamps(buf.ctypes.data) == 0  # reset the level counter
    h.solve_reduced()
    h.sync()
    assert L.ptzba_debug_cs_stamps(buf.ctypes.data) == 0
    res.append(buf)
buf = np.stack(res)  # [rep, ...]
st = buf[:, :64 * 6].reshape(-1, 64, 6)
wg = buf[:, 64 * 6:64 * 16].reshape(-1, 64, 10)
blk = buf[:, 64 * 16:64 * 16 + 4096].reshape(-1, 64, 8, 8)
hlp = buf[:, 64 * 16 + 4096:64 * 16 + 4096 + 64 * 24].reshape(-1, 64, 8, 3)
rt = buf[:, 64 * 16 + 4096 + 64 * 24:].reshape(-1, 64, 4).astype(float) * 10.0  # ns (s_memrealtime, 100 MHz)
nz = np.nonzero(st[0, :, 0])[0]
nl = len(nz)
# clock: memtime ticks per memrealtime tick (100 MHz)
dt_real = (blk[:, nz, 1, 1] - blk[:, nz, 0, 1]).astype(float)
dt_mem = (blk[:, nz, 3, 1] - blk[:, nz, 2, 1]).astype(float)
ghz = float(np.median(dt_mem / np.maximum(dt_real, 1)) * 0.1)
out = {"config": cfg, "levels": int(nl), "clock_ghz_memtime": ghz, "reps": len(res)}
print(f"{nl} levels; s_memtime runs at {ghz:.3f} GHz (vs s_memrealtime 100 MHz)")
ph = np.diff(st[:, nz, :4], axis=2).reshape(-1, 3)
gap = (st[:, nz[1:], 0] - st[:, nz[:-1], 3]).reshape(-1)
out["level_phases_ticks"] = {"stage": float(ph[:, 0].mean()), "panel_gemms": float(ph[:, 1].mean()),
                             "sweep": float(ph[:, 2].mean()), "end_to_next_start": float(gap.mean())}
print("mean [stage, updates, potrf+trsm] per level (ticks):", ph.mean(0).round(0), " mean end->next start:",
      gap.mean().round(0))
# sweep accounting, blocks 0..7 of wave 0 (stamp 0 block start, 2 after the helper poll, 3 after the row reads,
# 4 after the lookahead update + readlane gathers, 5 after the 4x4 factor, 6 after the row solve, 7 after publication)
b = blk[:, nz].astype(float)  # [rep, lvl, s, k]
names = {"poll (0->2, incl. prev-block reads)": (0, 2), "row reads (2->3)": (2, 3),
         "lookahead update + gathers (3->4)": (3, 4), "4x4 factor (4->5)": (4, 5), "row solve (5->6)": (5, 6),
         "store + publish (6->7)": (6, 7)}
acc = {}
for nm, (i, j) in names.items():
    d = b[:, :, :, j] - b[:, :, :, i]
    acc[nm] = {"per_block_mean": d.mean(axis=(0, 1)).round(1).tolist(), "mean": float(d.mean())}
blk_total = (b[:, :, 1:, 0] - b[:, :, :-1, 0])
acc["block period (0->next 0)"] = {"per_block_mean": blk_total.mean(axis=(0, 1)).round(1).tolist(),
                                   "mean": float(blk_total.mean())}
# helpers: when block t's update was published by the last helper, relative to wave 0's poll of it (block t + 1)
hl = hlp[:, nz].astype(float).max(axis=3)  # [rep, lvl, t]
slack = []
for t in range(1, 7):
    slack.append(float((b[:, :, t + 1, 2] - hl[:, :, t]).mean()))
acc["helper publish -> wave-0 poll done, blocks 2..7 (ticks; small = wave 0 waited on helpers)"] = slack
out["sweep"] = acc
for k, v in acc.items():
    print(f"  {k}: {v}")
# level timeline (ns, one clock for all XCDs): block 0's task start -> sweep end -> its stores complete; the level's
# last panel task done; the next level's block-0 start
r = rt[:, nz]
# (a level whose block 0 is an inverse or trailing task records no panel stamps: only levels with all three stamps, and
# pairs of consecutive such levels for the gap)
ok = (r[:, :, 0] > 0) & (r[:, :, 1] > 0) & (r[:, :, 2] > 0)
okp = ok[:, :-1] & ok[:, 1:] & (r[:, :-1, 3] > 0)
sel = lambda a, m: float(a[m].mean()) if m.any() else None  # noqa: E731
tl = {"start_to_sweep_end_ns": sel(r[:, :, 1] - r[:, :, 0], ok),
      "sweep_end_to_stores_done_ns": sel(r[:, :, 2] - r[:, :, 1], ok),
      "block0_stores_done_to_last_task_done_ns": sel(r[:, :, 3] - r[:, :, 2], ok & (r[:, :, 3] > 0)),
      "last_task_done_to_next_level_start_ns": sel(r[:, 1:, 0] - r[:, :-1, 3], okp),
      "level_start_to_next_start_ns": sel(r[:, 1:, 0] - r[:, :-1, 0], okp),
      "levels_with_panel_block0": int(ok[0].sum())}
out["level_timeline"] = tl
print("level timeline (ns):", {k: (round(v) if v is not None else None) for k, v in tl.items()})
js = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if js:
    json.dump(out, open(js, "w"), indent=1)
