"""Per-level phase timing of the tile Cholesky (a -DCS_TIMING build of libptzba, passed as PTZBA_LIB):
one reduced-system build + solve at config3, clock64 stamps of block 0 of every level launch:
[stage tiles, panel updates, potrf+trsm wave, (to next level start)]."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

p = synthetic.make_problem("config3", seed=0)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
              loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays)
ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=2).run()
L = ptzba.lib()
L.ptzba_debug_cs_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(64 * 6 + 64 * 10, dtype=np.int64)
h.linearize()
h.build_reduced(1e-3)
h.sync()
assert L.ptzba_debug_cs_stamps(buf.ctypes.data) == 0  # reset the level counter
h.solve_reduced()
h.sync()
assert L.ptzba_debug_cs_stamps(buf.ctypes.data) == 0
wg = buf[64 * 6:].reshape(64, 10)
buf = buf[:64 * 6].reshape(64, 6)
nz = np.nonzero(buf[:, 0])[0]
print("potrf stamps, successive differences (mean over levels 0..29):", np.diff(wg[:30, :9], axis=1).mean(0).round(0))
print(f"{len(nz)} levels, first->last start {buf[nz[-1], 0] - buf[nz[0], 0]} ticks")
ph = np.diff(buf[nz, :4], axis=1)
gap = buf[nz[1:], 0] - buf[nz[:-1], 3]
print("mean [stage, updates, potrf+trsm] per level:", ph.mean(0).round(0), " mean end->next start:", gap.mean().round(0))
for k in nz[:8]:
    print("  ", k, ph[k], "type", buf[k, 5])
