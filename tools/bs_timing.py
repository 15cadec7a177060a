"""Per-column phase timing of the back-substitution kernel (a -DBS_TIMING build of libptzba, passed as
PTZBA_LIB): runs config3 linearise + reduced system + solve once, prints per chain position the cycles
of [stage+barrier, solve, barrier, update, prefetch issue]."""
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
for _ in range(3):
    ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=2).run()
buf = np.zeros(2 * 128 * 6 + 8, dtype=np.int64)
L = ptzba.lib()
L.ptzba_debug_bs_stamps.argtypes = [ctypes.c_void_p]
assert L.ptzba_debug_bs_stamps(buf.ctypes.data) == 0
edges = buf[2 * 128 * 6:].reshape(2, 4)
buf = buf[:2 * 128 * 6].reshape(2, 128, 6)
print("edges (start, loop start, end) per chain:", [(int(e[1] - e[0]), int(e[2] - e[1])) for e in edges])
for ch in range(2):
    d = np.diff(buf[ch], axis=1)
    nz = np.nonzero(buf[ch, :, 0])[0]
    if len(nz) == 0:
        continue
    tot = buf[ch, nz[-1], 5] - buf[ch, nz[0], 0]
    print(f"chain {ch}: {len(nz)} columns, {tot} cycles total")
    print("   mean per column, successive stamp differences:", d[nz].mean(0).round(0),
          "(k_chol_backsolve: barrier1, solve, barrier2, update, prefetch; k_chol_backsolve_la: ring wait,"
          " M/L reads + owner wait, solve + publish, lookahead)")
    st = buf[ch, nz, 0]
    print("   mean start-to-start per column:", np.diff(st).mean().round(0))
    for q in nz[:6]:
        print("   ", q, d[q])
