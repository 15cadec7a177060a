"""Phase timing of K2 (k_schur) from a -DSK_TIMING build (PTZBA_LIB): clock64 stamps of thread 0 of the
first 16 workgroups: [list load, diag phase, first stage, batches: compute / stage / barrier sums, tail]."""
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
h.linearize()
h.build_reduced(1e-3)
h.sync()
buf = np.zeros((16, 16), dtype=np.int64)
L = ptzba.lib()
L.ptzba_debug_sk.argtypes = [ctypes.c_void_p]
assert L.ptzba_debug_sk(buf.ctypes.data) == 0
for b in range(16):
    r = buf[b]
    print(f"wg {b:2d} nl {r[8]:4d} chunk {r[9]} | list {r[1]-r[0]:6d} diag {r[2]-r[1]:6d} stage0 {r[3]-r[2]:6d} | "
          f"compute {r[4]:7d} stage {r[5]:7d} barrier {r[6]:7d} | write {r[10]-r[7]:6d} | total {r[10]-r[0]:7d}")

# per-item start / end (s_memrealtime, 10 ns ticks): occupancy of the launch and the tail
L.ptzba_debug_sk_items.argtypes = [ctypes.c_void_p]
it = np.zeros((4096, 4), dtype=np.int64)
assert L.ptzba_debug_sk_items(it.ctypes.data) == 0
n = int(np.count_nonzero(it[:, 1]))
it = it[:n]
t0 = it[:, 0].min()
st, en = (it[:, 0] - t0) * 10e-3, (it[:, 1] - t0) * 10e-3  # us
dur = en - st
print(f"{n} items, makespan {en.max():.1f} us, sum of item times {dur.sum():.0f} us "
      f"(= {dur.sum() / en.max():.0f} CUs busy on average)")
for c in sorted(set(it[:, 2])):
    m = it[:, 2] == c
    print(f"  chunk {c}: {m.sum()} items, duration mean {dur[m].mean():.1f} max {dur[m].max():.1f} us, nl mean {it[m, 3].mean():.0f}")
late = np.argsort(en)[-8:]
print("  last to finish (start, end, chunk, nl):", [(round(st[i], 1), round(en[i], 1), int(it[i, 2]), int(it[i, 3])) for i in late])
