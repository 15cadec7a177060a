"""Per-work-item timeline of K2 (k_schur_mf) from a -DSK_TIMING build (PTZBA_LIB): s_memrealtime start / end (100 MHz)
of every item of one build, its chunk and landmark count -> makespan, item-duration spread, how many items are still
running over time (load balance of the one-round item schedule)."""
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
for _ in range(3):
    h.build_reduced(1e-3)
h.sync()
it = np.zeros((4096, 4), dtype=np.int64)
L = ptzba.lib()
L.ptzba_debug_sk_items.argtypes = [ctypes.c_void_p]
assert L.ptzba_debug_sk_items(it.ctypes.data) == 0
it = it[it[:, 1] > 0]
t0 = it[:, 0].min()
st, en = (it[:, 0] - t0) * 1e-2, (it[:, 1] - t0) * 1e-2
dur = en - st
print(f"{len(it)} items, makespan {en.max():.1f} us, item duration mean {dur.mean():.1f} p10/p50/p90/max "
      f"{np.percentile(dur, 10):.1f}/{np.percentile(dur, 50):.1f}/{np.percentile(dur, 90):.1f}/{dur.max():.1f} us; "
      f"start spread {st.max():.1f} us")
c0 = it[:, 2] == 0
print(f"chunk-0 items {c0.sum()}: mean {dur[c0].mean():.1f} us, nl mean {it[c0, 3].mean():.0f}; others {(~c0).sum()}: "
      f"mean {dur[~c0].mean():.1f} us, nl mean {it[~c0, 3].mean():.0f}")
g = np.linspace(0, en.max(), 21)
print("running items over time:", [int(((st <= t) & (en > t)).sum()) for t in g])
print("us per landmark (item duration / nl): chunk-0 %.3f, others %.3f" % (
    np.mean(dur[c0] / np.maximum(it[c0, 3], 1)), np.mean(dur[~c0] / np.maximum(it[~c0, 3], 1))))
