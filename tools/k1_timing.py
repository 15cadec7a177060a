"""Phase timing of K1 (k_linearize) from a -DK1_TIMING build (PTZBA_LIB=.../libptzba_k1t.so, built with
tools/build_variant.sh k1t ba_kernels.hip -DK1_TIMING): per-wave averages of phase A (descriptor, projections,
frame tables), B (record stream), C (Jacobians, slot stores) and the final reductions, in cycles; and from
the per-task s_memrealtime stamps of one launch: makespan, how many waves are resident over time, the tail."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
p = synthetic.make_problem(cfg, seed=0)
h = ptzba.BAHandle(0)
h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
              loss=ptzba.LOSS_HUBER, f_scale=1.0)
h.set_state(p.init_ptz, p.init_rays)
L = ptzba.lib()
L.ptzba_debug_k1.argtypes = [ctypes.c_void_p, ctypes.c_int]
for _ in range(3):
    h.linearize()
h.sync()
n = 32768
it = np.zeros((n, 8), np.int64)
assert L.ptzba_debug_k1(it.ctypes.data, n) == 0
it = it[it[:, 1] > 0]
names = ["A (descriptor + projections)", "B (records)", "C (Jacobians + stores)", "final"]
print(f"{cfg}: {len(it)} waves per launch, {it[:, 6].mean():.1f} segments per wave")
tot = it[:, 2:6].sum()
for k in range(4):
    print(f"  phase {names[k]:32s} {it[:, 2 + k].mean():9.0f} cycles/wave  {100.0 * it[:, 2 + k].sum() / tot:5.1f} %")
t0 = it[:, 0].min()
st, en = (it[:, 0] - t0) * 1e-2, (it[:, 1] - t0) * 1e-2  # us
dur = en - st
print(f"one launch: {len(it)} tasks, makespan {en.max():.1f} us, mean task {dur.mean():.2f} us, "
      f"p10/p50/p90 {np.percentile(dur, 10):.2f}/{np.percentile(dur, 50):.2f}/{np.percentile(dur, 90):.2f} us")
grid = np.linspace(0, en.max(), 41)
act = [int(((st <= t) & (en > t)).sum()) for t in grid]
print("resident waves over time (every makespan/40):", act)
print(f"last task start {st.max():.1f} us; time with < 50% of peak residency: "
      f"{(np.array(act) < 0.5 * max(act)).mean() * 100:.0f} % of the samples")
order = np.argsort(st)
k = len(it) // 10
print("task duration by start order (deciles, us):", [round(float(dur[order[i * k:(i + 1) * k]].mean()), 2) for i in range(10)])
print("segments by start order (deciles):", [round(float(it[order[i * k:(i + 1) * k], 6].mean()), 1) for i in range(10)])
h.reset_kernel_times(1) if hasattr(h, "reset_kernel_times") else None
