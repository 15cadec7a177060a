"""Per-frame EKF update timing: GPU ptzekf_update vs the NumPy oracle restatement
of PtzSlam.ekf_update on the same state (the reference's CPU cost: 0.22 s at R=300, 0.62 s at R=500)."""
import sys
import time

import numpy as np

sys.path[:0] = ["pan-tilt-zoom-slam_amd", ".", "tests"]
import ptzba  # noqa: E402
from oracle import ptz_oracle as orc  # noqa: E402
from test_gpu_ekf import _random_state  # noqa: E402

for R in (300, 500, 1000):
    s, obs, keep = _random_state(R, 7, frac_obs=0.8)
    h = ptzba.EKFHandle(0)
    ts = []
    for it in range(12):
        h.set_state(s["rays"], s["state_cov"])
        t0 = time.perf_counter()
        ptz, vel, nm = h.update(s["u"], s["v"], [s["pan"], s["tilt"], s["f"]], obs, keep, 1080, 1920, 0.1)
        ts.append(time.perf_counter() - t0)
    gpu = float(np.median(ts[2:]))
    t0 = time.perf_counter()
    ref = orc.ekf_update(s, obs, keep, 1080, 1920)
    cpu = time.perf_counter() - t0
    print(f"R={R} matched={nm} gpu_update_ms={gpu * 1e3:.3f} oracle_cpu_ms={cpu * 1e3:.1f} "
          f"pan_diff={abs(ptz[0] - ref['pan']):.2e}")
    h.close()
