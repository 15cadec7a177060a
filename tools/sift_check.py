"""ptz_sift diagnostics: agreement with the oracle restatement on a small synthetic view, and the wall time
of one detectAndCompute call at 640x360 and 1920x1080 (host upload + all kernels + downloads)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"), os.path.join(ROOT, "tests")]
import frontend_data  # noqa: E402
import ptzba  # noqa: E402
from oracle import ptz_oracle as orc  # noqa: E402

I, _, _ = frontend_data.textured_pair(seed=3, width=257, height=181, d_pan=0.5, f=400.0)
kg, rg, dg = ptzba.sift(I, 0)
ko, ro, do = orc.sift_detect_compute(I, 0)
pairs = []
for i, k in enumerate(ko):
    d = np.abs(kg[:, :2] - k[:2]).max(1) + np.abs(kg[:, 3] - k[3]) / 360
    j = int(np.argmin(d))
    if d[j] < 1e-3:
        pairs.append((j, i))
pr = np.array(pairs)
print(f"257x181: gpu {len(kg)} oracle {len(ko)} matched {len(pr)}; max |d xy| "
      f"{np.abs(kg[pr[:, 0], :2] - ko[pr[:, 1], :2]).max():.2e} |d size| {np.abs(kg[pr[:, 0], 2] - ko[pr[:, 1], 2]).max():.2e} "
      f"|d angle| {np.abs(kg[pr[:, 0], 3] - ko[pr[:, 1], 3]).max():.2e}; descriptors: identical "
      f"{np.mean(np.all(dg[pr[:, 0]] == do[pr[:, 1]], axis=1)) * 100:.1f} % of keypoints, max |d| "
      f"{np.abs(dg[pr[:, 0]] - do[pr[:, 1]]).max():.0f}")
for w, h in ((640, 360), (1920, 1080)):
    img, _, _ = frontend_data.textured_pair(seed=4, width=w, height=h, f=1200.0)
    ptzba.sift(img, 1500)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        k, _, _ = ptzba.sift(img, 1500)
        ts.append(time.perf_counter() - t0)
    print(f"{w}x{h}: {len(k)} keypoints (nfeatures 1500), detectAndCompute {1e3 * min(ts):.1f} ms")
