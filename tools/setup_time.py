"""set_problem wall time and its host phases (ptzba_setup_timing) for a BASELINE config: python tools/setup_time.py
config4 [reps].  Prints one JSON line per call."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"))
import ptzba  # noqa: E402
import synthetic  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p = synthetic.make_problem(cfg, seed=0)
for rep in range(reps):
    h = ptzba.BAHandle(0)
    t0 = time.perf_counter()
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    t1 = time.perf_counter()
    print(json.dumps({"config": cfg, "rep": rep, "n_records": int(len(p.frame)), "set_problem_s": round(t1 - t0, 4),
                      "phases_ms": {k: round(v, 1) for k, v in h.setup_timing().items()}}), flush=True)
    h.close()
