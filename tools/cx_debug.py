#!/usr/bin/env python3
"""Diagnostics of the XCD-local factorisation tail (k_chol_xcd): the XCD id census of a 512-workgroup launch, then one
short solve per case with the tail forced on (PTZBA_CHOL_XCD=<L0>) and its control sets dumped afterwards (claim,
ticket and per-level completion counts of both parities against the tasks per level).

  python tools/cx_debug.py [config2|config3] [L0]
"""
import collections
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"), os.path.join(ROOT, "tools")]

import ptzba  # noqa: E402
import synthetic  # noqa: E402

W = 32


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
    l0 = sys.argv[2] if len(sys.argv) > 2 else "1"
    lib = ptzba.lib()
    n = 512
    ids = (ctypes.c_int * n)()
    assert lib.ptzba_debug_xcc_census(n, ids) == 0
    ids = list(ids)
    print("xcc census:", dict(sorted(collections.Counter(ids).items())), "first 16:", ids[:16], flush=True)
    os.environ["PTZBA_CHOL_XCD"] = l0
    p = synthetic.make_problem(cfg, seed=0)
    h = ptzba.BAHandle(0)
    h.set_problem(p.n_pose, p.n_landmark, p.frame, p.landmark, p.xy, p.u, p.v, precision=ptzba.FP32,
                  loss=ptzba.LOSS_HUBER, f_scale=1.0)
    h.set_state(p.init_ptz, p.init_rays)
    t0 = time.time()
    err = None
    try:
        r = h.solve_resident(restore=False, ftol=1e-12, xtol=1e-14, max_iter=2)
        print("solve:", r.cost, r.njev, r.nfev, r.status, f"{time.time() - t0:.2f} s", flush=True)
    except Exception as e:  # noqa: BLE001
        err = e
        print("solve failed:", e, f"{time.time() - t0:.2f} s", flush=True)
    ctl = (ctypes.c_uint32 * (4 * W))()
    done = (ctypes.c_uint32 * 8192)()
    ep = ctypes.c_uint32()
    fn = lib.ptzba_debug_chol_xcd
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    nd = fn(h.h, ctl, done, 8192, ctypes.byref(ep))
    tags = collections.Counter(list(done)[:nd])
    print("tail tasks", nd, "epoch", ep.value, "done tags", dict(tags))
    for par in range(2):
        print(f"set {par}: claim {ctl[2 * par * W]} ticket {ctl[2 * par * W + W]}")
    h.close()
    if err:
        sys.exit(1)


if __name__ == "__main__":
    main()
