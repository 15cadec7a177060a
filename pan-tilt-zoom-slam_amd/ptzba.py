"""
ctypes binding of libptzba.so (the MI355X bundle-adjustment / tracking library) and the
Levenberg-Marquardt driver that replaces the reference's optimizer call.

Binding style follows the reference's only FFI, rf_map_wrapper.py:13-82 (cdll.LoadLibrary, argtypes
declared per entry point, c_void_p handles, caller-owned float64 numpy buffers passed by pointer),
with two deliberate fixes: the library path is resolved next to this file instead of hard-coded
(rf_map_wrapper.py:14-17), and it is loaded lazily on first use, raising a clear error if the
native library is missing — there is NO CPU fallback for any entry point.

The optimizer replaced: `least_squares(_compute_residual, x0, verbose=2, x_scale='jac', ftol=1e-4,
method='trf', ...)` (bundle_adjustment.py:200-202).  `LMSolver` runs Levenberg-Marquardt with
Marquardt column scaling (the monotone max of diag(J^T J), cf. scipy x_scale='jac',
common.py:598-612), an exact Schur-complement step on the GPU, and scipy's termination tests
(ftol on accepted steps, xtol on the step norm, max iterations).  One iteration == one
linearisation (scipy `njev`); rejected trial steps are counted inside the iteration.
"""
import ctypes
import os
import threading
import time
from ctypes import POINTER, Structure, c_char_p, c_double, c_int, c_int32, c_int64, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PTZBA_LIB", os.path.join(_HERE, "libptzba.so"))

FP64, FP32 = 0, 1
LOSS_LINEAR, LOSS_HUBER = 0, 1
NSCALARS = 8

_lib = None


ORDER_NATURAL, ORDER_NESTED, ORDER_NESTED_FORCE = 0, 1, 2


class ptz_refine_opts(Structure):
    _fields_ = [("max_iter", c_int32), ("loss", c_int32), ("ftol", c_double), ("xtol", c_double),
                ("f_scale", c_double)]


class ptzba_lm_opts(Structure):
    _fields_ = [("ftol", c_double), ("xtol", c_double), ("gtol", c_double), ("lambda0", c_double),
                ("min_lambda", c_double), ("max_lambda", c_double), ("max_iter", c_int32), ("max_retries", c_int32),
                ("gauss_newton", c_int32), ("huber_curvature", c_double), ("curvature_switch", c_double)]


# LM defaults (include/ptzba.h ptzba_lm_opts).  lambda0 = min_lambda: Gauss-Newton steps from the start, as scipy's trf
# takes them while the step lies inside its trust region (bundle_adjustment.py:200-202 -> trf.py); a Marquardt start
# (1e-4, rounds 1-4) damps the frame chain's low-curvature modes and stops at ftol=1e-4 ~5e-4 deg short of the optimum
# at config 3 (profiles/r05a_ftol_study.jsonl).  Huber: IRLS curvature until an accepted step is predicted to reduce the
# cost by less than CURVATURE_SWITCH of it, then HUBER_CURVATURE * rho' beyond the unit (profiles/r05c_switch.jsonl)
LAMBDA0 = 1e-12
MIN_LAMBDA = 1e-12
HUBER_CURVATURE = 0.1
CURVATURE_SWITCH = 0.25


class ptzba_lm_record(Structure):
    _fields_ = [("cost", c_double), ("initial_cost", c_double), ("lam", c_double), ("iterations", c_int32),
                ("nfev", c_int32), ("trials", c_int32), ("retries", c_int32), ("status", c_int32), ("done", c_int32),
                ("accepted", c_int32)]


class ptzba_report(Structure):
    _fields_ = [("cost", c_double), ("initial_cost", c_double), ("time_s", c_double), ("iterations", c_int32),
                ("nfev", c_int32), ("trials", c_int32), ("status", c_int32)]


TIME_COMM = 0x10  # include/ptzba.h PTZBA_TIME_COMM: an event pair around every exchange (comm_times)
TIME_FLUSH = 0x10000  # include/ptzba.h PTZBA_TIME_FLUSH: cold-cache K1 timing
TIME_FLUSH_READ = 0x20000  # include/ptzba.h PTZBA_TIME_FLUSH_READ: ... by a read flush (clean caches)


class ptzba_problem_opts(Structure):
    _fields_ = [("precision", c_int32), ("loss", c_int32), ("f_scale", c_double), ("n_fixed", c_int32),
                ("ordering", c_int32), ("frame_win_hi", c_void_p), ("dist_world", c_int32), ("dist_rank", c_int32)]


# exchange kinds of a multi-GPU solve (include/ptzba.h PTZBA_X_*)
X_SYS, X_PART, X_SEP, X_SCAL, X_SUB = 0, 1, 2, 3, 4
X_NAMES = {X_SYS: "sys", X_PART: "part", X_SEP: "sep", X_SCAL: "scal", X_SUB: "sub"}
UNIQUE_ID_BYTES = 128
EXCHANGE_FN = ctypes.CFUNCTYPE(c_int32, c_void_p, c_int32, c_void_p, c_int64, c_void_p)


def _ptr(a):
    return c_void_p(a.ctypes.data) if a is not None else c_void_p(0)


def lib():
    """Load libptzba.so once (rf_map_wrapper.py:13-17 style) and declare argtypes."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libptzba.so not found at {LIB_PATH}: build it with "
                           f"`make -C pan-tilt-zoom-slam_amd/csrc` (hipcc, gfx950). There is no CPU fallback.")
    L = ctypes.cdll.LoadLibrary(LIB_PATH)
    V, I, I32, I64, D = c_void_p, c_int, c_int32, c_int64, c_double
    sigs = {
        "ptzba_new": ([I], V),
        "ptzba_delete": ([V], None),
        "ptzba_last_error": ([], c_char_p),
        "ptzba_version": ([], c_char_p),
        "ptzba_set_stream": ([V, V], I),
        "ptzba_use_own_stream": ([V], I),
        "ptzba_set_problem": ([V, I32, I32, I64, V, V, V, V, D, D, POINTER(ptzba_problem_opts)], I),
        "ptzba_problem_info": ([V, V], I),
        "ptzba_solver_info": ([V, V], I),
        "ptzba_residual": ([V, V, V], I),
        "ptzba_set_state": ([V, V, V], I),
        "ptzba_get_state": ([V, V, V], I),
        "ptzba_linearize": ([V], I),
        "ptzba_build_reduced": ([V, D], I),
        "ptzba_solve_reduced": ([V], I),
        "ptzba_step": ([V, D], I),
        "ptzba_set_huber_curvature": ([V, D], I),
        "ptzba_set_setup_front": ([V, I64], I),
        "ptzba_setup_timing": ([V, I32, V, V, V], I),
        "ptzba_solve": ([V, V, V, POINTER(ptzba_lm_opts), POINTER(ptzba_report)], I),
        "ptzba_solve_resident": ([V, I32, POINTER(ptzba_lm_opts), POINTER(ptzba_report)], I),
        "ptzba_lm_start": ([V], I),
        "ptzba_lm_init": ([V, POINTER(ptzba_lm_opts)], I),
        "ptzba_lm_build": ([V], I),
        "ptzba_lm_solve": ([V], I),
        "ptzba_lm_decide": ([V, I], I),
        "ptzba_lm_wait": ([V, I, POINTER(ptzba_lm_record)], I),
        "ptzba_read_scalars": ([V, V], I),
        "ptzba_accept": ([V, I], I),
        "ptzba_exchange": ([V, POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p)], I),
        "ptzba_exchange_packed": ([V, POINTER(c_void_p), POINTER(c_int64)], I),
        "ptzba_pack": ([V], I),
        "ptzba_unpack": ([V], I),
        "ptzba_sync": ([V], I),
        "ptzba_kernel_times": ([V, V, V], I),
        "ptzba_reset_kernel_times": ([V, I], I),
        "ptzba_comm_times": ([V, I32, V, V, V, V], I),
        "ptzba_dist_form_estimate": ([I32, I32, V, I32, D, D, V], I),
        "ptzba_save_state": ([V], I),
        "ptzba_restore_state": ([V], I),
        "ptz_ray_to_image": ([I, I64, D, D, V, V, V, V, V, V, V], I),
        "ptz_image_to_ray": ([I, I64, D, D, V, V, V, V, V, V, V], I),
        "ptz_project_rays": ([I, I64, D, D, D, D, D, V, V, V], I),
        "ptz_back_project_rays": ([I, I64, D, D, D, D, D, V, V, V], I),
        "ptz_h_jacobian": ([I, I64, D, D, D, D, D, V, V, V], I),
        "ptzba_build_landmarks": ([I32, V, I64, V, V, V, V, V, V, V, V], I),
        "ptzba_coupling_window": ([I32, I32, I64, V, V, V], I),
        "ptzba_plan_summary": ([I32, I32, V, I32, V], I),
        "ptzba_plan_export": ([I32, I32, V, I32, V, V, I64, V, I64, V], I),
        "ptz_match_knn2": ([I, I64, I64, I32, V, V, V, V], I),
        "ptz_desc_put": ([I, ctypes.c_uint64, I64, I32, V], I),
        "ptz_desc_drop": ([I, I32, V], I),
        "ptz_match_knn2_sets": ([I, I32, V, ctypes.c_uint64, I64, V, V], I),
        "ptz_match_sets_ransac": ([I, I32, V, V, ctypes.c_uint64, I64, V, V, D, I32, ctypes.c_uint64, V, V, V, V], I),
        "ptz_homography_ransac": ([I, I64, V, V, D, I32, ctypes.c_uint64, V, V, POINTER(c_int32)], I),
        "ptz_homography_ransac_batch": ([I, I32, V, V, V, D, I32, ctypes.c_uint64, V, V, V], I),
        "ptz_lk_track": ([I, I32, I32, V, V, I64, V, I32, I32, I32, D, D, V, V, V], I),
        "ptz_sift": ([I, I32, I32, V, I32, I32, V, V, V, POINTER(c_int32)], I),
        "ptz_orb": ([I, I32, I32, V, I32, I32, I32, V, V, POINTER(c_int32)], I),
        "ptz_match_hamming": ([I, I64, I64, I32, V, V, V, V, V], I),
        "ptz_py_shuffle_prefix": ([V, I64, V, I64, V], I),
        "ptz_set_order_pairs": ([I64, V, V, V, V, V], I),
        "ptz_keyframe_features": ([I32, I64, V, V, V, V, V, V, V, V], I),
        "ptz_keyframe_feature_counts": ([I32, I64, V, V, V, V, V, V], I),
        "ptz_pack_records": ([I32, I64, V, V, V, V, V, V, V, I64, V, V, V, V], I),
        "ptz_refine_poses": ([I, I32, V, I64, V, V, D, D, V, V, POINTER(ptz_refine_opts), V, V, V], I),
        "ptz_corner_min_eig": ([I, I32, I32, V, V, V], I),
        "ptzba_partition_landmarks": ([I32, I32, I64, V, V, I32, I32, V, POINTER(c_int32), V], I),
        "ptzba_set_exchange_hook": ([V, EXCHANGE_FN, V], I),
        "ptzba_comm_unique_id": ([V], I),
        "ptzba_comm_new": ([I, V, I32, I32], V),
        "ptzba_comm_delete": ([V], None),
        "ptzba_comm_split": ([V, I32, I32], V),
        "ptzba_comm_info": ([V, POINTER(c_int32), POINTER(c_int32)], I),
        "ptzba_comm_allreduce": ([V, V, I64, V], I),
        "ptzba_attach_comm": ([V, V], I),
        "ptzba_dist_info": ([V, V], I),
        "ptzba_owned_frames": ([V, V], I),
        "ptzba_dist_exchanges": ([V, V, I32, POINTER(c_int32)], I),
        "ptzba_dist_groups": ([V, V, I32, POINTER(c_int32)], I),
        "ptzba_exchange_group": ([V, I32, V], I),
        "ptzba_dist_plan_summary": ([I32, I32, V, I32, I32, V], I),
        "ptzba_dist_rank_phases": ([I32, I32, V, I32, I32, V, I32, POINTER(c_int32)], I),
        "ptzba_dist_plan_export": ([I32, I32, V, I32, I32, V, V, I64, V, I64, V, I32, V, I64, V], I),
        "ptzekf_new": ([I], V),
        "ptzekf_delete": ([V], None),
        "ptzekf_num_rays": ([V], I),
        "ptzekf_set_state": ([V, I32, V, V], I),
        "ptzekf_get_state": ([V, V, V], I),
        "ptzekf_add_pose_cov": ([V, V], I),
        "ptzekf_remove_rays": ([V, I64, V], I),
        "ptzekf_add_rays": ([V, I64, V, D], I),
        "ptzekf_project_visible": ([V, D, D, V, V, I32, I32, V, V, POINTER(c_int32)], I),
        "ptzekf_update": ([V, D, D, V, V, I64, V, V, I32, I32, D, V, POINTER(c_int32)], I),
    }
    for name, (args, res) in sigs.items():
        if "PTZBA_LIB" in os.environ and not hasattr(L, name):
            continue  # an older library built for an A/B run (tools/gpu_lib_ab.sh): entry points it predates stay unbound
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


EXPORTED_SYMBOLS = [
    "ptzba_new", "ptzba_delete", "ptzba_last_error", "ptzba_version", "ptzba_set_stream", "ptzba_use_own_stream", "ptzba_set_problem",
    "ptzba_problem_info", "ptzba_solver_info", "ptzba_residual", "ptzba_set_state", "ptzba_get_state", "ptzba_linearize",
    "ptzba_build_reduced", "ptzba_solve_reduced", "ptzba_step", "ptzba_set_huber_curvature", "ptzba_set_setup_front", "ptzba_setup_timing", "ptzba_solve", "ptzba_solve_resident", "ptzba_read_scalars", "ptzba_accept",
    "ptzba_lm_start", "ptzba_lm_init", "ptzba_lm_build", "ptzba_lm_solve", "ptzba_lm_decide", "ptzba_lm_wait",
    "ptzba_exchange", "ptzba_exchange_packed", "ptzba_pack", "ptzba_unpack", "ptzba_sync", "ptzba_kernel_times", "ptzba_reset_kernel_times", "ptzba_comm_times", "ptzba_dist_form_estimate", "ptzba_save_state", "ptzba_restore_state", "ptz_ray_to_image",
    "ptz_image_to_ray", "ptz_project_rays", "ptz_back_project_rays", "ptz_h_jacobian", "ptzba_build_landmarks", "ptzba_coupling_window", "ptz_match_knn2", "ptz_homography_ransac", "ptz_homography_ransac_batch", "ptz_lk_track", "ptz_sift", "ptz_match_hamming",
    "ptz_py_shuffle_prefix", "ptz_set_order_pairs", "ptz_keyframe_features", "ptz_pack_records",
    "ptz_refine_poses", "ptzekf_new", "ptzekf_delete", "ptzekf_num_rays", "ptzekf_set_state", "ptzekf_get_state", "ptzekf_add_pose_cov",
    "ptzekf_remove_rays", "ptzekf_add_rays", "ptzekf_project_visible", "ptzekf_update",
    "ptzba_partition_landmarks", "ptzba_set_exchange_hook", "ptzba_comm_unique_id", "ptzba_comm_new",
    "ptzba_comm_delete", "ptzba_comm_split", "ptzba_comm_info", "ptzba_comm_allreduce", "ptzba_attach_comm",
    "ptzba_dist_info", "ptzba_owned_frames", "ptz_corner_min_eig", "ptz_orb", "ptzba_plan_summary",
    "ptzba_plan_export", "ptzba_dist_exchanges", "ptzba_dist_groups", "ptzba_exchange_group", "ptzba_dist_plan_summary",
    "ptzba_dist_rank_phases", "ptzba_dist_plan_export", "ptz_desc_put", "ptz_desc_drop", "ptz_match_knn2_sets",
    "ptz_keyframe_feature_counts", "ptz_match_sets_ransac",
]


class PtzbaError(RuntimeError):
    pass


def _check(rc, what):
    if rc != 0:
        msg = lib().ptzba_last_error()
        raise PtzbaError(f"{what}: {msg.decode() if msg else 'error'}")


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape)
    return a


def default_device():
    return int(os.environ.get("PTZBA_DEVICE", "0"))


# ---------------------------------------------------------------------------------------------
# camera model (batched device calls)
# ---------------------------------------------------------------------------------------------
def ray_to_image(u, v, f, cam_pan, cam_tilt, theta, phi, device=0):
    """Batched TransFunction.from_ray_to_image (transformation.py:99-135)."""
    f, cp, ct, th, ph = np.broadcast_arrays(*[_f64(a) for a in (f, cam_pan, cam_tilt, theta, phi)])
    shape = f.shape
    f, cp, ct, th, ph = [np.ascontiguousarray(a.reshape(-1)) for a in (f, cp, ct, th, ph)]
    n = f.size
    x = np.empty(n)
    y = np.empty(n)
    _check(lib().ptz_ray_to_image(device, n, u, v, _ptr(f), _ptr(cp), _ptr(ct), _ptr(th), _ptr(ph), _ptr(x), _ptr(y)),
           "ptz_ray_to_image")
    return x.reshape(shape), y.reshape(shape)


def image_to_ray(u, v, f, cam_pan, cam_tilt, x, y, device=0):
    """Batched TransFunction.from_image_to_ray (transformation.py:137-175)."""
    f, cp, ct, xx, yy = np.broadcast_arrays(*[_f64(a) for a in (f, cam_pan, cam_tilt, x, y)])
    shape = f.shape
    f, cp, ct, xx, yy = [np.ascontiguousarray(a.reshape(-1)) for a in (f, cp, ct, xx, yy)]
    n = f.size
    th = np.empty(n)
    ph = np.empty(n)
    _check(lib().ptz_image_to_ray(device, n, u, v, _ptr(f), _ptr(cp), _ptr(ct), _ptr(xx), _ptr(yy), _ptr(th),
                                  _ptr(ph)), "ptz_image_to_ray")
    return th.reshape(shape), ph.reshape(shape)


def project_rays(u, v, f, pan, tilt, rays, displacement=None, device=0):
    """Batched PTZCamera.project_ray (ptz_camera.py:191-210): [n,2] rays -> [n,2] image points."""
    rays = _f64(rays, (-1, 2))
    out = np.empty_like(rays)
    d = None if displacement is None else _f64(displacement, (6,))
    _check(lib().ptz_project_rays(device, len(rays), u, v, float(f), float(pan), float(tilt), _ptr(d), _ptr(rays),
                                  _ptr(out)), "ptz_project_rays")
    return out


def back_project_rays(u, v, f, pan, tilt, points, displacement=None, device=0):
    """Batched PTZCamera.back_project_to_ray (ptz_camera.py:287-312): [n,2] points -> [n,2] rays."""
    pts = _f64(points, (-1, 2))
    out = np.empty_like(pts)
    d = None if displacement is None else _f64(displacement, (6,))
    _check(lib().ptz_back_project_rays(device, len(pts), u, v, float(f), float(pan), float(tilt), _ptr(d), _ptr(pts),
                                       _ptr(out)), "ptz_back_project_rays")
    return out


def h_jacobian(u, v, f, pan, tilt, rays, displacement=None, device=0):
    """PtzSlam.compute_h_jacobian (ptz_slam.py:73-138) on the GPU: dense H [2n, 3+2n]."""
    rays = _f64(rays, (-1, 2))
    n = len(rays)
    H = np.empty((2 * n, 3 + 2 * n))
    d = None if displacement is None else _f64(displacement, (6,))
    _check(lib().ptz_h_jacobian(device, n, u, v, float(f), float(pan), float(tilt), _ptr(d), _ptr(rays), _ptr(H)),
           "ptz_h_jacobian")
    return H


def match_knn2(des1, des2, device=None):
    """cv.BFMatcher().knnMatch(des1, des2, k=2) on the GPU (image_process.py:191): the two nearest train
    descriptors of every query, as (idx [n1, 2] int32, dist [n1, 2] float32 L2); ties to the lower index."""
    d1 = np.ascontiguousarray(des1, dtype=np.float32)
    d2 = np.ascontiguousarray(des2, dtype=np.float32)
    if d1.ndim != 2 or d2.ndim != 2 or (len(d2) and d1.shape[1] != d2.shape[1]):
        raise ValueError("descriptor arrays must be [n, dim] with the same dim")
    n1 = len(d1)
    idx = np.empty((n1, 2), np.int32)
    dist = np.empty((n1, 2), np.float32)
    if n1:
        _check(lib().ptz_match_knn2(default_device() if device is None else device, n1, len(d2), d1.shape[1], _ptr(d1),
                                    _ptr(d2), _ptr(idx), _ptr(dist)), "ptz_match_knn2")
    return idx, dist


def desc_put(key, des, device=None):
    """Upload descriptor rows (fp32 [n, dim]) under integer `key` on the device, kept for match_knn2_sets."""
    d = np.ascontiguousarray(des, dtype=np.float32)
    if d.ndim != 2:
        raise ValueError("descriptor array must be [n, dim]")
    _check(lib().ptz_desc_put(default_device() if device is None else device, int(key), len(d), max(d.shape[1], 1),
                              _ptr(d)), "ptz_desc_put")


def desc_put_new(key, des, device=None):
    """desc_put, returning the number of rows uploaded."""
    if len(des):
        d = np.ascontiguousarray(des, dtype=np.float32).reshape(len(des), -1)
    else:  # an empty set keeps its column count (an empty 2-D array), else 1
        shp = np.shape(des)
        d = np.zeros((0, shp[1] if len(shp) == 2 and shp[1] > 0 else 1), np.float32)
    desc_put(key, d, device)
    return len(d)


def desc_drop(keys, device=None):
    """Free the device descriptor sets under `keys` (unknown keys are ignored)."""
    k = np.ascontiguousarray(list(keys), dtype=np.uint64)
    if len(k):
        _check(lib().ptz_desc_drop(default_device() if device is None else device, len(k), _ptr(k)), "ptz_desc_drop")


def match_knn2_sets(query_keys, query_lens, train_key, device=None):
    """match_knn2 of the concatenated device descriptor sets `query_keys` (row counts `query_lens`, as uploaded)
    against the set `train_key`: (idx [n1, 2] int32, dist [n1, 2] float32), bit for bit match_knn2's."""
    qk = np.ascontiguousarray(list(query_keys), dtype=np.uint64)
    n1 = int(sum(query_lens))
    idx = np.empty((n1, 2), np.int32)
    dist = np.empty((n1, 2), np.float32)
    if n1:
        _check(lib().ptz_match_knn2_sets(default_device() if device is None else device, len(qk), _ptr(qk),
                                         int(train_key), n1, _ptr(idx), _ptr(dist)), "ptz_match_knn2_sets")
    return idx, dist


def match_sets_ransac(query_keys, query_rows, train_key, train_rows, query_xy, train_xy, threshold=1.0, n_hyp=2000,
                      seed=0, device=None):
    """ptz_match_sets_ransac: kNN-2 of resident query sets against a resident train set, ratio test, homography RANSAC
    per set.  Returns [(index1 int32, index2 int32) or None (8 or fewer ratio-test survivors)] per query set."""
    qk = np.ascontiguousarray(list(query_keys), dtype=np.uint64)
    rows = np.ascontiguousarray(list(query_rows), dtype=np.int64)
    qxy = np.ascontiguousarray(query_xy, dtype=np.float64).reshape(-1, 2)
    txy = np.ascontiguousarray(train_xy, dtype=np.float64).reshape(-1, 2)
    if len(qxy) != int(rows.sum()) or len(txy) != int(train_rows):
        raise ValueError("point arrays do not match the descriptor sets")
    st = np.zeros(len(qk), np.int32)
    off = np.zeros(len(qk) + 1, np.int64)
    i1 = np.empty(max(len(qxy), 1), np.int32)
    i2 = np.empty(max(len(qxy), 1), np.int32)
    _check(lib().ptz_match_sets_ransac(default_device() if device is None else device, len(qk), _ptr(qk), _ptr(rows),
                                       int(train_key), int(train_rows), _ptr(qxy), _ptr(txy), float(threshold),
                                       int(n_hyp), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(st), _ptr(off), _ptr(i1),
                                       _ptr(i2)), "ptz_match_sets_ransac")
    return [None if st[q] else (i1[off[q]:off[q + 1]], i2[off[q]:off[q + 1]]) for q in range(len(qk))]


def homography_ransac(points1, points2, threshold, n_hyp=2000, seed=0, device=None):
    """Homography RANSAC on the GPU (the cv.findHomography call of image_process.py:433): returns
    (inlier mask [n] bool, H [3, 3], inlier count)."""
    p1 = _f64(points1, (-1, 2))
    p2 = _f64(points2, (-1, 2))
    if len(p1) != len(p2):
        raise ValueError("point arrays differ in length")
    mask = np.zeros(len(p1), np.uint8)
    H = np.zeros(9)
    nin = c_int32(0)
    _check(lib().ptz_homography_ransac(default_device() if device is None else device, len(p1), _ptr(p1), _ptr(p2),
                                       float(threshold), int(n_hyp), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(mask), _ptr(H),
                                       ctypes.byref(nin)), "ptz_homography_ransac")
    return mask.astype(bool), H.reshape(3, 3), int(nin.value)


def homography_ransac_batch(sets, threshold, n_hyp=2000, seed=0, device=None):
    """Several independent homography RANSACs in one call (ptz_homography_ransac_batch): `sets` is a list of
    (points1 [n, 2], points2 [n, 2]) with n >= 4.  Returns a list of (mask [n] bool, H [3, 3], inlier count), each
    equal to homography_ransac(points1, points2, threshold, n_hyp, seed)."""
    if not sets:
        return []
    p1 = [_f64(a, (-1, 2)) for a, _ in sets]
    p2 = [_f64(b, (-1, 2)) for _, b in sets]
    if any(len(a) != len(b) for a, b in zip(p1, p2)):
        raise ValueError("point arrays differ in length")
    off = np.concatenate([[0], np.cumsum([len(a) for a in p1])]).astype(np.int64)
    P1 = np.ascontiguousarray(np.concatenate(p1))
    P2 = np.ascontiguousarray(np.concatenate(p2))
    mask = np.zeros(int(off[-1]), np.uint8)
    H = np.zeros((len(sets), 9))
    nin = np.zeros(len(sets), np.int32)
    _check(lib().ptz_homography_ransac_batch(default_device() if device is None else device, len(sets), _ptr(off),
                                             _ptr(P1), _ptr(P2), float(threshold), int(n_hyp),
                                             int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(mask), _ptr(H), _ptr(nin)),
           "ptz_homography_ransac_batch")
    return [(mask[off[k]:off[k + 1]].astype(bool), H[k].reshape(3, 3), int(nin[k])) for k in range(len(sets))]


def lk_track(img0, img1, points, win=31, levels=4, max_iter=30, eps=0.01, min_eig=1e-4, device=None):
    """Pyramidal Lucas-Kanade on the GPU (the cv.calcOpticalFlowPyrLK call of image_process.py:402, winSize
    31 x 31, OpenCV's default maxLevel 3 / 30 iterations / eps 0.01): 8-bit grey images [h, w], points [n, 2]
    (x, y).  Returns (next points [n, 2] float32, status [n] uint8, err [n] float32 = mean |I - J|)."""
    a = np.ascontiguousarray(img0, dtype=np.uint8)
    b = np.ascontiguousarray(img1, dtype=np.uint8)
    if a.ndim != 2 or a.shape != b.shape:
        raise ValueError("images must be 2-D 8-bit grey of the same shape")
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.float32).reshape(-1, 2))
    n = len(pts)
    out = np.empty((n, 2), np.float32)
    st = np.zeros(n, np.uint8)
    err = np.zeros(n, np.float32)
    if n:
        _check(lib().ptz_lk_track(default_device() if device is None else device, a.shape[1], a.shape[0], _ptr(a),
                                  _ptr(b), n, _ptr(pts), int(levels), int(win), int(max_iter), float(eps),
                                  float(min_eig), _ptr(out), _ptr(st), _ptr(err)), "ptz_lk_track")
    return out, st, err


def corner_min_eig(img, device=None):
    """cv.cornerMinEigenVal(img, blockSize=3, ksize=3) on the GPU (ptz_corner_min_eig): 8-bit grey [h, w].
    Returns (eig [h, w] float32, local-max flags [h, w] bool: goodFeaturesToTrack's candidates)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim != 2:
        raise ValueError("image must be 2-D 8-bit grey")
    eig = np.empty(a.shape, np.float32)
    flag = np.empty(a.shape, np.uint8)
    _check(lib().ptz_corner_min_eig(default_device() if device is None else device, a.shape[1], a.shape[0], _ptr(a),
                                    _ptr(eig), _ptr(flag)), "ptz_corner_min_eig")
    return eig, flag.astype(bool)


def match_hamming_cross(des1, des2, device=None):
    """cv.BFMatcher(cv.NORM_HAMMING, crossCheck=True).match(des1, des2) on the GPU (image_process.py:249-250):
    binary descriptors [n, nbytes] uint8.  Returns (query index, train index, bit distance) arrays of the
    mutual nearest neighbours, in query order."""
    a = np.ascontiguousarray(des1, dtype=np.uint8)
    b = np.ascontiguousarray(des2, dtype=np.uint8)
    if a.ndim != 2 or b.ndim != 2 or (len(a) and len(b) and a.shape[1] != b.shape[1]):
        raise ValueError("descriptor arrays must be [n, nbytes] with the same nbytes")
    nb = a.shape[1] if len(a) else b.shape[1]
    pad = (-nb) % 4
    if pad:  # zero bytes add no distance
        a = np.ascontiguousarray(np.pad(a, ((0, 0), (0, pad))))
        b = np.ascontiguousarray(np.pad(b, ((0, 0), (0, pad))))
    i12 = np.empty(len(a), np.int32)
    d12 = np.empty(len(a), np.int32)
    i21 = np.empty(len(b), np.int32)
    if len(a) and len(b):
        _check(lib().ptz_match_hamming(default_device() if device is None else device, len(a), len(b), nb + pad,
                                       _ptr(a), _ptr(b), _ptr(i12), _ptr(d12), _ptr(i21)), "ptz_match_hamming")
    else:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int32)
    q = np.flatnonzero(i21[i12] == np.arange(len(a)))
    return q, i12[q].astype(np.int64), d12[q]


def sift(img, nfeatures=0, device=None):
    """SIFT detectAndCompute on the GPU (image_process.py:67-68, OpenCV's defaults): 8-bit grey image [h, w].
    Returns (keypoints [n, 4] float32 = x, y, size, angle; response [n]; descriptors [n, 128] float32 with
    integer values), ordered by decreasing response, at most nfeatures (> 0)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim != 2:
        raise ValueError("sift expects a 2-D 8-bit grey image")
    dev = default_device() if device is None else device
    n = c_int32(0)
    cap = nfeatures if nfeatures > 0 else 4096
    while True:
        kp = np.zeros((cap, 4), np.float32)
        resp = np.zeros(cap, np.float32)
        des = np.zeros((cap, 128), np.float32)
        _check(lib().ptz_sift(dev, a.shape[1], a.shape[0], _ptr(a), int(nfeatures), cap, _ptr(kp), _ptr(resp),
                              _ptr(des), ctypes.byref(n)), "ptz_sift")
        if n.value <= cap:
            break
        cap = n.value
    k = n.value
    return kp[:k], resp[:k], des[:k]


def orb(img, nfeatures=500, descriptor="orb", device=None):
    """ORB detection + ORB (32-byte) or LATCH (64-byte) description on the GPU (ptz_orb; image_process.py:105-155):
    8-bit grey image [h, w].  Returns (keypoints [n, 6] float32 = x, y, size, angle, response, octave;
    descriptors [n, 32 | 64] uint8), ordered by level, then response.  Every tie at the per-level cuts is kept,
    so n may exceed nfeatures (the reference truncates; image_process.detect_compute_orb does)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim != 2:
        raise ValueError("orb expects a 2-D 8-bit grey image")
    kind = {"orb": 0, "latch": 1}[descriptor]
    nb = 64 if kind else 32
    dev = default_device() if device is None else device
    n = c_int32(0)
    cap = max(2 * int(nfeatures), 64)
    while True:
        kp = np.zeros((cap, 6), np.float32)
        des = np.zeros((cap, nb), np.uint8)
        _check(lib().ptz_orb(dev, a.shape[1], a.shape[0], _ptr(a), int(nfeatures), kind, cap, _ptr(kp), _ptr(des),
                             ctypes.byref(n)), "ptz_orb")
        if n.value <= cap:
            break
        cap = n.value
    k = n.value
    return kp[:k], des[:k]


def refine_poses(u, v, init_ptz, rays, points, subsets=None, ftol=1e-4, xtol=1e-8, max_iter=100, loss=LOSS_LINEAR,
                 f_scale=1.0, device=0):
    """Pose-only LM with the rays fixed (relocalization.py:22-40, 186), batched over hypotheses.
    init_ptz [n_hyp, 3]; rays / points [n, 2]; subsets: optional list of index arrays (one per
    hypothesis).  Returns (ptz [n_hyp, 3], cost [n_hyp], iterations [n_hyp], status [n_hyp])."""
    ptz = _f64(init_ptz).reshape(-1, 3).copy()
    rays = _f64(rays).reshape(-1, 2)
    points = _f64(points).reshape(-1, 2)
    if len(rays) != len(points):
        raise ValueError("rays and points differ in length")
    n_hyp = len(ptz)
    off = idx = None
    if subsets is not None:
        if len(subsets) != n_hyp:
            raise ValueError("one subset per hypothesis")
        off = np.zeros(n_hyp + 1, np.int64)
        off[1:] = np.cumsum([len(s) for s in subsets])
        idx = np.ascontiguousarray(np.concatenate([np.asarray(s, np.int64) for s in subsets]) if n_hyp else
                                   np.zeros(0), dtype=np.int32)
    cost = np.zeros(n_hyp)
    its = np.zeros(n_hyp, np.int32)
    st = np.zeros(n_hyp, np.int32)
    opts = ptz_refine_opts(int(max_iter), int(loss), float(ftol), float(xtol), float(f_scale))
    _check(lib().ptz_refine_poses(int(device), n_hyp, _ptr(ptz), len(rays), _ptr(rays), _ptr(points), float(u),
                                  float(v), _ptr(off), _ptr(idx), ctypes.byref(opts), _ptr(cost), _ptr(its), _ptr(st)),
           "ptz_refine_poses")
    return ptz, cost, its, st


def build_landmarks_flat(kp_count, pair_i, pair_j, pair_count, idx_a, idx_b):
    """First-seen landmark ids (image_process.py:611-653) in native code, over flat pair arrays.
    Returns (landmark id per match int64, n_landmark, n_inconsistent)."""
    kp = np.ascontiguousarray(kp_count, dtype=np.int64)
    pi = np.ascontiguousarray(pair_i, dtype=np.int32)
    pj = np.ascontiguousarray(pair_j, dtype=np.int32)
    cnt = np.ascontiguousarray(pair_count, dtype=np.int64)
    a = np.ascontiguousarray(idx_a, dtype=np.int64)
    b = np.ascontiguousarray(idx_b, dtype=np.int64)
    assert len(pi) == len(pj) == len(cnt) and len(a) == len(b) == int(cnt.sum())
    out = np.empty(len(a), np.int64)
    nl = c_int64(0)
    ninc = c_int64(0)
    _check(lib().ptzba_build_landmarks(len(kp), _ptr(kp), len(pi), _ptr(pi), _ptr(pj), _ptr(cnt), _ptr(a), _ptr(b),
                                       _ptr(out), ctypes.addressof(nl), ctypes.addressof(ninc)), "ptzba_build_landmarks")
    return out, int(nl.value), int(ninc.value)


def build_landmarks(kp_count, pairs):
    """build_landmarks_flat over an ordered list of (i, j, idx_a, idx_b).  Returns (list of per-pair
    landmark arrays, n_landmark, n_inconsistent)."""
    cnt = np.array([len(p[2]) for p in pairs], np.int64)
    cat = lambda k: np.concatenate([np.asarray(p[k], np.int64) for p in pairs]) if pairs else np.zeros(0, np.int64)
    out, nl, ninc = build_landmarks_flat(kp_count, [p[0] for p in pairs], [p[1] for p in pairs], cnt, cat(2), cat(3))
    offs = np.concatenate([[0], np.cumsum(cnt)])
    return [out[offs[k]:offs[k + 1]] for k in range(len(pairs))], nl, ninc


def py_shuffle_prefix(lens, keep, rand=None):
    """random.shuffle(list(range(n)))[:keep] for each n in `lens`, in order, drawn from the Mersenne Twister
    of `rand` (default: the global `random` module, as image_process.py:592-597), whose state advances
    exactly as the interpreter's own shuffles would.  Returns the concatenated prefixes (int64)."""
    import random as _random
    rand = _random if rand is None else rand
    version, internal, gauss = rand.getstate()
    mt = np.array(internal, dtype=np.uint32)
    lens = np.ascontiguousarray(lens, dtype=np.int64)
    out = np.empty(int(np.minimum(lens, keep).sum()), np.int64)
    _check(lib().ptz_py_shuffle_prefix(_ptr(mt), len(lens), _ptr(lens), int(keep), _ptr(out)), "ptz_py_shuffle_prefix")
    rand.setstate((version, tuple(mt.tolist()), gauss))
    return out


def set_order_pairs(a, b):
    """Iteration order of set(zip(a, b)) (CPython 3.8+ tuple hash and set probing), in native code."""
    a = np.ascontiguousarray(a, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.int64)
    oa = np.empty(len(a), np.int64)
    ob = np.empty(len(a), np.int64)
    n = c_int64(0)
    _check(lib().ptz_set_order_pairs(len(a), _ptr(a), _ptr(b), _ptr(oa), _ptr(ob), ctypes.addressof(n)),
           "ptz_set_order_pairs")
    return oa[:n.value], ob[:n.value]


def keyframe_features(n_frames, m_i, m_j, k1, k2, lm):
    """Per-keyframe (local keypoint, landmark) lists in the reference's set() order
    (bundle_adjustment.py:218-239).  Returns (off [n_frames+1], local, global) CSR arrays."""
    m_i = np.ascontiguousarray(m_i, dtype=np.int32)
    m_j = np.ascontiguousarray(m_j, dtype=np.int32)
    k1 = np.ascontiguousarray(k1, dtype=np.int64)
    k2 = np.ascontiguousarray(k2, dtype=np.int64)
    lm = np.ascontiguousarray(lm, dtype=np.int64)
    off = np.empty(n_frames + 1, np.int64)
    loc = np.empty(2 * len(m_i), np.int64)
    glo = np.empty(2 * len(m_i), np.int64)
    _check(lib().ptz_keyframe_features(int(n_frames), len(m_i), _ptr(m_i), _ptr(m_j), _ptr(k1), _ptr(k2), _ptr(lm),
                                       _ptr(off), _ptr(loc), _ptr(glo)), "ptz_keyframe_features")
    return off, loc[:off[-1]], glo[:off[-1]]


def keyframe_feature_counts(n_frames, m_i, m_j, k1, k2, lm):
    """len() of each keyframe's keyframe_features list (distinct (local, global) pairs), without forming the lists."""
    m_i = np.ascontiguousarray(m_i, dtype=np.int32)
    m_j = np.ascontiguousarray(m_j, dtype=np.int32)
    k1 = np.ascontiguousarray(k1, dtype=np.int64)
    k2 = np.ascontiguousarray(k2, dtype=np.int64)
    lm = np.ascontiguousarray(lm, dtype=np.int64)
    out = np.empty(int(n_frames), np.int64)
    _check(lib().ptz_keyframe_feature_counts(int(n_frames), len(m_i), _ptr(m_i), _ptr(m_j), _ptr(k1), _ptr(k2),
                                             _ptr(lm), _ptr(out)), "ptz_keyframe_feature_counts")
    return out


def pack_records(n_frames, m_i, m_j, k1, k2, lm, kp_off, kp_xy, n_landmark):
    """Pair-form records (frame int32 [2m], landmark int32 [2m], xy [2m, 2]) in _compute_residual order and
    the x0 source record of each landmark (bundle_adjustment.py:67-99, 186-195)."""
    m_i = np.ascontiguousarray(m_i, dtype=np.int32)
    m_j = np.ascontiguousarray(m_j, dtype=np.int32)
    k1 = np.ascontiguousarray(k1, dtype=np.int64)
    k2 = np.ascontiguousarray(k2, dtype=np.int64)
    lm = np.ascontiguousarray(lm, dtype=np.int64)
    kp_off = np.ascontiguousarray(kp_off, dtype=np.int64)
    kp_xy = np.ascontiguousarray(kp_xy, dtype=np.float64).reshape(-1, 2)
    m = len(m_i)
    fr = np.empty(2 * m, np.int32)
    ll = np.empty(2 * m, np.int32)
    xy = np.empty((2 * m, 2), np.float64)
    src = np.empty(int(n_landmark), np.int64)
    _check(lib().ptz_pack_records(int(n_frames), m, _ptr(m_i), _ptr(m_j), _ptr(k1), _ptr(k2), _ptr(lm), _ptr(kp_off),
                                  _ptr(kp_xy), int(n_landmark), _ptr(fr), _ptr(ll), _ptr(xy), _ptr(src)),
           "ptz_pack_records")
    return fr, ll, xy, src


# ---------------------------------------------------------------------------------------------
# BA handle
# ---------------------------------------------------------------------------------------------
def frame_coupling_window(n_pose, frame, landmark):
    """Highest frame sharing a landmark with each frame (>= the frame itself): the coupling window
    ptzba_set_problem derives from its own records.  Computed on the full record set it is the
    `frame_win_hi` every rank of a sharded solve passes, so all ranks choose the same system order."""
    frame = np.ascontiguousarray(frame, np.int32)
    landmark = np.ascontiguousarray(landmark, np.int32)
    n_lm = int(landmark.max()) + 1 if len(landmark) else 0
    win = np.empty(int(n_pose), np.int32)
    _check(lib().ptzba_coupling_window(int(n_pose), n_lm, len(frame), _ptr(frame), _ptr(landmark), _ptr(win)),
           "ptzba_coupling_window")
    return win


def plan_summary(frame_win_hi, n_fixed=1, ordering=None):
    """The system order and factorisation plan ptzba_set_problem would choose for a coupling window
    (ptzba_plan_summary, host only): dict(n_aug, ld, levels, nd_depth, chains, longest_chain, bs_steps,
    max_level_tasks, panel_pairs)."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    out = np.zeros(8, np.int64)
    _check(lib().ptzba_plan_summary(len(win), int(n_fixed), _ptr(win), ORDER_NESTED if ordering is None else int(ordering),
                                    _ptr(out)), "ptzba_plan_summary")
    return dict(n_aug=int(out[0]), ld=int(out[1]), levels=int(out[2]), nd_depth=int(out[3]), chains=int(out[4]),
                longest_chain=int(out[5]), bs_steps=int(out[6]), max_level_tasks=int(out[7] & 0xFFFFFFFF),
                panel_pairs=1 + int(out[7] >> 32))


def plan_export(frame_win_hi, n_fixed=1, ordering=None):
    """(pos [n_pose], tasks [n_tasks, 4] int32, level_off [levels + 1], n_aug, second_pair) of the plan
    ptzba_set_problem would choose (ptzba_plan_export, host only) -- for replaying the tile tasks on the CPU."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    o = ORDER_NESTED if ordering is None else int(ordering)
    c = np.zeros(4, np.int64)
    _check(lib().ptzba_plan_export(len(win), int(n_fixed), _ptr(win), o, None, None, 0, None, 0, _ptr(c)), "ptzba_plan_export")
    pos = np.empty(len(win), np.int32)
    tasks = np.empty((int(c[0]), 4), np.int32)
    off = np.empty(int(c[1]) + 1, np.int32)
    _check(lib().ptzba_plan_export(len(win), int(n_fixed), _ptr(win), o, _ptr(pos), _ptr(tasks), int(c[0]), _ptr(off),
                                   int(c[1]) + 1, _ptr(c)), "ptzba_plan_export")
    return pos, tasks, off, int(c[2]), bool(c[3])


def dist_plan_summary(frame_win_hi, world, rank, n_fixed=1):
    """The rank-tree plan of `rank` in a part-owned solve of `world` ranks (ptzba_dist_plan_summary, host only):
    dict(part_owned, nd_depth, base, phases, levels, est_us, tasks, max_level_tasks, x_part, x_sub, x_sep (doubles per
    trial), part_group, sub_group, sep_group (group sizes), n_aug, bs_steps)."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    out = np.zeros(16, np.int64)
    _check(lib().ptzba_dist_plan_summary(len(win), int(n_fixed), _ptr(win), int(world), int(rank), _ptr(out)),
           "ptzba_dist_plan_summary")
    keys = ("part_owned", "nd_depth", "base", "phases", "levels", "est_us", "tasks", "max_level_tasks", "x_part", "x_sub",
            "x_sep", "part_group", "sub_group", "sep_group", "n_aug", "bs_steps")
    return {k: int(v) for k, v in zip(keys, out)}


def dist_plan_export(frame_win_hi, world, rank, n_fixed=1):
    """Rank `rank`'s rank-tree plan (ptzba_dist_plan_export, host only) for a CPU replay: (pos [n_pose], tasks
    [n, 4] int32, level_off, n_aug, phases [(lv0, lv1, kind, r0, nr)], exchanged tiles per phase [[k, 2] int32])."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    c = np.zeros(5, np.int64)
    args = (len(win), int(n_fixed), _ptr(win), int(world), int(rank))
    _check(lib().ptzba_dist_plan_export(*args, None, None, 0, None, 0, None, 0, None, 0, _ptr(c)), "ptzba_dist_plan_export")
    pos = np.empty(len(win), np.int32)
    tasks = np.empty((int(c[0]), 4), np.int32)
    off = np.empty(int(c[1]) + 1, np.int32)
    ph = np.empty((int(c[3]), 6), np.int32)
    xt = np.empty((max(int(c[4]), 1), 2), np.int32)
    _check(lib().ptzba_dist_plan_export(*args, _ptr(pos), _ptr(tasks), int(c[0]), _ptr(off), int(c[1]) + 1, _ptr(ph),
                                        int(c[3]), _ptr(xt), int(c[4]), _ptr(c)), "ptzba_dist_plan_export")
    xts, o = [], 0
    for r in ph:
        xts.append(xt[o:o + int(r[5])])
        o += int(r[5])
    return pos, tasks, off, int(c[2]), [tuple(int(x) for x in r[:5]) for r in ph], xts


def dist_rank_phases(frame_win_hi, world, rank, n_fixed=1):
    """Phases of `rank` in a part-owned solve of `world` ranks (ptzba_dist_rank_phases, host only): [(exchange kind
    before the phase, group first rank, group size, first frame, end frame)]; [] when the solve is replicated."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    n = c_int32(0)
    _check(lib().ptzba_dist_rank_phases(len(win), int(n_fixed), _ptr(win), int(world), int(rank), None, 0,
                                        ctypes.byref(n)), "ptzba_dist_rank_phases")
    out = np.zeros((max(n.value, 1), 5), np.int32)
    _check(lib().ptzba_dist_rank_phases(len(win), int(n_fixed), _ptr(win), int(world), int(rank), _ptr(out), n.value,
                                        ctypes.byref(n)), "ptzba_dist_rank_phases")
    return [tuple(int(x) for x in row) for row in out[:n.value]]


# the collective model of choose_dist_form: a ring all-reduce costs ALPHA_US + 2 (p - 1) / p * bytes / LINK_GBS.  alpha is
# RCCL's small-message latency on an 8-GPU node, assumed (no multi-GPU node has run this build; bench.py --gpus N now
# measures it per exchange kind, `collectives` in its line); LINK_GBS one xGMI link per direction (conservative: RCCL's
# rings over the 7 links only shrink the byte term)
DIST_ALPHA_US = 15.0
DIST_LINK_GBS = 153.0


def dist_form_estimate(frame_win_hi, world, n_fixed=1, alpha_us=DIST_ALPHA_US, link_gbs=DIST_LINK_GBS):
    """ptzba_dist_form_estimate (host only): predicted per-trial cost of the rank-tree and the replicated form of a
    `world`-rank solve -- the slowest rank's factorisation estimate plus its collectives (dict, microseconds)."""
    win = np.ascontiguousarray(frame_win_hi, np.int32)
    out = np.zeros(8)
    _check(lib().ptzba_dist_form_estimate(len(win), int(n_fixed), _ptr(win), int(world), float(alpha_us), float(link_gbs),
                                          _ptr(out)), "ptzba_dist_form_estimate")
    return dict(tree_us=float(out[0]) if out[0] > 0 else None, replicated_us=float(out[1]), tree_factorisation_us=float(out[2]),
                full_factorisation_us=float(out[3]), tree_collectives=int(out[4]), tree_doubles=int(out[5]),
                replicated_doubles=int(out[6]), form="tree" if out[7] > 0 else "replicated",
                model=f"slowest rank's plan_est_us + ring all-reduces (alpha {alpha_us} us, {link_gbs} GB/s per link)")


def choose_dist_form(frame_win_hi, world, n_fixed=1, **kw):
    """The form of a `world`-rank solve with the smaller predicted trial: 'tree' (part-owned,
    partition_landmarks' split, set_problem(dist_world=world)) or 'replicated' (contiguous landmark blocks, one
    all-reduce of the packed system).  Returns (form, estimate dict)."""
    if world < 2:
        return "single", None
    est = dist_form_estimate(frame_win_hi, world, n_fixed, **kw)
    return est["form"], est


def replicated_shards(landmark, n_landmark, world):
    """Landmark -> rank of the replicated form: contiguous landmark blocks of ~equal record counts (-1: no records)."""
    cnt = np.bincount(np.asarray(landmark, np.int64), minlength=int(n_landmark))
    cum = np.cumsum(cnt)
    tot = max(int(cum[-1]) if len(cum) else 0, 1)
    owner = np.minimum((np.concatenate([[0], cum[:-1]]) * world) // tot, world - 1).astype(np.int32)
    owner[cnt == 0] = -1
    return owner


def partition_landmarks(n_pose, n_landmark, frame, landmark, world, n_fixed=1):
    """Landmark -> rank of a sharded solve (ptzba_partition_landmarks, host only): returns (rank_of_landmark
    [n_landmark] int32 (-1: no records), mode (1 part-owned, 0 replicated), (m, c_end, n_pose) split)."""
    frame = np.ascontiguousarray(frame, np.int32)
    landmark = np.ascontiguousarray(landmark, np.int32)
    out = np.empty(int(n_landmark), np.int32)
    mode = c_int32(0)
    split = np.zeros(3, np.int32)
    _check(lib().ptzba_partition_landmarks(int(n_pose), int(n_landmark), len(frame), _ptr(frame), _ptr(landmark),
                                           int(n_fixed), int(world), _ptr(out), ctypes.byref(mode), _ptr(split)),
           "ptzba_partition_landmarks")
    return out, int(mode.value), tuple(int(x) for x in split)


class DevArray:
    """__cuda_array_interface__ view of a device pointer owned by libptzba (fp64, for torch collectives)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 3,
                                         "strides": None}


def torch_exchange_hook(h, dist, device):
    """An exchange hook over torch.distributed for handle `h` (after set_problem with dist_world / dist_rank): the
    rank tree's groups are created on every rank from h.dist_groups() (collective: all ranks call this in the same
    order), and each exchange sums over the group h.exchange_group(kind) names.  For gloo rehearsals of several ranks
    on one device; a real multi-GPU run attaches the library's own RCCL communicator instead (Comm, attach_comm)."""
    import torch
    world = dist.get_world_size()
    groups = {(r0, nr): dist.new_group(list(range(r0, r0 + nr))) for r0, nr, _ in h.dist_groups()}

    def hook(kind, ptr, count, stream):
        r0, nr = h.exchange_group(kind)
        t = torch.as_tensor(DevArray(ptr, count), device=device)
        # (a replicated-form handle -- no dist_world -- reports a group of <= 1 rank: its exchanges sum over all ranks)
        dist.all_reduce(t, group=None if (nr <= 1 or nr == world) else groups[(r0, nr)])

    return hook


class Comm:
    """Library-owned RCCL communicator (ptzba_comm_*): one per rank, created from an RCCL unique id that rank 0
    makes with unique_id() and ships to the others over any channel (include/ptzba.h)."""

    def __init__(self, unique_id, rank, world, device=-1, _ptr_value=None):
        if _ptr_value is not None:
            self.c = _ptr_value
        else:
            uid = (ctypes.c_char * UNIQUE_ID_BYTES).from_buffer_copy(bytes(unique_id))
            self.c = lib().ptzba_comm_new(int(device), uid, int(rank), int(world))
        if not self.c:
            raise PtzbaError(f"ptzba_comm_new: {lib().ptzba_last_error().decode()}")
        self.rank, self.world = rank, world

    @staticmethod
    def unique_id():
        buf = (ctypes.c_char * UNIQUE_ID_BYTES)()
        _check(lib().ptzba_comm_unique_id(buf), "ptzba_comm_unique_id")
        return bytes(buf)

    def split(self, color, key):
        c = lib().ptzba_comm_split(self.c, int(color), int(key))
        if not c:
            raise PtzbaError(f"ptzba_comm_split: {lib().ptzba_last_error().decode()}")
        g = Comm(None, -1, -1, _ptr_value=c)
        g.rank, g.world = g.info()
        return g

    def info(self):
        """(rank, world) of this communicator as RCCL reports them (-1 when unknown)."""
        r, w = c_int32(-1), c_int32(-1)
        _check(lib().ptzba_comm_info(self.c, ctypes.byref(r), ctypes.byref(w)), "ptzba_comm_info")
        return r.value, w.value

    def allreduce(self, dev_ptr, count, stream=0):
        _check(lib().ptzba_comm_allreduce(self.c, c_void_p(dev_ptr), int(count), c_void_p(stream or 0)),
               "ptzba_comm_allreduce")

    def close(self):
        if getattr(self, "c", None):
            lib().ptzba_comm_delete(self.c)
            self.c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BAHandle:
    """One device-resident BA problem (opaque C handle, rf_map_wrapper.RFMap style)."""

    def __init__(self, device=0):
        L = lib()
        self.device = device
        self.h = L.ptzba_new(device)
        if not self.h:
            raise PtzbaError(f"ptzba_new({device}): {L.ptzba_last_error().decode()}")
        self.n_pose = self.n_landmark = self.n_obs = 0

    def close(self):
        if getattr(self, "h", None):
            lib().ptzba_delete(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        """Queue the handle's work on this hipStream_t (0 / None = the default stream)."""
        _check(lib().ptzba_set_stream(self.h, c_void_p(stream_ptr or 0)), "ptzba_set_stream")

    def use_own_stream(self):
        _check(lib().ptzba_use_own_stream(self.h), "ptzba_use_own_stream")

    def set_problem(self, n_pose, n_landmark, frame, landmark, xy, u, v, weight=None, precision=FP64,
                    loss=LOSS_LINEAR, f_scale=1.0, n_fixed=1, ordering=ORDER_NESTED, frame_win_hi=None,
                    dist_world=0, dist_rank=0):
        """frame_win_hi: optional global coupling window (see include/ptzba.h); pass the same array on
        every rank of a sharded solve (frame_coupling_window() of the full record set).  dist_world >= 2: this
        rank's share of a sharded solve, its landmarks chosen by partition_landmarks (part-owned solve when the
        frame chain splits, else replicated); the exchanges then run inside the library (attach_comm /
        set_exchange_hook)."""
        frame = np.ascontiguousarray(frame, dtype=np.int32)
        landmark = np.ascontiguousarray(landmark, dtype=np.int32)
        xy = _f64(xy, (-1, 2))
        n = len(frame)
        if len(landmark) != n or len(xy) != n:
            raise ValueError("frame/landmark/xy length mismatch")
        w = None if weight is None else _f64(weight, (n,))
        self._win = None if frame_win_hi is None else np.ascontiguousarray(frame_win_hi, dtype=np.int32)
        if self._win is not None and len(self._win) != int(n_pose):
            raise ValueError("frame_win_hi must have n_pose entries")
        opts = ptzba_problem_opts(int(precision), int(loss), float(f_scale), int(n_fixed), int(ordering),
                                  _ptr(self._win).value if self._win is not None else None, int(dist_world),
                                  int(dist_rank))
        _check(lib().ptzba_set_problem(self.h, int(n_pose), int(n_landmark), n, _ptr(frame), _ptr(landmark), _ptr(xy),
                                       _ptr(w), float(u), float(v), ctypes.byref(opts)), "ptzba_set_problem")
        self.n_pose, self.n_landmark, self.n_obs = int(n_pose), int(n_landmark), n
        self.precision = precision
        self.loss = int(loss)

    # multi-GPU exchanges run inside the library (include/ptzba.h PTZBA_X_*)
    internal_exchange = False

    def attach_comm(self, comm):
        """Exchange through the library's own RCCL communicator (Comm); None detaches."""
        _check(lib().ptzba_attach_comm(self.h, c_void_p(comm.c if comm is not None else 0)), "ptzba_attach_comm")
        self._comm = comm
        self.internal_exchange = comm is not None or getattr(self, "_hook", None) is not None

    def set_exchange_hook(self, fn):
        """fn(kind, dev_ptr, count, stream) -> None sums `count` fp64 values in place over the ranks of the exchange
        `kind` (X_SYS / X_PART (the rank's group) / X_SEP / X_SCAL), e.g. torch.distributed over gloo.  None removes."""
        if fn is None:
            self._hook = None
            _check(lib().ptzba_set_exchange_hook(self.h, EXCHANGE_FN(0), None), "ptzba_set_exchange_hook")
        else:
            def tramp(ctx, kind, ptr, count, stream):
                try:
                    fn(int(kind), int(ptr), int(count), int(stream or 0))
                    return 0
                except Exception as e:  # reported through ptzba_last_error's caller
                    import traceback
                    traceback.print_exc()
                    self._hook_error = e
                    return 1
            self._hook = EXCHANGE_FN(tramp)  # kept alive with the handle
            _check(lib().ptzba_set_exchange_hook(self.h, self._hook, None), "ptzba_set_exchange_hook")
        self.internal_exchange = fn is not None or getattr(self, "_comm", None) is not None

    def dist_info(self):
        out = np.zeros(8, np.int64)
        _check(lib().ptzba_dist_info(self.h, _ptr(out)), "ptzba_dist_info")
        return dict(mode="part-owned" if out[0] else "replicated", base=int(out[1]), group_size=int(out[2]),
                    group_leader=bool(out[3]), sep_doubles=int(out[4]), part_doubles=int(out[5]),
                    sys_doubles=int(out[6]), scal_doubles=int(out[7]))

    def dist_exchanges(self):
        """This rank's exchanges per LM trial: [(kind, group first rank, group size, doubles)]."""
        n = c_int32(0)
        _check(lib().ptzba_dist_exchanges(self.h, None, 0, ctypes.byref(n)), "ptzba_dist_exchanges")
        out = np.zeros((max(n.value, 1), 4), np.int64)
        _check(lib().ptzba_dist_exchanges(self.h, _ptr(out), n.value, ctypes.byref(n)), "ptzba_dist_exchanges")
        return [tuple(int(x) for x in row) for row in out[:n.value]]

    def dist_groups(self):
        """Every rank group of the rank tree below the whole world: [(first rank, size, depth)] (same on all ranks)."""
        n = c_int32(0)
        _check(lib().ptzba_dist_groups(self.h, None, 0, ctypes.byref(n)), "ptzba_dist_groups")
        out = np.zeros((max(n.value, 1), 3), np.int32)
        _check(lib().ptzba_dist_groups(self.h, _ptr(out), n.value, ctypes.byref(n)), "ptzba_dist_groups")
        return [tuple(int(x) for x in row) for row in out[:n.value]]

    def exchange_group(self, kind):
        """(first rank, size) of the group exchange `kind` sums over on this rank."""
        out = np.zeros(2, np.int32)
        _check(lib().ptzba_exchange_group(self.h, int(kind), _ptr(out)), "ptzba_exchange_group")
        return int(out[0]), int(out[1])

    def owned_frames(self):
        out = np.zeros(self.n_pose, np.uint8)
        _check(lib().ptzba_owned_frames(self.h, _ptr(out)), "ptzba_owned_frames")
        return out.astype(bool)

    def solver_info(self):
        out = np.zeros(8, np.int64)
        _check(lib().ptzba_solver_info(self.h, _ptr(out)), "ptzba_solver_info")
        return dict(n_aug=int(out[0]), ld=int(out[1]), levels=int(out[2]),
                    ordering="nested" if (out[3] & 0xFF) != ORDER_NATURAL else "natural", nd_depth=int(out[3]) >> 8,
                    backsolve=("lookahead", "left-looking", "blocked")[int(out[4])], n_slot=int(out[5]), schur_items=int(out[6]),
                    pattern_tiles=int(out[7]))

    def info(self):
        out = np.zeros(8, np.int64)
        _check(lib().ptzba_problem_info(self.h, _ptr(out)), "ptzba_problem_info")
        keys = ["n_pose", "n_landmark", "n_obs", "n_segments", "n_sys", "n_active_landmarks", "max_seg_per_landmark",
                "device_bytes"]
        return dict(zip(keys, [int(x) for x in out]))

    def residual(self, x_full):
        x_full = _f64(x_full, (-1,))
        if x_full.size != 3 * self.n_pose + 2 * self.n_landmark:
            raise ValueError("x_full has wrong size")
        r = np.empty(2 * self.n_obs)
        _check(lib().ptzba_residual(self.h, _ptr(x_full), _ptr(r)), "ptzba_residual")
        return r

    def set_state(self, ptz, rays):
        ptz = _f64(ptz, (self.n_pose, 3))
        rays = _f64(rays, (self.n_landmark, 2))
        _check(lib().ptzba_set_state(self.h, _ptr(ptz), _ptr(rays)), "ptzba_set_state")

    def save_state(self):
        """Snapshot the current state on the device (restart point for restore_state)."""
        _check(lib().ptzba_save_state(self.h), "ptzba_save_state")

    def restore_state(self):
        """Restore the saved state on the device (stream-ordered; no host transfer)."""
        _check(lib().ptzba_restore_state(self.h), "ptzba_restore_state")

    def get_state(self):
        ptz = np.empty((self.n_pose, 3))
        rays = np.empty((self.n_landmark, 2))
        _check(lib().ptzba_get_state(self.h, _ptr(ptz), _ptr(rays)), "ptzba_get_state")
        return ptz, rays

    def linearize(self):
        _check(lib().ptzba_linearize(self.h), "ptzba_linearize")

    def setup_timing(self):
        """Host phase times (ms) of the last set_problem, {phase: ms} in call order."""
        cap = 64
        names = (ctypes.c_char_p * cap)()
        ms = np.zeros(cap)
        n = ctypes.c_int32(0)
        _check(lib().ptzba_setup_timing(self.h, cap, ctypes.cast(names, c_void_p), _ptr(ms), ctypes.byref(n)),
               "ptzba_setup_timing")
        k = min(cap, n.value)
        return {names[i].decode(): float(ms[i]) for i in range(k)}

    def set_setup_front(self, min_records):
        """Device front of set_problem from `min_records` records on (0 always, -1 the library default, 64K; ptzba_set_setup_front)."""
        _check(lib().ptzba_set_setup_front(self.h, int(min(min_records, 2 ** 62))), "ptzba_set_setup_front")

    def set_huber_curvature(self, hc):
        """Host-driven LM: the huber curvature weight (units of rho' beyond the unit) of later linearisations."""
        _check(lib().ptzba_set_huber_curvature(self.h, float(hc)), "ptzba_set_huber_curvature")

    def build_reduced(self, lam):
        _check(lib().ptzba_build_reduced(self.h, float(lam)), "ptzba_build_reduced")

    def solve_reduced(self):
        _check(lib().ptzba_solve_reduced(self.h), "ptzba_solve_reduced")

    def step(self, lam):
        _check(lib().ptzba_step(self.h, float(lam)), "ptzba_step")

    def read_scalars(self):
        out = np.zeros(NSCALARS)
        _check(lib().ptzba_read_scalars(self.h, _ptr(out)), "ptzba_read_scalars")
        return out

    def accept(self, ok):
        _check(lib().ptzba_accept(self.h, 1 if ok else 0), "ptzba_accept")

    # device-driven LM (include/ptzba.h ptzba_lm_*)
    def lm_start(self):
        _check(lib().ptzba_lm_start(self.h), "ptzba_lm_start")

    def lm_init(self, opts):
        _check(lib().ptzba_lm_init(self.h, ctypes.byref(opts)), "ptzba_lm_init")

    def lm_build(self):
        _check(lib().ptzba_lm_build(self.h), "ptzba_lm_build")

    def lm_solve(self):
        _check(lib().ptzba_lm_solve(self.h), "ptzba_lm_solve")

    def lm_decide(self, k):
        _check(lib().ptzba_lm_decide(self.h, int(k)), "ptzba_lm_decide")

    def solve(self, ptz, rays, ftol=1e-4, xtol=1e-8, gtol=0.0, max_iter=100, lambda0=LAMBDA0, min_lambda=MIN_LAMBDA,
              max_lambda=1e16, max_retries=30, gauss_newton=False, huber_curvature=HUBER_CURVATURE,
              curvature_switch=CURVATURE_SWITCH):
        """One-shot ptzba_solve (C-driven LM to termination).  Returns (ptz [N,3], rays [M,2], LMResult)."""
        ptz = _f64(ptz, (self.n_pose, 3)).copy()
        rays = _f64(rays, (self.n_landmark, 2)).copy()
        opts = ptzba_lm_opts(ftol, xtol, gtol, 0.0 if gauss_newton else lambda0, min_lambda, max_lambda, int(max_iter),
                             int(max_retries), 1 if gauss_newton else 0, huber_curvature, curvature_switch)
        rep = ptzba_report()
        _check(lib().ptzba_solve(self.h, _ptr(ptz), _ptr(rays), ctypes.byref(opts), ctypes.byref(rep)), "ptzba_solve")
        res = LMResult(status=rep.status, message=STATUS_MSG.get(rep.status, "?"), cost=rep.cost,
                       initial_cost=rep.initial_cost, njev=rep.iterations, nfev=rep.nfev, iterations=rep.iterations,
                       lam=float("nan"), time=rep.time_s, history=[], trials=rep.trials)
        return ptz, rays, res

    def solve_resident(self, restore=False, ftol=1e-4, xtol=1e-8, gtol=0.0, max_iter=100, lambda0=LAMBDA0,
                       min_lambda=MIN_LAMBDA, max_lambda=1e16, max_retries=30, gauss_newton=False,
                       huber_curvature=HUBER_CURVATURE, curvature_switch=CURVATURE_SWITCH):
        """ptzba_solve_resident: the C-driven LM on the device-resident state (restore=True: from the
        save_state snapshot).  The state stays on the device.  Returns LMResult."""
        opts = ptzba_lm_opts(ftol, xtol, gtol, 0.0 if gauss_newton else lambda0, min_lambda, max_lambda, int(max_iter),
                             int(max_retries), 1 if gauss_newton else 0, huber_curvature, curvature_switch)
        rep = ptzba_report()
        _check(lib().ptzba_solve_resident(self.h, 1 if restore else 0, ctypes.byref(opts), ctypes.byref(rep)),
               "ptzba_solve_resident")
        return LMResult(status=rep.status, message=STATUS_MSG.get(rep.status, "?"), cost=rep.cost,
                        initial_cost=rep.initial_cost, njev=rep.iterations, nfev=rep.nfev, iterations=rep.iterations,
                        lam=float("nan"), time=rep.time_s, history=[], trials=rep.trials)

    def lm_wait(self, k):
        r = ptzba_lm_record()
        _check(lib().ptzba_lm_wait(self.h, int(k), ctypes.byref(r)), "ptzba_lm_wait")
        return r

    def exchange(self):
        sp = c_void_p(0)
        cnt = c_int64(0)
        sc = c_void_p(0)
        _check(lib().ptzba_exchange(self.h, ctypes.byref(sp), ctypes.byref(cnt), ctypes.byref(sc)), "ptzba_exchange")
        return sp.value, int(cnt.value), sc.value

    def exchange_packed(self):
        """(device pointer, count) of the packed exchange buffer (see include/ptzba.h)."""
        p, n = c_void_p(), c_int64()
        _check(lib().ptzba_exchange_packed(self.h, ctypes.byref(p), ctypes.byref(n)), "ptzba_exchange_packed")
        return p.value, n.value

    def pack(self):
        _check(lib().ptzba_pack(self.h), "ptzba_pack")

    def unpack(self):
        _check(lib().ptzba_unpack(self.h), "ptzba_unpack")

    def sync(self):
        _check(lib().ptzba_sync(self.h), "ptzba_sync")

    def reset_kernel_times(self, enable=True, groups=0xF, stride=1, flush=False):
        """Restart kernel timing; `groups` bitmask: 1 K1, 2 Schur, 4 Cholesky solve, 8 back-substitution, TIME_COMM (16)
        every exchange (comm_times);
        events around every `stride`-th launch of a group (each event record adds a gap to the stream).
        flush: cold-cache K1 timing, a 1 GiB scratch buffer streamed through the caches before each timed K1 launch
        (outside the events): True / "write" writes it (dirty lines left behind), "read" reads it (clean lines)."""
        fl = (TIME_FLUSH | (TIME_FLUSH_READ if flush == "read" else 0)) if flush else 0
        flags = (int(groups) | (max(1, min(255, int(stride))) << 8) | fl) if enable else 0
        _check(lib().ptzba_reset_kernel_times(self.h, flags), "ptzba_reset_kernel_times")

    def comm_times(self):
        """Exchanges timed since reset_kernel_times(groups=... | TIME_COMM): a list of (kind, doubles, ms), one per
        collective in stream order (kind: X_SYS / X_PART / X_SEP / X_SCAL / X_SUB)."""
        n = np.zeros(1, np.int32)
        _check(lib().ptzba_comm_times(self.h, 0, None, None, None, _ptr(n)), "ptzba_comm_times")
        m = int(n[0])
        kinds = np.zeros(max(m, 1), np.int32)
        dbl = np.zeros(max(m, 1), np.int64)
        ms = np.zeros(max(m, 1))
        _check(lib().ptzba_comm_times(self.h, m, _ptr(kinds), _ptr(dbl), _ptr(ms), _ptr(n)), "ptzba_comm_times")
        return [(int(k), int(d), float(t)) for k, d, t in zip(kinds[:m], dbl[:m], ms[:m])]

    def kernel_times(self):
        ms = np.zeros(4)
        cnt = np.zeros(4, np.int64)
        _check(lib().ptzba_kernel_times(self.h, _ptr(ms), _ptr(cnt)), "ptzba_kernel_times")
        names = ["linearize", "schur", "cholesky_solve", "backsub"]
        return {k: (float(m), int(c)) for k, m, c in zip(names, ms, cnt)}


# ---------------------------------------------------------------------------------------------
# Levenberg-Marquardt driver
# ---------------------------------------------------------------------------------------------
class EKFHandle:
    """Device-resident EKF tracking state (rays [R,2] + covariance [(3+2R)^2]) and its update
    (include/ptzba.h, ptzekf_*).  Mirrors the state half of PtzSlam (ptz_slam.py:21-71, 210-315)."""

    def __init__(self, device=0):
        L = lib()
        self._h = L.ptzekf_new(int(device))
        if not self._h:
            raise PtzbaError(f"ptzekf_new: {L.ptzba_last_error().decode()}")
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().ptzekf_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def n_ray(self):
        return int(lib().ptzekf_num_rays(self._h))

    def set_state(self, rays, cov):
        rays = _f64(rays).reshape(-1, 2)
        n = len(rays)
        cov = _f64(cov)
        if cov.shape != (3 + 2 * n, 3 + 2 * n):
            raise ValueError(f"state_cov must be [{3 + 2 * n}, {3 + 2 * n}], got {cov.shape}")
        _check(lib().ptzekf_set_state(self._h, n, _ptr(rays), _ptr(cov)), "ptzekf_set_state")

    def get_state(self, rays=True, cov=True):
        n = self.n_ray
        r = np.empty((n, 2)) if rays else None
        c = np.empty((3 + 2 * n, 3 + 2 * n)) if cov else None
        _check(lib().ptzekf_get_state(self._h, _ptr(r), _ptr(c)), "ptzekf_get_state")
        return r, c

    def add_pose_cov(self, q):
        q = _f64(q).reshape(3, 3)
        _check(lib().ptzekf_add_pose_cov(self._h, _ptr(q)), "ptzekf_add_pose_cov")

    def remove_rays(self, index):
        idx = np.ascontiguousarray(np.asarray(index).reshape(-1), dtype=np.int64)
        _check(lib().ptzekf_remove_rays(self._h, len(idx), _ptr(idx)), "ptzekf_remove_rays")

    def add_rays(self, rays, var):
        rays = _f64(rays).reshape(-1, 2)
        _check(lib().ptzekf_add_rays(self._h, len(rays), _ptr(rays), float(var)), "ptzekf_add_rays")

    def project_visible(self, u, v, ptz, height, width, displacement=None):
        n = self.n_ray
        xy = np.empty((max(n, 1), 2))
        idx = np.empty(max(n, 1))
        cnt = c_int32(0)
        d6 = None if displacement is None else _f64(displacement, (6,))
        _check(lib().ptzekf_project_visible(self._h, float(u), float(v), _ptr(d6), _ptr(_f64(ptz, (3,))),
                                            int(height), int(width), _ptr(xy), _ptr(idx), ctypes.byref(cnt)),
               "ptzekf_project_visible")
        c = cnt.value
        return xy[:c].copy(), idx[:c].copy()

    def update(self, u, v, ptz, obs_xy, obs_index, height, width, observe_var=0.1, displacement=None):
        """Returns (updated ptz [3], velocity [3], n_matched)."""
        ptz = _f64(ptz, (3,)).copy()
        obs_xy = _f64(obs_xy).reshape(-1, 2)
        obs_index = np.ascontiguousarray(np.asarray(obs_index).reshape(-1), dtype=np.int64)
        if len(obs_index) != len(obs_xy):
            raise ValueError("observed keypoints and indices differ in length")
        vel = np.zeros(3)
        nm = c_int32(0)
        d6 = None if displacement is None else _f64(displacement, (6,))
        _check(lib().ptzekf_update(self._h, float(u), float(v), _ptr(d6), _ptr(ptz), len(obs_index), _ptr(obs_xy),
                                   _ptr(obs_index), int(height), int(width), float(observe_var), _ptr(vel),
                                   ctypes.byref(nm)), "ptzekf_update")
        return ptz, vel, nm.value


class LMResult:
    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __repr__(self):
        return (f"LMResult(status={self.status}, cost={self.cost:.6g}, initial_cost={self.initial_cost:.6g}, "
                f"njev={self.njev}, nfev={self.nfev}, time={self.time:.4f}s)")


STATUS_DAMPING = 5  # include/ptzba.h PTZBA_STATUS_DAMPING
STATUS_MSG = {0: "max iterations", 1: "gtol", 2: "ftol", 3: "xtol", -1: "failed",
              STATUS_DAMPING: "damping limit: no cost decrease resolvable up to max_lambda"}


class LMSolver:
    """Levenberg-Marquardt over a BAHandle.

    `allreduce(kind)` (optional) is called at the two exchange points of a multi-GPU solve:
    kind == 'sys' after build_reduced (sum of the reduced camera system), kind == 'scal' after
    linearize / solve_reduced (sum of the partial scalars).  Single GPU: None.

    device_loop=True (default): the accept/reject decisions run on the device (ptzba_lm_*) and the host
    enqueues trial k+1's reduced-system build before it waits for trial k's decision, so the GPU never
    idles on a host round trip.  device_loop=False (or verbose): the same decisions on the host after
    reading each trial's scalars (also used for handles without ptzba_lm_*, e.g. test doubles)."""

    def __init__(self, handle, ftol=1e-4, xtol=1e-8, gtol=0.0, max_iter=100, lambda0=LAMBDA0, min_lambda=MIN_LAMBDA,
                 max_lambda=1e16, gauss_newton=False, allreduce=None, verbose=0, max_retries=30, device_loop=True,
                 huber_curvature=HUBER_CURVATURE, curvature_switch=CURVATURE_SWITCH):
        self.h = handle
        self.huber_curvature, self.curvature_switch = huber_curvature, curvature_switch
        self.ftol, self.xtol, self.gtol = ftol, xtol, gtol
        self.max_iter = max_iter
        self.lambda0 = 0.0 if gauss_newton else lambda0
        self.min_lambda, self.max_lambda = min_lambda, max_lambda
        self.gauss_newton = gauss_newton
        self.allreduce = allreduce
        self.verbose = verbose
        self.max_retries = max_retries
        self.device_loop = device_loop and hasattr(handle, "lm_start")
        if getattr(handle, "internal_exchange", False):
            self.allreduce = None  # the handle's library calls run the exchanges themselves

    def _scalars(self):
        if self.allreduce is not None:
            self.allreduce("scal")
        return self.h.read_scalars()

    def run(self, iterations=None, check_termination=True):
        if self.device_loop and check_termination and not self.verbose:
            return self._run_device(iterations)
        return self._run_host(iterations, check_termination)

    def _run_device(self, iterations=None):
        h = self.h
        t0 = time.perf_counter()
        max_iter = self.max_iter if iterations is None else iterations
        h.lm_start()
        if self.allreduce is not None:
            self.allreduce("scal")
        h.lm_init(ptzba_lm_opts(self.ftol, self.xtol, self.gtol, self.lambda0, self.min_lambda, self.max_lambda,
                                int(max_iter), int(self.max_retries), 1 if self.gauss_newton else 0,
                                self.huber_curvature, self.curvature_switch))

        def build():
            h.lm_build()
            if self.allreduce is not None:
                self.allreduce("sys")

        if max_iter <= 0:
            h.sync()
            cost = float(h.read_scalars()[0])
            return LMResult(status=0, message=STATUS_MSG[0], cost=cost, initial_cost=cost, njev=0, nfev=1,
                            iterations=0, lam=self.lambda0, time=time.perf_counter() - t0, history=[], trials=0)
        build()
        limit = max_iter * (self.max_retries + 1)
        k = 0
        while True:
            h.lm_solve()
            if self.allreduce is not None:
                self.allreduce("scal")
            h.lm_decide(k)
            if k + 1 < limit:
                build()  # next trial's build queued behind this decision (harmless after the last one)
            rec = h.lm_wait(k)
            if k == 0 and not np.isfinite(rec.initial_cost):
                # scipy least_squares' own check (least_squares.py: "Residuals are not finite in the initial point"):
                # a drop-in must not report a damping-limit stop for a problem it could never evaluate
                h.sync()
                raise ValueError("Residuals are not finite in the initial point.")
            k += 1
            if rec.done or k >= limit:
                break
        # no stream sync here: what is still queued (the speculative build after the final decision) is
        # skipped on the device, and every reader of the state (get_state, ...) orders itself on the stream
        t1 = time.perf_counter()
        return LMResult(status=rec.status, message=STATUS_MSG.get(rec.status, "?"), cost=rec.cost,
                        initial_cost=rec.initial_cost, njev=rec.iterations, nfev=rec.nfev, iterations=rec.iterations,
                        lam=rec.lam, time=t1 - t0, history=[], trials=rec.trials)

    def _run_host(self, iterations=None, check_termination=True):
        h = self.h
        t0 = time.perf_counter()
        # huber curvature switch (ptzba_lm_opts; the device loop's k_lm_decide rule): IRLS until an accepted step
        # is predicted to reduce the cost by less than curvature_switch of it, then huber_curvature, the current point re-linearised
        # every host run starts from IRLS (curvature 1), switch or not: a previous run on this handle may have left its
        # reduced curvature behind (ptzba_set_problem / ptzba_lm_start reset it, a host run did not before round 6)
        huber = getattr(h, "loss", LOSS_LINEAR) == LOSS_HUBER and hasattr(h, "set_huber_curvature")
        switch = huber and self.curvature_switch > 0 and self.huber_curvature < 1.0
        if huber:
            h.set_huber_curvature(1.0)
        h.linearize()
        s = self._scalars()
        cost = s[0]
        if not np.isfinite(cost):
            raise ValueError("Residuals are not finite in the initial point.")  # (scipy least_squares' check)
        initial_cost = cost
        lam = self.lambda0
        nu = 2.0
        njev = 1
        nfev = 1
        status = 0
        history = []
        max_iter = self.max_iter if iterations is None else iterations
        it = 0
        while it < max_iter:
            accepted = False
            retries = 0
            while not accepted and retries < self.max_retries:
                h.build_reduced(lam)
                if self.allreduce is not None:
                    self.allreduce("sys")
                h.solve_reduced()
                s = self._scalars()
                nfev += 1
                new_cost, pred, dx2, x2, info, gmax = s[1], s[2], s[3], s[4], s[5], s[6]
                ok_num = info == 0 and np.isfinite(new_cost) and np.isfinite(pred)
                actual = cost - new_cost
                rho = actual / pred if (ok_num and pred > 0) else -1.0
                if ok_num and (rho > 0 or (self.gauss_newton and lam == 0.0 and actual >= 0)):
                    accepted = True
                    h.accept(True)
                    if self.gauss_newton and lam == 0.0:
                        pass
                    else:
                        lam = max(self.min_lambda, lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3))
                    nu = 2.0
                else:
                    h.accept(False)
                    lam = max(lam * nu, 1e-9) if lam > 0 else 1e-9
                    nu *= 2.0
                    retries += 1
                    if lam > self.max_lambda:
                        break
            if not accepted:
                status = STATUS_DAMPING if retries < self.max_retries else -1
                break
            it += 1
            njev += 1
            old = cost
            cost = new_cost
            history.append((it, cost, lam, retries))
            if self.verbose:
                print(f"  iter {it:3d} cost {cost:.8e} dF {old - cost:.3e} lambda {lam:.2e} retries {retries}")
            if check_termination:
                if actual < self.ftol * old and rho > 0.25:  # scipy common.py check_termination
                    status = 2
                    break
                if np.sqrt(dx2) < self.xtol * (self.xtol + np.sqrt(x2)):
                    status = 3
                    break
                if self.gtol > 0 and gmax < self.gtol:
                    status = 1
                    break
                if it >= max_iter:
                    break
            if switch and pred < self.curvature_switch * old:
                switch = False
                h.set_huber_curvature(self.huber_curvature)
                h.linearize()
                self._scalars()
        if huber:
            # leave the handle in the documented state (IRLS) for direct linearize() / build_reduced() callers; the
            # state's linearisation slot is not touched (a following run re-linearises first)
            h.set_huber_curvature(1.0)
        h.sync()
        t1 = time.perf_counter()
        return LMResult(status=status, message=STATUS_MSG.get(status, "?"), cost=cost, initial_cost=initial_cost,
                        njev=it, nfev=nfev, iterations=it, lam=lam, time=t1 - t0, history=history)


_solve_handles = {}
_solve_lock = threading.Lock()


def release_solve_handles(device=None):
    """Free the BA handle(s) that solve() keeps between calls (all devices, or one): their device memory
    (records, slot tables, reduced system) is returned at once instead of at process exit."""
    with _solve_lock:
        devs = list(_solve_handles) if device is None else [device]
        for d in devs:
            h = _solve_handles.pop(d, None)
            if h is not None:
                h.close()


LAST_SOLVE_TIMING = {}  # host wall times of the last shared-handle solve() (set_problem, LM incl. state I/O)


def warm_up(device=0, precision=FP64):
    """First-use costs of solve()'s shared handle -- its creation (stream, pinned staging, device buffers) and the
    first launch of each BA kernel (code object loading) -- paid here instead of inside the first keyframe BA call
    (a keyframe map calls it when it receives its first keyframe, which has no BA: scene_map.Map.add_first_keyframe).
    Solves a 3-frame problem of 12 rays (both losses, from a perturbed x0) on the shared handle; nothing it computes
    is kept."""
    th = np.deg2rad(np.array([[a, b] for a in (-2.0, -1.0, 0.0, 1.0, 2.0, 3.0) for b in (-3.0, 1.0)]))
    ptz = np.array([[0.0, -2.0, 3000.0], [1.0, -2.0, 3000.0], [2.0, -2.0, 3000.0]])
    frame = np.repeat(np.arange(3, dtype=np.int32), len(th))
    landmark = np.tile(np.arange(len(th), dtype=np.int32), 3)
    xy = np.stack([640.0 + 3000.0 * np.tan(th[landmark, 0] - np.deg2rad(ptz[frame, 0])),
                   360.0 + 3000.0 * np.tan(th[landmark, 1] - np.deg2rad(ptz[frame, 1]))], 1)  # (near the model)
    rays = np.rad2deg(th)
    # x0 off the model (0.05 deg, 5 px of focal length): the solve takes real trials -- Schur build, factorisation,
    # back-substitution, decisions, the Huber curvature switch -- so their kernels' first launches happen here too
    # (from the exact model x0 the LM stopped at its first gradient test and a keyframe call paid them, ~8 ms)
    ptz0 = ptz + np.array([0.05, -0.05, 5.0])
    rays0 = rays + 0.05
    for loss in (LOSS_LINEAR, LOSS_HUBER):
        solve(3, len(th), frame, landmark, xy, 640.0, 360.0, ptz0, rays0, precision=precision, loss=loss, device=device,
              max_iter=5)


# solve()'s shared handles: records from which set_problem builds on the device (ptzba_set_setup_front; None: the
# library's default, 64K records -- a sliding window's ~170K records build on the device)
SETUP_FRONT_MIN = None


def solve(n_pose, n_landmark, frame, landmark, xy, u, v, init_ptz, init_rays, weight=None, precision=FP64,
          loss=LOSS_LINEAR, f_scale=1.0, device=0, keep_handle=True, **lm_kw):
    """Convenience one-shot solve.  Returns (ptz [N,3], rays [M,2], LMResult).  keep_handle=True (default): one
    handle per device is kept between calls (a keyframe map solves on every new keyframe: creating and
    destroying a handle -- stream, pinned records, device buffers -- cost ~6 ms per call); set_problem replaces
    its problem and release_solve_handles() frees it.  keep_handle=False: a private handle, closed on return.
    The shared handle is used under a lock: concurrent callers on one device run one at a time."""
    if not keep_handle:
        h = BAHandle(device)
        try:
            h.set_problem(n_pose, n_landmark, frame, landmark, xy, u, v, weight=weight, precision=precision, loss=loss,
                          f_scale=f_scale)
            h.set_state(init_ptz, init_rays)
            res = LMSolver(h, **lm_kw).run()
            ptz, rays = h.get_state()
            return ptz, rays, res
        finally:
            h.close()
    with _solve_lock:
        h = _solve_handles.get(device)
        if h is None or h.h is None:
            h = _solve_handles[device] = BAHandle(device)
        if SETUP_FRONT_MIN is not None:
            h.set_setup_front(SETUP_FRONT_MIN)
        try:
            t0 = time.perf_counter()
            h.set_problem(n_pose, n_landmark, frame, landmark, xy, u, v, weight=weight, precision=precision, loss=loss,
                          f_scale=f_scale)
            t1 = time.perf_counter()
            h.set_state(init_ptz, init_rays)
            t2 = time.perf_counter()
            res = LMSolver(h, **lm_kw).run()
            t3 = time.perf_counter()
            ptz, rays = h.get_state()
            LAST_SOLVE_TIMING.clear()
            for k, v in h.setup_timing().items():  # set_problem's host phases, ms -> s (keyframe BA breakdowns)
                LAST_SOLVE_TIMING["setup_" + k.replace("+", "_").replace(" ", "_") + "_s"] = v * 1e-3
            LAST_SOLVE_TIMING.update(set_problem_s=t1 - t0, lm_s=time.perf_counter() - t1, lm_set_state_s=t2 - t1,
                                     lm_run_s=t3 - t2, lm_get_state_s=time.perf_counter() - t3)
            return ptz, rays, res
        except Exception:
            _solve_handles.pop(device, None)
            h.close()
            raise
