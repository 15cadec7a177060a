#!/usr/bin/env python3
"""
Headline benchmark (BASELINE.json): BA iterations/sec at 500 keyframes x 20k ray landmarks
(config 3: fp32 LM + Huber on MI355X), plus pan/tilt/focal RMSE.

One bench "step" = one Levenberg-Marquardt iteration = one linearisation (residual + Jacobian +
normal-equation blocks over all pair-form records) + reduced-camera-system build + dense Cholesky
solve + back-substitution + trial evaluation, rejected trial steps counted inside the iteration
(scipy `njev` semantics).  The solver runs the reference's termination rule
(ftol=1e-4, bundle_adjustment.py:200); when a solve converges the state is reset to x0 and solving
continues until exactly K iterations were timed.  Inputs are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config config3] [--form pair|dedup]

N > 1 (one process per GPU): `--gpus N` without a torch.distributed environment re-launches this script
under `python -m torch.distributed.run --nproc-per-node N` (a child process, started before anything
touches the GPU); under the launcher the records are sharded by landmark block across ranks (poses
replicated) and the reduced camera system and the partial scalars are summed with an RCCL all-reduce
over xGMI each iteration (`scaling: strong`, same problem at every N).  Since round 3 the landmarks follow the
nested-dissection split of the frame chain (ptzba_partition_landmarks) and each rank factors only its part + the
separator: the exchange is the separator block; the library issues the collectives itself over its
own RCCL communicator (ptzba_comm, created from an RCCL unique id).  A world size that differs from
--gpus is an error.  `--dry-run` stops after the rendezvous (launcher plumbing test, no GPU).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "pan-tilt-zoom-slam_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)  # ~0.16 s timed at config 3: host jitter averages out
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="config3")
    ap.add_argument("--form", default="pair", choices=["pair", "dedup"])
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp64"])
    ap.add_argument("--loss", default="huber", choices=["huber", "linear"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-accuracy", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "k1_traffic.json"))
    ap.add_argument("--cpu-sample-kf", default="40,60,80",
                    help="keyframe windows of the CPU baseline fit (comma separated)")
    ap.add_argument("--cpu-window-only", action="store_true",
                    help="CPU baseline from the keyframe-window fit only (skip the full-size timing)")
    ap.add_argument("--no-cpu-window-fit", action="store_true", help="skip the secondary window-fit CPU leg")
    ap.add_argument("--cpu-full-nfev", type=int, default=2,
                    help="residual evaluations the full-size CPU leg is bounded to (2 = two Jacobians, one step)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the fp64 / linear-loss leg")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-cache K1 pass")
    ap.add_argument("--dry-run", action="store_true", help="launcher / rendezvous plumbing only (no GPU work)")
    ap.add_argument("--config4-steps", type=int, default=3,
                    help="secondary leg after a config3 headline: timed LM iterations of config 4 (5000 KF x 200k rays) at "
                         "the same N (0: skip)")
    ap.add_argument("--stream-frames", type=int, default=300,
                    help="config-5 leg: frames of demo_stream.py after the headline (0: skip); 300 = 60 keyframes, so the "
                         "30-keyframe sliding window is full for the second half (100 frames never fill it)")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a):
    """--gpus N > 1 outside a torch.distributed launch: run N ranks of this script under
    torch.distributed.run (a child process; this parent never touches the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


class _DevArray:
    """__cuda_array_interface__ view of a device pointer owned by libptzba (for torch all-reduce)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (ptr, False), "version": 3,
                                         "strides": None}


def shard_by_landmark(landmark, n_landmark, rank, world):
    """Contiguous landmark blocks with ~equal record counts; returns record mask of this rank."""
    cnt = np.bincount(landmark, minlength=n_landmark).astype(np.int64)
    cum = np.cumsum(cnt)
    tot = cum[-1]
    bounds = [0] + [int(np.searchsorted(cum, tot * k / world)) for k in range(1, world)] + [n_landmark]
    lo, hi = bounds[rank], bounds[rank + 1]
    return (landmark >= lo) & (landmark < hi)


def algorithmic_bytes_k1(info, precision, weighted):
    """Bytes one K1 (k_linearize) launch must move with this data layout (DESIGN.md §4 Roofline):
      per record : obs delta x,y (2 reals) + 1-byte segment key [+ weight real]
      per segment: frame id read in phase A and C (2 x 4 B), record offset (int64), base obs (2 fp64),
                   U|g_pose block out (12 reals), W+frame out (8 reals)
      per landmark (active): work-order id + CSR bounds (12 B), ray tables (8 reals + 8 fp64),
                   8-double output
      per frame  : frame tables (8 reals + 8 fp64)"""
    s = 4 if precision == "fp32" else 8
    rec = 2 * s + 1 + (s if weighted else 0)
    seg = 4 + 4 + 8 + 16 + 12 * s + 8 * s
    lm = 12 + 8 * s + 64 + 64
    return (info["n_obs"] * rec + info["n_segments"] * seg + info["n_active_landmarks"] * lm +
            info["n_pose"] * (8 * s + 64))


def survey_bytes_k1(info, precision):
    """SURVEY §8d formula B = N_rec*S_rec + (3 N_kf + 2 N_lm) s + N_lm 5 s + N_kf 9 s (S_rec = 16/24)."""
    s = 4 if precision == "fp32" else 8
    srec = 16 if precision == "fp32" else 24
    return info["n_obs"] * srec + (3 * info["n_pose"] + 2 * info["n_landmark"]) * s + info["n_landmark"] * 5 * s + \
        info["n_pose"] * 9 * s


def _cpu_window(prob, n_kf):
    """Sub-problem of the first n_kf keyframes: matches whose both records lie inside the window."""
    keep = (prob.frame < n_kf)
    m_keep = keep[0::2] & keep[1::2]
    rec_keep = np.repeat(m_keep, 2)
    frame = prob.frame[rec_keep].astype(np.int64)
    lm_old = prob.landmark[rec_keep].astype(np.int64)
    uniq, lm = np.unique(lm_old, return_inverse=True)
    xy = prob.xy[rec_keep]
    x0 = np.concatenate([prob.init_ptz[1:n_kf].reshape(-1), prob.init_rays[uniq].reshape(-1)])
    return frame, lm, xy, len(uniq), x0


def cpu_baseline(prob, windows, full=False, full_nfev=3):
    """Faithful CPU restatement (oracle): vectorised reference residual + scipy trf (x_scale='jac',
    ftol=1e-4, FD Jacobian with jac_sparsity), 1 thread.  Default: timed on keyframe windows of the headline
    problem and extrapolated to the full record count with a least-squares power law t = c R^alpha fitted
    over the windows (SURVEY's full-size run is super-linear in R).  full=True: the full problem itself,
    bounded to `full_nfev` residual evaluations (one Jacobian), i.e. a measurement, not a fit."""
    import scipy
    from threadpoolctl import threadpool_limits, threadpool_info
    sys.path.insert(0, ROOT)
    from oracle import ptz_oracle as orc
    R_full = len(prob.frame)
    env = dict(os_cpu_count=os.cpu_count(), scipy=scipy.__version__, numpy=np.__version__, threads_used=1,
               blas=[{k: d.get(k) for k in ("internal_api", "num_threads")} for d in threadpool_info()])
    with threadpool_limits(limits=1):
        if full:
            frame = prob.frame.astype(np.int64)
            lm = prob.landmark.astype(np.int64)
            x0 = np.concatenate([prob.init_ptz[1:].reshape(-1), prob.init_rays.reshape(-1)])
            t0 = time.perf_counter()
            res = orc.solve_scipy(x0, prob.n_pose, prob.n_landmark, prob.u, prob.v, prob.init_ptz[0], frame, lm,
                                  prob.xy, ftol=1e-4, max_nfev=full_nfev)
            dt = time.perf_counter() - t0
            its = max(res.njev, 1) / dt
            return dict(value=its, unit="BA it/s", cores=1, kind="port", env=env, seconds=dt,
                        sample=f"scipy trf (x_scale='jac', ftol=1e-4, FD jac_sparsity) on the FULL {prob.meta.get('config')} "
                               f"({R_full} pair records), 1 thread, stopped after max_nfev={full_nfev}: {res.njev} Jacobian(s), "
                               f"{res.nfev} evaluations in {dt:.1f} s; it/s = njev / wall time (scipy's iteration "
                               f"count, as SURVEY §6's 0.0155 it/s)")
        pts = []
        for n_kf in windows:
            frame, lm, xy, m, x0 = _cpu_window(prob, n_kf)
            t0 = time.perf_counter()
            res = orc.solve_scipy(x0, n_kf, m, prob.u, prob.v, prob.init_ptz[0], frame, lm, xy, ftol=1e-4)
            dt = time.perf_counter() - t0
            pts.append((n_kf, len(frame), m, res.njev, dt, dt / max(res.njev, 1)))
    lr = np.log([p[1] for p in pts])
    lt = np.log([p[5] for p in pts])
    alpha, logc = np.polyfit(lr, lt, 1) if len(pts) > 1 else (1.0, lt[0] - lr[0])
    alpha = max(float(alpha), 1.0)  # never extrapolate sub-linearly in the record count
    t_full = float(np.exp(logc + alpha * np.log(R_full))) if len(pts) > 1 else pts[0][5] * R_full / pts[0][1]
    desc = "; ".join(f"{p[0]} KF: {p[1]} records, {p[2]} landmarks, {p[3]} its in {p[4]:.2f} s" for p in pts)
    return dict(value=1.0 / t_full, unit="BA it/s", cores=1, kind="port", env=env, fit_alpha=alpha,
                sample=f"scipy trf (x_scale='jac', ftol=1e-4, FD jac_sparsity), 1 thread, on keyframe windows of "
                       f"{prob.meta.get('config')} [{desc}]; seconds/iteration fitted as c*R^{alpha:.3f} and evaluated at "
                       f"the full R = {R_full} records")


def stream_leg(frames):
    """BASELINE configs[4] beside the headline: demo_stream.py (the demo_soccer.py:31-51 loop: GPU SIFT / LK / RANSAC
    front-end on rendered 1080p frames, EKF tracking, 30-keyframe sliding-window BA, scene_map.py:91-115's per-keyframe
    "BA time") for `frames` frames in a child process, after the timed region.  A secondary field, not the metric."""
    cmd = [sys.executable, os.path.join(PKG, "demo_stream.py"), "--frames", str(frames), "--window", "30"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # report, never hide
        return {"error": repr(e)}
    keep = ("workload", "frontend", "frames", "fps_end_to_end", "tracking_ms", "keyframes", "keyframe_ba_ms",
            "lost_frames", "pose_rmse_vs_truth", "keyframe_ba_breakdown_ms", "keyframe_ba_slowest_breakdown_ms",
            "render_s_outside_loop", "gc", "gc_pauses_ms")
    return {k: d[k] for k in keep if k in d}


def _git_blob(path):
    """Provenance of a committed measurement file: its git blob id (None outside a checkout)."""
    try:
        return subprocess.run(["git", "-C", ROOT, "hash-object", path], capture_output=True, text=True,
                              timeout=10).stdout.strip() or None
    except Exception:
        return None


K1_PASS_ITERS = 64  # LM iterations of the dedicated K1 timing pass (>= 64 event-bracketed K1 launches)
K1_COLD_ITERS = 16  # LM iterations of the cold-cache K1 pass (a 1 GiB flush before each K1 launch)
BASELINE_METRIC = "BA iterations/sec at 500 KF x 20k rays; pan-tilt-focal RMSE vs reference"  # BASELINE.json metric


def metric_name(cfg):
    """BASELINE.json's metric for the headline config; the same wording with the config's own size otherwise (a
    --config config4 line must not carry the headline's name)."""
    import synthetic
    if cfg == "config3":
        return BASELINE_METRIC
    n_kf, n_rays = synthetic.CONFIGS[cfg][:2]
    return f"BA iterations/sec at {n_kf} KF x {n_rays // 1000}k rays; pan-tilt-focal RMSE vs reference"


class Ctx:
    """Per-process run context: rank / world, torch.distributed, the stream, the library's RCCL communicator."""

    def __init__(self, a, world, rank, local, dist, backend, stream, comm):
        self.a, self.world, self.rank, self.local, self.dist, self.backend = a, world, rank, local, dist, backend
        self.stream, self.comm = stream, comm


def setup_leg(cx, cfg):
    """Problem of BASELINE config `cfg` (synthetic, seed 0), sharded over the ranks in the form the planner predicts
    faster (ptzba.choose_dist_form: rank tree or replicated; PTZBA_DIST_MODE=part|replicated forces one), on a handle
    with x0 saved on the device.  Returns a dict of everything the legs report."""
    import ptzba
    import synthetic
    a, world, rank = cx.a, cx.world, cx.rank
    t0 = time.perf_counter()
    prob = synthetic.make_problem(cfg, seed=0)
    t_gen = time.perf_counter() - t0
    frame, landmark, xy, w = prob.frame, prob.landmark, prob.xy, None
    if a.form == "dedup":
        frame, landmark, xy, w, _ = synthetic.dedup_records(frame, landmark, xy)
    # the coupling window of the WHOLE problem: every rank passes the same one, so all ranks choose the same system
    # order and take bit-identical pose steps
    win_hi = ptzba.frame_coupling_window(prob.n_pose, frame, landmark)
    dist_mode, split, form_est = "single", None, None
    if world > 1:
        form, form_est = ptzba.choose_dist_form(win_hi, world)
        env = os.environ.get("PTZBA_DIST_MODE")
        if env in ("part", "tree"):
            form = "tree"
        elif env == "replicated":
            form = "replicated"
        if form == "tree":
            owner, mode, split = ptzba.partition_landmarks(prob.n_pose, prob.n_landmark, frame, landmark, world)
            if mode != 1:
                form = "replicated"
        if form == "replicated":
            owner = ptzba.replicated_shards(landmark, prob.n_landmark, world)
        sel = owner[landmark] == rank
        dist_mode = "part-owned" if form == "tree" else "replicated"
        frame, landmark, xy = frame[sel], landmark[sel], xy[sel]
        w = None if w is None else w[sel]
    precision = ptzba.FP32 if a.precision == "fp32" else ptzba.FP64
    loss = ptzba.LOSS_HUBER if a.loss == "huber" else ptzba.LOSS_LINEAR
    h = ptzba.BAHandle(cx.local if world > 1 else 0)
    h.set_stream(cx.stream.cuda_stream)
    t1 = time.perf_counter()
    h.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v, weight=w, precision=precision,
                  loss=loss, f_scale=1.0, frame_win_hi=win_hi, dist_world=world if dist_mode == "part-owned" else 0,
                  dist_rank=rank)
    t_setup = time.perf_counter() - t1
    xinfo = None
    if world > 1:
        # the library runs every exchange itself: through its own RCCL communicator (one per rank, from an RCCL unique
        # id rank 0 makes and torch.distributed ships), or -- gloo rehearsals of several ranks on one device --
        # through a hook over torch.distributed
        if cx.comm is None:
            h.set_exchange_hook(ptzba.torch_exchange_hook(h, cx.dist, f"cuda:{cx.local}"))
        else:
            h.attach_comm(cx.comm)
        xinfo = h.dist_info()
        xinfo["exchanges"] = h.dist_exchanges()  # (kind, group first rank, group size, doubles) per trial
        if xinfo["sys_doubles"] == 0 and xinfo["mode"] == "replicated":
            xinfo["sys_doubles"] = h.exchange_packed()[1]
        xinfo["form"] = dist_mode
        xinfo["form_estimate"] = form_est
    # x0 is uploaded once and kept on the device: each solve restarts from it without a PCIe transfer
    h.set_state(prob.init_ptz, prob.init_rays)
    h.save_state()
    return dict(cfg=cfg, prob=prob, frame=frame, landmark=landmark, xy=xy, w=w, h=h, info=h.info(),
                sinfo=h.solver_info(), xinfo=xinfo, dist_mode=dist_mode, split=split, precision=precision, loss=loss,
                generate_s=t_gen, set_problem_s=t_setup)


def run_iters(hh, k, ar=None):
    """k LM iterations (scipy njev) of restarted ftol=1e-4 solves from the device-resident x0 (ptzba_solve_resident: the
    restart is enqueued by C the moment the final decision is on the host; PTZBA_BENCH_PYLOOP=1: the Python loop)."""
    import ptzba
    pyloop = os.environ.get("PTZBA_BENCH_PYLOOP") == "1"
    done = 0
    solves = 0
    while done < k:
        if pyloop or ar is not None:
            hh.restore_state()
            res = ptzba.LMSolver(hh, ftol=1e-4, xtol=1e-8, max_iter=k - done, allreduce=ar).run()
        else:
            res = hh.solve_resident(restore=True, ftol=1e-4, xtol=1e-8, max_iter=k - done)
        done += max(res.njev, 1)
        solves += 1
        if res.njev == 0:
            break
    return done, solves


def timed(cx, hh, steps):
    """Exactly `steps` iterations between a barrier + device synchronisation on both sides; the max over ranks."""
    import torch
    if cx.dist:
        cx.dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its, nsolve = run_iters(hh, steps)
    torch.cuda.synchronize()
    if cx.dist:
        cx.dist.barrier()
    el = time.perf_counter() - t0
    if cx.dist:
        tt = torch.tensor([el], dtype=torch.float64, device=f"cuda:{cx.local}")
        cx.dist.all_reduce(tt, op=cx.dist.ReduceOp.MAX)
        el = float(tt.item())
    return its, nsolve, el


KIND_NAMES = {0: "X_SYS", 1: "X_PART", 2: "X_SEP", 3: "X_SCAL", 4: "X_SUB"}


def breakdown(cx, h, iters):
    """Kernel-group times (HIP events: K1, Schur, factorisation + back-solve, trial) over `iters` iterations after the
    timed region, and at N > 1 every collective (ptzba_comm_times: an event pair around each exchange on the handle's
    stream) -- per rank, gathered to every rank."""
    import ptzba
    h.reset_kernel_times(True, groups=0xF | (ptzba.TIME_COMM if cx.world > 1 else 0))
    its, _ = run_iters(h, iters)
    ktn = h.kernel_times()
    kt = {k: v[0] for k, v in ktn.items()}
    rec = None
    if cx.world > 1:
        ct = h.comm_times()
        by = {}
        for kind, n, ms in ct:
            d = by.setdefault(KIND_NAMES.get(kind, str(kind)), {"n": 0, "ms": 0.0, "bytes": 0})
            d["n"] += 1
            d["ms"] += ms
            d["bytes"] += 8 * n
        for d in by.values():
            d["avg_ms"] = d["ms"] / d["n"]
            d["avg_bytes"] = d["bytes"] / d["n"]
        tot_ms = sum(ms for _, _, ms in ct)
        rec = {"rank": cx.rank, "kernel_ms": kt, "iterations": its,
               "collective_ms_per_iteration": tot_ms / max(its, 1),
               "collective_bytes_per_iteration": sum(8 * n for _, n, _ in ct) / max(its, 1),
               "n_collectives_per_iteration": len(ct) / max(its, 1),
               # the factorisation group's span (one per trial) contains the tree's in-phase exchanges: net of them
               "factorisation_ms_net": kt["cholesky_solve"] - sum(ms for kind, _, ms in ct if kind in (2, 4)) /
               max(1, ktn["cholesky_solve"][1]),
               "trials": ktn["cholesky_solve"][1],
               "by_kind": by, "samples": [(int(k), int(n), round(float(ms), 5)) for k, n, ms in ct[:64]]}
        allr = [None] * cx.world
        cx.dist.all_gather_object(allr, rec)
        rec = allr
    h.reset_kernel_times(False)
    return kt, rec


def collective_fit(per_rank):
    """alpha and bandwidth of the collectives as measured: least squares ms = alpha + bytes / B over every timed
    exchange of every rank (X_SCAL's 128 B give alpha, the separator / system blocks the byte term)."""
    pts = [(n * 8, ms) for r in per_rank or [] for (_, n, ms) in r.get("samples", [])]
    if len(pts) < 2 or len({b for b, _ in pts}) < 2:
        return None
    x = np.array([b for b, _ in pts], float)
    y = np.array([m for _, m in pts], float)
    A = np.stack([np.ones_like(x), x], 1)
    (c0, c1), *_ = np.linalg.lstsq(A, y, rcond=None)
    small = y[x <= 1024]
    return {"alpha_us": 1e3 * float(c0), "gbps": (1e-6 / float(c1)) if c1 > 0 else None,
            "small_message_us_median": 1e3 * float(np.median(small)) if len(small) else None, "samples": len(pts),
            "note": "each exchange's HIP-event span on its rank's stream (includes waiting for the slowest rank)"}


def secondary_leg(cx, cfg, steps, warmup):
    """A second BASELINE config after the headline, same N (config 4: 5000 KF x 200k rays, the workload BASELINE names
    for 8 GPUs): a few timed iterations, the kernel breakdown and the per-rank collectives.  A secondary field."""
    t0 = time.perf_counter()
    leg = setup_leg(cx, cfg)
    h = leg["h"]
    try:
        run_iters(h, max(warmup, 1))
        iters, solves, el = timed(cx, h, steps)
        kt, per_rank = breakdown(cx, h, 2)
    finally:
        h.close()
    prob, info = leg["prob"], leg["info"]
    out = {"workload": f"{cfg}: {prob.n_pose} KF x {prob.n_landmark} matched rays, {int(len(prob.frame))} pair-form "
                       f"records, {cx.a.loss} loss, {cx.a.precision} LM",
           "metric": metric_name(cfg), "value": iters / el, "unit": "BA it/s", "ms_per_step": 1e3 * el / iters,
           "iterations_timed": iters, "solves_timed": solves, "warmup": max(warmup, 1), "n_gpus": cx.world,
           "kernel_ms": kt, "records_rank0": info["n_obs"], "reduced_system": leg["sinfo"],
           "parallelism": leg["dist_mode"] if cx.world > 1 else "single GPU",
           "generate_s": leg["generate_s"], "set_problem_s": leg["set_problem_s"],
           "leg_wall_s": time.perf_counter() - t0}
    if cx.world > 1:
        out["exchange"] = leg["xinfo"]
        out["per_rank"] = per_rank
        out["collective_fit"] = collective_fit(per_rank)
    return out


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if a.gpus > 1 and env_world is None:
        sys.exit(launch_ranks(a))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(3)
    import torch
    dist = None
    backend = "none"
    if world > 1:
        import torch.distributed as dist
        # one process per GPU over RCCL ("nccl").  PTZBA_DIST_BACKEND=gloo rehearses the same protocol
        # with several ranks on one device (the ranks then share GPU local % device_count)
        backend = os.environ.get("PTZBA_DIST_BACKEND", "gloo" if a.dry_run else "nccl")
        if not a.dry_run:
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
        if dist.get_world_size() != a.gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {a.gpus}", file=sys.stderr)
            sys.exit(3)
        backend = dist.get_backend()
    if a.dry_run:
        if dist:
            dist.barrier()
        if rank == 0:
            print(json.dumps({"metric": metric_name(a.config), "value": None, "unit": "BA it/s", "n_gpus": world,
                              "world_size": world, "backend": backend, "dry_run": True}))
        if dist:
            dist.destroy_process_group()
        return
    if world == 1:
        torch.cuda.set_device(0)
    import ptzba
    import synthetic

    comm = None
    if world > 1 and backend != "gloo":
        uid = [ptzba.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = ptzba.Comm(uid[0], rank, world, device=local)
    stream = torch.cuda.current_stream()
    cx = Ctx(a, world, rank, local, dist, backend, stream, comm)
    leg = setup_leg(cx, a.config)
    prob, frame, landmark, xy, w, h = leg["prob"], leg["frame"], leg["landmark"], leg["xy"], leg["w"], leg["h"]
    info, sinfo, xinfo, dist_mode, split = leg["info"], leg["sinfo"], leg["xinfo"], leg["dist_mode"], leg["split"]
    precision, loss = leg["precision"], leg["loss"]

    # warmup
    run_iters(h, max(a.warmup, 1))
    # K1's HIP events stay on during the timed region (roofline), around every 4th K1 launch (each event
    # record adds a gap to the stream; the launches are identical work); the other groups' events are
    # timed in a separate pass afterwards
    h.reset_kernel_times(True, groups=1, stride=4)
    iters, solves, elapsed = timed(cx, h, a.steps)
    k1_ms_region, k1_n_region = h.kernel_times()["linearize"]
    # the roofline's K1 figure: a dedicated pass after the timed region, EVERY K1 launch of K1_PASS_ITERS LM iterations
    # event-bracketed (stride 1), so the figure does not depend on --steps (the in-region sample is kept beside it)
    h.reset_kernel_times(True, groups=1, stride=1)
    run_iters(h, K1_PASS_ITERS)
    k1_ms, k1_n = h.kernel_times()["linearize"]
    kt, per_rank = breakdown(cx, h, min(5, a.steps))
    # cold-cache K1: a 1 GiB scratch buffer streamed through the caches before each timed K1 launch (outside its events)
    # evicts L2 and the 256 MB Infinity Cache, so the launch streams its records from HBM (SURVEY §8d caveat): written
    # (rounds 2-4's `cold_cache`: dirty caches whose write-backs run during the launch) and read (round 5 on:
    # `cold_cache_read`, clean caches)
    k1_cold_ms = k1_cold_n = k1_dirty_ms = k1_dirty_n = None
    if not a.no_cold:
        h.reset_kernel_times(True, groups=1, flush="read")
        run_iters(h, K1_COLD_ITERS)
        k1_cold_ms, k1_cold_n = h.kernel_times()["linearize"]
        h.reset_kernel_times(True, groups=1, flush="write")
        run_iters(h, K1_COLD_ITERS)
        k1_dirty_ms, k1_dirty_n = h.kernel_times()["linearize"]
    h.reset_kernel_times(False)

    # accuracy: the benched arithmetic's solve vs the pinned oracle's tight optimum of the reference cost (the metric's
    # "pan-tilt-focal RMSE vs reference": tests/golden/config3_optimum.npz, made by tests/golden/make_golden.py
    # gen_config3 -- the oracle restatement of bundle_adjustment.py:25-106 minimised to a step < 1e-11, pinned to the
    # reference's own residual on all 29.2M values), vs a full fp64 solve of the same records, and vs ground truth
    accuracy = None
    secondary = None
    opt = None
    opt_path = os.path.join(ROOT, "tests", "golden", f"{a.config}_optimum.npz")
    if os.path.exists(opt_path):
        z = np.load(opt_path)
        if int(z["n_records"]) == len(prob.frame) and int(z["frame_sum"]) == int(prob.frame.astype(np.int64).sum()):
            opt = {k: z[k] for k in ("ptz_tight", "rays_tight", "tight_cost", "ptz_tight_huber", "rays_tight_huber",
                                     "tight_cost_huber")}
    if not a.no_accuracy and world == 1:
        key = "_huber" if a.loss == "huber" else ""
        if opt is not None:
            # the solve exactly as benched (ftol=1e-4, the reference's termination) from x0
            h.set_state(prob.init_ptz, prob.init_rays)
            rb = ptzba.LMSolver(h, ftol=1e-4, xtol=1e-8, max_iter=100).run()
            ptzb, raysb = h.get_state()
        h.set_state(prob.init_ptz, prob.init_rays)
        r32 = ptzba.LMSolver(h, ftol=1e-10, xtol=1e-12, max_iter=50).run()
        ptz32, rays32 = h.get_state()
        h64 = ptzba.BAHandle(0)
        h64.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v, weight=w,
                        precision=ptzba.FP64, loss=loss, f_scale=1.0)
        h64.set_state(prob.init_ptz, prob.init_rays)
        r64 = ptzba.LMSolver(h64, ftol=1e-12, xtol=1e-12, max_iter=50).run()
        ptz64, _ = h64.get_state()
        h64.close()
        accuracy = dict(rmse_fp32_vs_fp64=[float(x) for x in synthetic.pose_rmse(ptz32, ptz64)],
                        rmse_fp64_vs_ground_truth=[float(x) for x in synthetic.pose_rmse(ptz64, prob.gt_ptz)],
                        cost_fp32=r32.cost, cost_fp64=r64.cost, iters_fp32=r32.njev, iters_fp64=r64.njev,
                        components=["pan_deg", "tilt_deg", "f_px"])
        if opt is not None:
            pt, rt, ct = opt["ptz_tight" + key], opt["rays_tight" + key], float(opt["tight_cost" + key])
            rr = lambda y: float(np.sqrt(np.mean((np.asarray(y) - rt) ** 2)))  # noqa: E731
            accuracy["rmse_vs_oracle_optimum"] = {
                "reference": f"tests/golden/{a.config}_optimum.npz ({a.loss} loss): tight optimum of the oracle restatement "
                             "of the reference residual (bundle_adjustment.py:25-106), max step < 1e-11; gate 1e-4",
                "bench_solve_ftol_1e-4": [float(x) for x in synthetic.pose_rmse(ptzb, pt)],
                "bench_solve_rays_deg": rr(raysb), "bench_solve_iterations": rb.njev,
                "bench_solve_cost_rel": (rb.cost - ct) / ct,
                f"{a.precision}_tight": [float(x) for x in synthetic.pose_rmse(ptz32, pt)], f"{a.precision}_tight_rays_deg": rr(rays32),
                "fp64_tight": [float(x) for x in synthetic.pose_rmse(ptz64, pt)],
                "components": ["pan_deg", "tilt_deg", "f_px"]}
    if not a.no_secondary and world == 1 and not (a.precision == "fp64" and a.loss == "linear"):
        # the reference's own arithmetic and loss (fp64, linear: bundle_adjustment.py:200), same records
        hs = ptzba.BAHandle(0)
        hs.set_stream(stream.cuda_stream)
        hs.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v, weight=w,
                       precision=ptzba.FP64, loss=ptzba.LOSS_LINEAR, f_scale=1.0)
        hs.set_state(prob.init_ptz, prob.init_rays)
        hs.save_state()
        run_iters(hs, max(a.warmup, 1))
        hs.reset_kernel_times(True, groups=1, stride=4)
        s_it, s_solves, s_el = timed(cx, hs, a.steps)
        s_k1, _ = hs.kernel_times()["linearize"]
        hs.reset_kernel_times(True, groups=0xF)
        run_iters(hs, min(5, a.steps))
        s_kt = hs.kernel_times()
        hs.reset_kernel_times(False)
        if opt is not None and not a.no_accuracy:  # the reference's arithmetic vs the linear-loss optimum
            hs.set_state(prob.init_ptz, prob.init_rays)
            rs = ptzba.LMSolver(hs, ftol=1e-4, xtol=1e-8, max_iter=100).run()
            ptzs, _ = hs.get_state()
            s_rmse = {"ftol_1e-4": [float(x) for x in synthetic.pose_rmse(ptzs, opt["ptz_tight"])], "iterations": rs.njev}
        else:
            s_rmse = None
        s_alg = survey_bytes_k1(hs.info(), "fp64")
        s_alg_layout = algorithmic_bytes_k1(hs.info(), "fp64", w is not None)
        s_ach = s_alg / (s_k1 * 1e-3) / 1e9 if s_k1 > 0 else 0.0
        secondary = {"precision": "fp64", "loss": "linear", "value": s_it / s_el, "unit": "BA it/s",
                     "ms_per_step": 1e3 * s_el / s_it, "iterations_timed": s_it, "solves_timed": s_solves,
                     "roofline": {"bound": "hbm", "achieved": s_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": s_ach / HBM_PEAK_GBS, "k1_avg_ms": s_k1, "algorithmic_bytes_per_launch": s_alg,
                                  "layout_bytes_per_launch": s_alg_layout,
                                  "frac_layout_bytes": s_alg_layout / (s_k1 * 1e-3) / 1e9 / HBM_PEAK_GBS if s_k1 > 0 else 0.0,
                                  "note": "fp64 K1 moves > 256 MB per launch (larger than the Infinity Cache)"},
                     "kernel_ms": {k: v[0] for k, v in s_kt.items()}}
        if s_rmse:
            secondary["rmse_vs_oracle_optimum"] = s_rmse
        hs.close()

    # the drop-in call as a caller sees it (scene_map.py:91-115 times bundle_adjustment() as "BA time"): host
    # preparation + upload (set_problem), x0 upload, the LM solve at the reference's ftol, the result download --
    # NOT the metric (which excludes upload), reported beside it
    dropin = None
    if not a.no_secondary and world == 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hd = ptzba.BAHandle(0)
        hd.set_problem(prob.n_pose, prob.n_landmark, frame, landmark, xy, prob.u, prob.v, weight=w, precision=precision,
                       loss=loss, f_scale=1.0)
        t1 = time.perf_counter()
        hd.set_state(prob.init_ptz, prob.init_rays)
        rd = ptzba.LMSolver(hd, ftol=1e-4, xtol=1e-8, max_iter=100).run()
        hd.get_state()
        t2 = time.perf_counter()
        hd.close()
        dropin = {"set_problem_s": t1 - t0, "solve_and_io_s": t2 - t1, "total_s": t2 - t0, "iterations": rd.njev,
                  "what": "ptzba.BAHandle: set_problem (host packing + upload) + set_state + LMSolver(ftol=1e-4) + "
                          "get_state, one cold call (new handle)"}

    traffic = traffic_src = None  # PMC passes are taken on the whole problem (N = 1); a shard's launch moves less
    if world == 1 and os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            key = f"{a.config}/{a.form}/{a.precision}/{a.loss}"
            if key in tj:
                traffic = tj[key]["hbm_bytes_per_launch"]
                rel = os.path.relpath(a.traffic_json, ROOT)
                traffic_src = {"file": rel, "git_blob": _git_blob(a.traffic_json), "key": key,
                               "measured_by": tj[key].get("measured_by", "tools/gpu_measure.sh (rocprofv3 --pmc "
                                                          "FETCH_SIZE / WRITE_SIZE, separate passes)")}
        except Exception:
            traffic = None
    h.close()

    # BASELINE configs[3] (5000 KF x 200k rays) at the same N after the headline: the anchor of the config the
    # multi-GPU design is for (a secondary field, not the metric)
    cfg4 = None
    if a.config == "config3" and a.config4_steps > 0:
        try:
            cfg4 = secondary_leg(cx, "config4", a.config4_steps, 1)
        except Exception as e:  # report, never hide
            cfg4 = {"error": repr(e)}

    if rank == 0:
        # roofline bytes: SURVEY §8d's per-unit formula (234 MB at config 3 fp32 pair form) is `achieved`;
        # this layout's own bytes (1-byte keys, dense W / U|g slot writes that §8d excludes) ride beside it
        alg_layout = algorithmic_bytes_k1(info, a.precision, w is not None)
        alg = survey_bytes_k1(info, a.precision)
        achieved = alg / (k1_ms * 1e-3) / 1e9 if k1_ms > 0 else 0.0
        achieved_layout = alg_layout / (k1_ms * 1e-3) / 1e9 if k1_ms > 0 else 0.0
        out = {
            "metric": metric_name(a.config),
            "value": iters / elapsed,
            "unit": "BA it/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * elapsed / iters,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32" if a.precision == "fp32" else "f64",
            "data": "synthetic (SURVEY §8d generator, seed 0)",
            "world_size": world,
            "backend": backend,
            "config": {"workload": f"{a.config}: {prob.n_pose} KF x {synthetic.CONFIGS[a.config][1]} generated rays "
                                   f"({prob.n_landmark} matched), {info['n_obs']} {a.form}-form records/rank, "
                                   f"{a.loss} loss, {a.precision} LM",
                       "n_keyframes": prob.n_pose, "n_landmarks": prob.n_landmark, "n_records": int(len(prob.frame)),
                       "n_matches": int(prob.n_match), "n_pairs": prob.n_pairs, "form": a.form,
                       "arithmetic": ({"records_K1": "fp32 (deltas from fp64 segment bases)",
                                       "schur_K2": "fp16x3 split MFMA (hi*hi + hi*lo + lo*hi of rtz fp16 splits, "
                                                   "22 significant bits) on v_mfma_f32_16x16x32_f16, fp32 accumulate "
                                                   "over 4 batches, fp64 flush",
                                       "reduced_system_and_state": "fp64 (v_mfma_f64_16x16x4_f64 tile Cholesky)"}
                                      if a.precision == "fp32" else
                                      {"records_K1": "fp64", "schur_K2": "fp64 VALU",
                                       "reduced_system_and_state": "fp64"}),
                       "parallelism": (f"{dist_mode} x{world} (landmark shards; "
                                       + ("each rank factors its part of the frame chain + the separator, "
                                          f"split A/C/B at frames {split[0]}/{split[1]}"
                                          if dist_mode == "part-owned" else "every rank factors the whole summed system")
                                       + f"; exchanges by the library over {'RCCL (ptzba_comm)' if comm else backend}"
                                       + "; form chosen by ptzba.choose_dist_form)")
                                      if world > 1 else "single GPU",
                       "reduced_system": sinfo,
                       "exchange": xinfo,
                       "allreduce_bytes_per_trial": (8 * (xinfo["sep_doubles"] + xinfo["part_doubles"] +
                                                          xinfo["sys_doubles"] + xinfo["scal_doubles"])
                                                     if xinfo else 0),
                       "iterations_timed": iters, "solves_timed": solves},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "k_linearize (K1)",
                         "k1_avg_ms": k1_ms, "k1_launches_timed": k1_n, "k1_event_stride": 1,
                         "k1_method": f"dedicated pass after the timed region: every K1 launch of {K1_PASS_ITERS} LM "
                                      "iterations between HIP events on the handle's stream",
                         "k1_avg_ms_timed_region": k1_ms_region, "k1_launches_timed_region": k1_n_region,
                         "k1_event_stride_timed_region": 4,
                         "algorithmic_bytes_per_launch": alg,
                         "bytes_basis": "SURVEY §8d: N_rec*S_rec + (3 N_kf + 2 N_lm) s + N_lm 5 s + N_kf 9 s",
                         "layout_bytes_per_launch": alg_layout, "achieved_layout_bytes": achieved_layout,
                         "frac_layout_bytes": achieved_layout / HBM_PEAK_GBS},
            "kernel_ms": kt,
        }
        if world > 1:
            out["per_rank"] = per_rank
            out["collective_fit"] = collective_fit(per_rank)
        if k1_cold_ms:
            # key semantics as in rounds 2-4: `cold_cache` is the WRITE flush, the read flush (round 5 on,
            # clean caches) is `cold_cache_read`
            ach_d = alg / (k1_dirty_ms * 1e-3) / 1e9
            out["roofline"]["cold_cache"] = {
                "k1_avg_ms": k1_dirty_ms, "launches": k1_dirty_n, "achieved": ach_d, "frac": ach_d / HBM_PEAK_GBS,
                "method": "1 GiB scratch WRITE before each timed K1 launch (rounds 2-4's method: the caches are left "
                          "dirty, so ~256 MB of unrelated write-backs run during the timed launch)"}
            ach_c = alg / (k1_cold_ms * 1e-3) / 1e9
            out["roofline"]["cold_cache_read"] = {
                "k1_avg_ms": k1_cold_ms, "launches": k1_cold_n, "achieved": ach_c, "frac": ach_c / HBM_PEAK_GBS,
                "frac_layout_bytes": alg_layout / (k1_cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "method": "1 GiB scratch READ before each timed K1 launch (L2 and the 256 MB Infinity Cache hold clean "
                          "unrelated lines)"}
            out["roofline"]["cold_cache_schema"] = 2
        if accuracy:
            out["accuracy"] = accuracy
        if secondary:
            out["fp64_linear"] = secondary
        if dropin:
            out["dropin_call"] = dropin
        if cfg4 is not None:
            out["config4"] = cfg4
        if not a.no_cpu_baseline and world == 1:
            # the full-size timing is the baseline (the scipy restatement on the 14.6M-record
            # problem itself); the keyframe-window power-law fit is kept beside it as a secondary field
            try:
                if not a.cpu_window_only:
                    cb = cpu_baseline(prob, [], full=True, full_nfev=a.cpu_full_nfev)
                    out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample", "env")}
                    out["cpu_baseline"]["seconds"] = cb["seconds"]
                if not a.no_cpu_window_fit or a.cpu_window_only:
                    cw = cpu_baseline(prob, [int(x) for x in str(a.cpu_sample_kf).split(",") if x])
                    fit = {k: cw[k] for k in ("value", "unit", "cores", "kind", "sample", "fit_alpha")}
                    if a.cpu_window_only:
                        out["cpu_baseline"] = dict(fit, env=cw["env"])
                    else:
                        out["cpu_baseline_window_fit"] = fit
                cbv = out.get("cpu_baseline", {}).get("value")
                out["vs_cpu_baseline"] = out["value"] / cbv if cbv else None
            except Exception as e:  # report, never hide
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        if a.stream_frames > 0 and world == 1:
            out["config5"] = stream_leg(a.stream_frames)
        print(json.dumps(out))
    if comm is not None:
        comm.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
