/*
 * ptzba.h — C-ABI of libptzba.so, the MI355X (gfx950) PTZ-SLAM bundle-adjustment + tracking library.
 *
 * Boundary style mirrors the reference's only native FFI, the rf_map ctypes shim
 * (reference: slam_system/rf_map/python_package/rf_map.hpp:15-19, 47-64; rf_map_wrapper.py:13-82):
 * extern "C" entry points, opaque handle from ptzba_new() / ptzba_delete(), caller-owned contiguous float64
 * host buffers passed as plain pointers, in/out buffers carry the initial state in and the result out,
 * the library never frees caller memory, one call at a time per handle.
 * Improvement over the reference's void+assert: every call returns int status (0 = ok) and
 * ptzba_last_error() returns a message; outputs are left unchanged on failure.
 *
 * Entry points and the reference interface each one replaces:
 *   ptzba_set_problem   <- the data hand-off of bundle_adjustment.py:167-202 (points, src/dst/landmark
 *                          index lists, u, v, ref pose) and the file-based stub
 *                          backup/bundle_adjustment_python.hpp:21-24 (bundle_adjustment_opt, body empty)
 *   ptzba_residual      <- bundle_adjustment._compute_residual (bundle_adjustment.py:25-106), same order
 *   ptzba_linearize ... ptzba_accept
 *                       <- scipy.optimize.least_squares(_compute_residual, x0, x_scale='jac',
 *                          ftol=1e-4, method='trf') at bundle_adjustment.py:200-202 (one LM iteration
 *                          = linearize + reduced camera system + solve + accept/reject)
 *   ptz_ray_to_image    <- TransFunction.from_ray_to_image (transformation.py:99-135), batched
 *   ptz_image_to_ray    <- TransFunction.from_image_to_ray (transformation.py:137-175), batched
 *   ptz_project_rays    <- PTZCamera.project_ray(s) (ptz_camera.py:191-234), batched, signed q2
 *   ptz_back_project_rays <- PTZCamera.back_project_to_ray(s) (ptz_camera.py:287-325), batched
 *   ptz_h_jacobian      <- PtzSlam.compute_h_jacobian (ptz_slam.py:73-138) (central FD, same steps)
 *   ptzba_build_landmarks <- build_matching_graph landmark-id bookkeeping (image_process.py:611-653)
 *   ptz_py_shuffle_prefix / ptz_keyframe_features / ptz_pack_records <- BA data prep
 *
 * Angles are degrees, focal length / pixels as in the reference.  Poses are [pan, tilt, f] per
 * frame; rays are [theta, phi] per landmark.  Frame 0 is the fixed gauge frame (bundle_adjustment.py:197).
 */
#ifndef PTZBA_H
#define PTZBA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTZBA_EXPORT __attribute__((visibility("default")))

typedef struct ptzba_ctx* ptzba_handle;

/* precision: arithmetic/record type of the per-observation kernels.  The reduced camera system,
 * its factorisation and the parameter state are always fp64. */
enum { PTZBA_FP64 = 0, PTZBA_FP32 = 1 };
/* loss (scipy least_squares `loss=`): linear, or huber with f_scale */
enum { PTZBA_LOSS_LINEAR = 0, PTZBA_LOSS_HUBER = 1 };

/* ordering of the reduced camera system: natural frame order, or one level of nested dissection
 * (left block | right block reversed | separator) when it shortens the factorisation's critical path */
enum { PTZBA_ORDER_NATURAL = 0, PTZBA_ORDER_NESTED = 1, PTZBA_ORDER_NESTED_FORCE = 2 /* tests */ };

typedef struct {
    int32_t precision;             /* PTZBA_FP64 | PTZBA_FP32 */
    int32_t loss;                  /* PTZBA_LOSS_LINEAR | PTZBA_LOSS_HUBER */
    double f_scale;                /* huber scale (scipy f_scale); ignored for linear */
    int32_t n_fixed;               /* number of leading fixed (gauge) frames; the reference fixes frame 0 -> 1 */
    int32_t ordering;              /* PTZBA_ORDER_NATURAL | PTZBA_ORDER_NESTED */
    const int32_t* frame_win_hi;   /* optional [n_pose]: highest frame sharing a landmark with each frame,
                                      over ALL records of a sharded problem; every rank must pass the same
                                      array so all ranks pick the same system order.  NULL: local records */
    int32_t dist_world;            /* ranks of a sharded solve (0 or 1: single process).  >= 2 with the
                                      landmarks partitioned by ptzba_partition_landmarks: PART-OWNED solve */
    int32_t dist_rank;             /* this process's rank in [0, dist_world) */
} ptzba_problem_opts;

/* ---------------- multi-GPU: part-owned solve of the reduced camera system (rank tree) ----------------
 * The frame chain splits by nested dissection (one level: A | C | B, or two: A1 | C1 | A2 | C2 | A3 | C3 | A4) into
 * a separator tree.  The ranks are dealt over it: a node with R >= 2 ranks gives ceil(R / 2) to its lower-frame
 * child and the rest to the other; a node reached with one rank is that rank's OWN subtree, a leaf reached with
 * R >= 2 ranks is SHARED by them.  ptzba_partition_landmarks sends each landmark down the tree to the child whose
 * frames it sees (separator-only landmarks to the nearer child), a shared leaf's landmarks in equal-record
 * contiguous blocks.  A rank factors its base (own subtree or shared leaf) and then each ancestor separator up to
 * the root, in phases; before each later phase the library sums that separator's columns (its tiles, g and diag U,
 * b via the augmented row) over the node's rank group -- PTZBA_X_SUB for an inner separator, PTZBA_X_SEP for the
 * root -- and a shared leaf's columns before the first phase (PTZBA_X_PART).  An update from one phase into a later
 * phase's tile is applied by one member of the phase's group only, so the separators' Schur-complement work is split
 * over the group and every contribution is summed exactly once.  Each rank back-substitutes its phases; frames
 * outside them keep their values on a rank (ptzba_owned_frames).  With dist_world >= 2 but no valid split (every
 * frame couples to the last one), the solve is REPLICATED: every rank factors the whole summed system (exchange
 * PTZBA_X_SYS).  dist_world < 2: a single-process problem.
 * mode_out: 1 part-owned, 0 replicated; rank_of_landmark [n_landmark] (landmarks without records: -1);
 * split_out[3] (may be NULL) = (m, c_end, n_pose): A = [n_fixed, m), C = [m, c_end), B = [c_end, n_pose). */
/* host only: the system order and factorisation plan ptzba_set_problem chooses for a coupling window
 * (frame_win_hi[f] = last frame coupled to f, e.g. from ptzba_coupling_window) and ordering.  out8: [0] n_aug,
 * [1] ld, [2] factorisation levels, [3] dissection levels (0 natural, 1, 2), [4] back-substitution chains,
 * [5] longest chain (tile columns), [6] blocked back-solve steps (0: none), [7] most tasks in one level
 * | (second update-panel pair in use) << 32. */
PTZBA_EXPORT int ptzba_plan_summary(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t ordering,
                                    int64_t* out8);
/* host only: the same choice's frame positions pos_out[n_pose] (system row of each frame's pan, -1 fixed), the
 * factorisation tasks (int4 records {type | panels 2, 3; i; j; panels 0, 1}, tasks_cap records) and level
 * offsets (levels_cap >= levels + 1).  counts: [0] tasks, [1] levels, [2] n_aug, [3] second panel pair in use.
 * Call with null outputs to size them. */
PTZBA_EXPORT int ptzba_plan_export(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t ordering,
                                   int32_t* pos_out, int32_t* tasks_out, int64_t tasks_cap, int32_t* level_off_out,
                                   int64_t levels_cap, int64_t* counts);
/* host only: the rank-tree plan of rank `rank` in a part-owned solve of `world` ranks for a coupling window.  out16:
 * [0] part-owned (0: replicated / none), [1] dissection levels of the order, [2] base node, [3] phases,
 * [4] factorisation levels, [5] estimated factorisation us, [6] tasks, [7] most tasks in one level,
 * [8] / [9] / [10] X_PART / X_SUB / X_SEP doubles per trial, [11] / [12] / [13] their group sizes, [14] n_aug,
 * [15] blocked back-solve steps. */
PTZBA_EXPORT int ptzba_dist_plan_summary(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world,
                                         int32_t rank, int64_t* out16);
/* host only: rank `rank`'s whole rank-tree plan (CPU replay in the tests): pos_out [n_pose], tasks (int4 records),
 * level offsets, phases_out [6 per phase] = {first level, end level, exchange kind, group first rank, group size,
 * exchanged tiles}, xt_out = every phase's exchanged tiles (ti, tj) concatenated.  counts: [0] tasks, [1] levels,
 * [2] n_aug, [3] phases, [4] exchanged tiles; null outputs only query the counts. */
PTZBA_EXPORT int ptzba_dist_plan_export(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world,
                                        int32_t rank, int32_t* pos_out, int32_t* tasks_out, int64_t tasks_cap,
                                        int32_t* level_off_out, int64_t levels_cap, int32_t* phases_out,
                                        int32_t phases_cap, int32_t* xt_out, int64_t xt_cap, int64_t* counts);
/* host only: the phases of rank `rank` of `world` (n_out of them, 0 when the solve is replicated), out[5 k ..] =
 * {exchange kind before the phase, group first rank, group size, first frame, end frame}; out may be NULL to count */
PTZBA_EXPORT int ptzba_dist_rank_phases(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world,
                                        int32_t rank, int32_t* out, int32_t cap, int32_t* n_out);
PTZBA_EXPORT int ptzba_partition_landmarks(int32_t n_pose, int32_t n_landmark, int64_t n_obs, const int32_t* obs_frame,
                                           const int32_t* obs_landmark, int32_t n_fixed, int32_t world,
                                           int32_t* rank_of_landmark, int32_t* mode_out, int32_t* split_out);
/* Host only (round 6): the planner's predicted cost per LM trial of the two forms of a `world`-rank solve -- the rank tree
 * (ptzba_partition_landmarks' part-owned split) and the replicated solve (contiguous landmark blocks, one all-reduce of the
 * packed system) -- as the slowest rank's factorisation estimate plus its collectives, each a ring all-reduce
 * alpha_us + 2 (p - 1) / p * bytes / (link_gbs GB/s).  out8: [0] tree us (0: no tree), [1] replicated us, [2] / [3] their
 * factorisation us, [4] / [5] the tree rank's collectives and doubles per trial, [6] replicated doubles, [7] the form
 * with the smaller estimate (1 tree, 0 replicated).  ptzba.choose_dist_form and bench.py --gpus N use it. */
PTZBA_EXPORT int ptzba_dist_form_estimate(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world,
                                          double alpha_us, double link_gbs, double* out8);

/* per-iteration scalars read back after ptzba_step (all fp64):
 * [0] cost at the current state, [1] cost at the trial state, [2] predicted reduction,
 * [3] |delta|^2, [4] |x|^2, [5] factorisation status (0 ok, >0 not positive definite),
 * [6] max |gradient| (unscaled), [7] reserved */
#define PTZBA_NSCALARS 8

/* ---------------- lifecycle ---------------- */
PTZBA_EXPORT ptzba_handle ptzba_new(int device);
PTZBA_EXPORT void ptzba_delete(ptzba_handle h);
PTZBA_EXPORT const char* ptzba_last_error(void);
PTZBA_EXPORT const char* ptzba_version(void);
/* Run all work of the handle on this hipStream_t, e.g. torch.cuda.current_stream().cuda_stream, so
 * collectives issued on that stream are ordered with the handle's kernels.  NULL is the default
 * (null) stream, which is what torch's current stream usually is.  A new handle uses a private
 * non-blocking stream; ptzba_use_own_stream returns to it. */
PTZBA_EXPORT int ptzba_set_stream(ptzba_handle h, void* hip_stream);
PTZBA_EXPORT int ptzba_use_own_stream(ptzba_handle h);

/* ---------------- problem ---------------- */
/* Pair-form observation records in the reference residual order: record 2m is (frame i, landmark l,
 * keypoint of i), record 2m+1 is (frame j, landmark l, keypoint of j) of match m
 * (bundle_adjustment.py:67-99).  obs_xy is [n_obs][2]; obs_weight may be NULL (all 1) or hold
 * integer multiplicities of de-duplicated records. */
PTZBA_EXPORT int ptzba_set_problem(ptzba_handle h, int32_t n_pose, int32_t n_landmark, int64_t n_obs,
                                   const int32_t* obs_frame, const int32_t* obs_landmark,
                                   const double* obs_xy, const double* obs_weight, double u, double v,
                                   const ptzba_problem_opts* opts);
/* structural counts: [0] n_pose [1] n_landmark [2] n_obs [3] n_segments (unique frame,landmark)
 * [4] reduced-system size [5] landmarks with observations [6] max segments per landmark
 * [7] bytes of device memory held */
PTZBA_EXPORT int ptzba_problem_info(ptzba_handle h, int64_t* info8);
/* host phase times of the last ptzba_set_problem (sort, segments, K2 structure, plan, uploads ...): names[k] (static
 * strings) and ms[k] for k < min(cap, *n_out); *n_out = the number of phases recorded */
PTZBA_EXPORT int ptzba_setup_timing(ptzba_handle h, int32_t cap, const char** names, double* ms, int32_t* n_out);
/* solver layout: [0] n_aug (system rows incl. padding), [1] ld, [2] factorisation launches (levels),
 * [3] ordering actually used (PTZBA_ORDER_*) | dissection levels << 8 (0 natural, 1 or 2), [4] back-substitution form (0 lookahead, 1 left-looking:
 * systems whose lists exceed LDS), [5] dense landmark x frame slots, [6] Schur work items,
 * [7] factor pattern tiles */
PTZBA_EXPORT int ptzba_solver_info(ptzba_handle h, int64_t* info8);

/* residual r[2*n_obs] = projection - observation, record order (== _compute_residual) at
 * x_full = [3*n_pose poses | 2*n_landmark rays] (fp64 host). Uses the handle's precision. */
PTZBA_EXPORT int ptzba_residual(ptzba_handle h, const double* x_full, double* r_out);

/* ---------------- state ---------------- */
PTZBA_EXPORT int ptzba_set_state(ptzba_handle h, const double* ptz /*3*n_pose*/, const double* rays /*2*n_landmark*/);
PTZBA_EXPORT int ptzba_get_state(ptzba_handle h, double* ptz, double* rays);
/* Device-resident restart point: save_state snapshots the current state on the device, restore_state
 * copies it back and resets the Marquardt scaling (as set_state does) -- both stream-ordered, no host
 * transfer or synchronisation (restarting a solve from x0 without a PCIe upload). */
PTZBA_EXPORT int ptzba_save_state(ptzba_handle h);
PTZBA_EXPORT int ptzba_restore_state(ptzba_handle h);

/* ---------------- one Levenberg-Marquardt iteration, split at the exchange points -------------
 * Single GPU:  ptzba_linearize; loop { ptzba_step(lambda); ptzba_read_scalars; ptzba_accept(ok) }.
 * Multi-GPU: with a communicator or hook attached (ptzba_attach_comm / ptzba_set_exchange_hook below) the
 * same calls run the exchanges themselves.  Without one, a replicated sharded solve may still use the
 * caller's own protocol: after ptzba_build_reduced the caller all-reduces (sum) the exchange buffer's
 * reduced system, then ptzba_solve_reduced, then all-reduces the partial scalars, then ptzba_accept.
 * ptzba_step == build_reduced + solve_reduced. */
PTZBA_EXPORT int ptzba_linearize(ptzba_handle h);
PTZBA_EXPORT int ptzba_build_reduced(ptzba_handle h, double lambda);
PTZBA_EXPORT int ptzba_solve_reduced(ptzba_handle h);
/* Device-driven Levenberg-Marquardt: the accept/reject decisions, damping update and termination
 * tests of the host loop (ptzba.LMSolver; scipy common.py:705-718 rules) run on the device, so trials
 * queue back to back.  Sequence: lm_start (linearise at the current state) [all-reduce scalars];
 * lm_init; then per trial k: lm_build [all-reduce system]; lm_solve [all-reduce scalars];
 * lm_decide(k).  lm_wait(k) blocks until trial k's decision is on the host (a ring of 4 records: wait
 * for trial k before deciding trial k + 4).  Enqueueing trial k + 1's build before waiting for trial k
 * hides the host round trip; a build after the final decision is harmless.  The state is double-buffered on
 * the device (an accepted trial is committed by the decision itself); lm_wait of the final decision makes it the
 * state ptzba_get_state / ptzba_save_state see, so every decided trial must be waited for. */
typedef struct {
  double ftol, xtol, gtol;                    /* scipy's ftol/xtol/gtol tests (gtol <= 0: off) */
  double lambda0, min_lambda, max_lambda;     /* Marquardt damping: start, floor, give-up bound.  lambda0 =
                                                 min_lambda (1e-12, the default) starts with Gauss-Newton steps, as
                                                 scipy's trf does while its step lies inside the trust region */
  int32_t max_iter, max_retries, gauss_newton; /* accepted iterations; rejections in a row; lambda0 = 0 GN */
  /* huber loss only: the records' curvature weight beyond the unit is rho' (IRLS, a majoriser of the loss) until an
   * accepted step was predicted to reduce the cost by less than curvature_switch of it; from then on huber_curvature * rho' (the
   * loss's own Newton curvature is 0 there, scipy's robust scaling; floored), the current point re-linearised at
   * once.  curvature_switch = 0 or huber_curvature = 1: IRLS throughout.  Defaults 0.1 / 0.25.  ABI (ptzba_version
   * 0.2): these two fields were added after the 9-field struct of 0.1; they are read for the Huber loss only and
   * huber_curvature = 0 selects the default 0.1, so a caller that zero-fills them keeps IRLS throughout. */
  double huber_curvature, curvature_switch;
} ptzba_lm_opts;
/* termination status (scipy least_squares numbering where it has one): DAMPING = the trial was rejected at
 * every damping up to max_lambda, i.e. no cost decrease is resolvable any more (scipy's trf ends such a run
 * through its xtol test once the trust radius collapses); FAILED = max_retries rejections in a row */
enum {
  PTZBA_STATUS_FAILED = -1,
  PTZBA_STATUS_MAX_ITER = 0,
  PTZBA_STATUS_GTOL = 1,
  PTZBA_STATUS_FTOL = 2,
  PTZBA_STATUS_XTOL = 3,
  PTZBA_STATUS_DAMPING = 5
};
typedef struct {
  double cost, initial_cost, lambda;
  int32_t iterations, nfev, trials, retries, status, done, accepted;  /* status: PTZBA_STATUS_* */
} ptzba_lm_record;
PTZBA_EXPORT int ptzba_lm_start(ptzba_handle h);
PTZBA_EXPORT int ptzba_lm_init(ptzba_handle h, const ptzba_lm_opts* opts);
PTZBA_EXPORT int ptzba_lm_build(ptzba_handle h);
PTZBA_EXPORT int ptzba_lm_solve(ptzba_handle h);
PTZBA_EXPORT int ptzba_lm_decide(ptzba_handle h, int trial);
PTZBA_EXPORT int ptzba_lm_wait(ptzba_handle h, int trial, ptzba_lm_record* out);
/* One-shot solve (single process): ptz_inout [3*n_pose] / rays_inout [2*n_landmark] carry x0 in and the
 * optimum out (left unchanged on failure); opts NULL = the reference's option set (ftol 1e-4, xtol 1e-8,
 * gtol off, 100 iterations).  Runs the device-driven LM above to termination.  Replaces the optimizer
 * call of bundle_adjustment.py:200-202 and the empty file-based C stub bundle_adjustment_opt
 * (rf_map/python_package/backup/bundle_adjustment_python.hpp:21-24). */
typedef struct {
  double cost, initial_cost, time_s;
  int32_t iterations, nfev, trials, status;  /* status as ptzba_lm_record */
} ptzba_report;
PTZBA_EXPORT int ptzba_solve(ptzba_handle h, double* ptz_inout, double* rays_inout, const ptzba_lm_opts* opts,
                             ptzba_report* report);
/* The same solve on the device-resident state (no host state transfer): restore != 0 first restores the
 * ptzba_save_state snapshot.  The state stays on the device (ptzba_get_state reads it).  Back-to-back solves
 * from C keep the restart's host reaction out of the device's timeline (bench.py's restart loop). */
PTZBA_EXPORT int ptzba_solve_resident(ptzba_handle h, int restore, const ptzba_lm_opts* opts, ptzba_report* report);
/* host-driven LM (ptzba_linearize / ptzba_step): the huber curvature weight (in (0, 1], units of rho' beyond the
 * unit) of the following linearisations; set_problem resets it to 1 (IRLS) */
PTZBA_EXPORT int ptzba_set_huber_curvature(ptzba_handle h, double hc);
/* Which front builds the record arrays in the following ptzba_set_problem calls of this handle (round 6): the device
 * front (one rocPRIM radix sort + segment / record kernels) from min_records records on, the host's counting sorts
 * below.  0: always the device, INT64_MAX: never, -1: the default (64K records since round 6, 4M before: configs 3 and 4
 * and a sliding window's ~170K records on the device, the small drop-in problems on the host).  Both fronts produce the
 * same arrays bit for bit. */
PTZBA_EXPORT int ptzba_set_setup_front(ptzba_handle h, int64_t min_records);
PTZBA_EXPORT int ptzba_step(ptzba_handle h, double lambda);
PTZBA_EXPORT int ptzba_read_scalars(ptzba_handle h, double* out /*PTZBA_NSCALARS*/);
PTZBA_EXPORT int ptzba_accept(ptzba_handle h, int accept);
/* Device pointers of the exchange regions (fp64): reduced system (ld*ld + 3*ld doubles, ld = the padded
 * system dimension: the lower triangle of S row-major in the system order, then b, g_pose and diag U)
 * and the additive partial scalars (PTZBA_NSCALARS). */
PTZBA_EXPORT int ptzba_exchange(ptzba_handle h, void** sys_ptr, int64_t* sys_count, void** scal_ptr);
/* Packed exchange for sharded solves: a contiguous device buffer (fp64, *count doubles) holding only
 * the tiles of the reduced system the Schur kernel can write, then b | g_pose | dU.  Sequence per
 * iteration: ptzba_build_reduced -> ptzba_pack -> all-reduce(sum) of the buffer -> ptzba_unpack ->
 * ptzba_solve_reduced.  Pack/unpack are queued on the handle's stream. */
PTZBA_EXPORT int ptzba_exchange_packed(ptzba_handle h, void** buf, int64_t* count);
PTZBA_EXPORT int ptzba_pack(ptzba_handle h);
PTZBA_EXPORT int ptzba_unpack(ptzba_handle h);
/* ---------------- exchanges of a multi-GPU solve (done by the library) ----------------
 * Kinds (all are in-place SUMS over ranks of fp64 device buffers, on the handle's stream):
 *   PTZBA_X_SYS  replicated solve: the packed reduced system (all ranks);
 *   PTZBA_X_PART part-owned solve: a shared leaf's columns, inside the leaf's rank group;
 *   PTZBA_X_SUB  part-owned solve: an inner separator's columns, inside its node's rank group;
 *   PTZBA_X_SEP  part-owned solve: the root separator's columns, all ranks;
 *   PTZBA_X_SCAL partial LM scalars, all ranks (8 doubles replicated, 16 part-owned).
 * ptzba_exchange_group tells the group [r0, r0 + nr) of a kind on this rank (a hook sums over exactly it).
 * With an exchange set, ptzba_linearize / ptzba_build_reduced / ptzba_solve_reduced / ptzba_lm_* /
 * ptzba_solve run them internally at the right points: the caller issues no collective.  Two ways:
 *   ptzba_attach_comm: the library's own RCCL communicator (ptzba_comm_new from an RCCL unique id);
 *   ptzba_set_exchange_hook: a callback (e.g. torch.distributed over gloo for single-device rehearsals).
 * Neither set: no exchange (single GPU, or the caller's own protocol through ptzba_exchange*). */
enum { PTZBA_X_SYS = 0, PTZBA_X_PART = 1, PTZBA_X_SEP = 2, PTZBA_X_SCAL = 3, PTZBA_X_SUB = 4 };
typedef int (*ptzba_exchange_fn)(void* ctx, int32_t kind, double* dev_buf, int64_t count, void* hip_stream);
PTZBA_EXPORT int ptzba_set_exchange_hook(ptzba_handle h, ptzba_exchange_fn fn, void* ctx);
/* library-owned RCCL communicator ("a handle per rank, created with an RCCL unique id").
 * RCCL is loaded at run time (dlopen of librccl.so.1, or the path in PTZBA_RCCL_LIB).  Rank 0 calls
 * ptzba_comm_unique_id and ships the PTZBA_UNIQUE_ID_BYTES bytes to the other ranks (any channel); every
 * rank then calls ptzba_comm_new (collective).  device < 0: use the current HIP device. */
#define PTZBA_UNIQUE_ID_BYTES 128
typedef struct ptzba_comm_s* ptzba_comm;
PTZBA_EXPORT int ptzba_comm_unique_id(void* id_out);
PTZBA_EXPORT ptzba_comm ptzba_comm_new(int device, const void* unique_id, int32_t rank, int32_t world);
PTZBA_EXPORT void ptzba_comm_delete(ptzba_comm c);
/* collective over the parent: ranks of equal color form a new communicator, ordered by key */
PTZBA_EXPORT ptzba_comm ptzba_comm_split(ptzba_comm parent, int32_t color, int32_t key);
PTZBA_EXPORT int ptzba_comm_info(ptzba_comm c, int32_t* rank, int32_t* world);
/* in-place sum of count fp64 values of a device buffer on hip_stream (NULL: default stream) */
PTZBA_EXPORT int ptzba_comm_allreduce(ptzba_comm c, double* dev_buf, int64_t count, void* hip_stream);
/* the handle all-reduces through comm (not owned; NULL detaches).  A part-owned handle splits its rank groups'
 * communicators off comm at its first exchange (collective: every rank of the solve reaches it). */
PTZBA_EXPORT int ptzba_attach_comm(ptzba_handle h, ptzba_comm comm);
/* [0] mode (1 part-owned, 0 replicated), [1] base node of the rank tree (-1 replicated), [2] ranks sharing the
 * base, [3] first rank of the base's group, [4] root-separator exchange doubles, [5] shared-leaf exchange doubles
 * (0: none), [6] system exchange doubles (replicated), [7] scalar exchange doubles */
PTZBA_EXPORT int ptzba_dist_info(ptzba_handle h, int64_t* info8);
/* this rank's exchanges per LM trial, in order: out[4 k .. 4 k + 3] = {kind, group first rank, group size, doubles}
 * (out may be NULL to count; cap = entries out holds) */
PTZBA_EXPORT int ptzba_dist_exchanges(ptzba_handle h, int64_t* out, int32_t cap, int32_t* n_out);
/* every rank group of the rank tree below the whole world, {first rank, size, tree depth} each (the same list on
 * every rank: a hook creates its groups from it) */
PTZBA_EXPORT int ptzba_dist_groups(ptzba_handle h, int32_t* out, int32_t cap, int32_t* n_out);
/* the group {first rank, size} exchange `kind` runs over on this rank (the whole world for X_SEP / X_SCAL / X_SYS) */
PTZBA_EXPORT int ptzba_exchange_group(ptzba_handle h, int32_t kind, int32_t* r0_nr);
/* frames whose pose this rank's solve updates (its part and C; all frames when replicated): mask [n_pose] */
PTZBA_EXPORT int ptzba_owned_frames(ptzba_handle h, uint8_t* mask_out);

/* wait for all queued work of the handle */
PTZBA_EXPORT int ptzba_sync(ptzba_handle h);
/* average device time (ms) per launch of the kernel groups [K1 linearisation, Schur build, Cholesky
 * solve, back-substitution], measured with HIP events on the handle's stream; launches timed.
 * reset: `enable` bits 0-3 select the groups to time (1 K1, 2 Schur, 4 Cholesky, 8 back-subst.;
 * 0 off); bits 8-15 = sampling stride s (0/1: every launch): a group records its event pair around
 * every s-th launch only.  Each recorded event adds a few-microsecond gap to the stream.
 * PTZBA_TIME_FLUSH (bit 16): cold-cache K1 timing -- before each timed K1 launch a kernel writes a
 * 1 GiB scratch buffer (larger than L2 + the 256 MB Infinity Cache), outside the timed event pair; the
 * caches are left full of dirty lines, whose write-backs then run during the timed launch.
 * PTZBA_TIME_FLUSH_READ (bit 17, with bit 16): the scratch buffer is READ instead -- the caches hold
 * clean unrelated lines, so the timed launch pays its own HBM traffic only. */
#define PTZBA_TIME_COMM 0x10  /* enable bit 4: an event pair around every exchange (ptzba_comm_times) */
#define PTZBA_TIME_FLUSH 0x10000
#define PTZBA_TIME_FLUSH_READ 0x20000
PTZBA_EXPORT int ptzba_kernel_times(ptzba_handle h, double* ms_out /*4*/, int64_t* count_out /*4*/);
PTZBA_EXPORT int ptzba_reset_kernel_times(ptzba_handle h, int enable);
/* The exchanges timed since the last ptzba_reset_kernel_times with PTZBA_TIME_COMM (bit 4): per exchange its kind
 * (PTZBA_X_*), its size in doubles and the elapsed ms between the events recorded on the handle's stream around it
 * (the collective's kernel, or a hook's stream work); the first min(cap, *n_out) records (up to 2048 per reset).
 * New in round 6 (a multi-rank run reports what its collectives cost). */
PTZBA_EXPORT int ptzba_comm_times(ptzba_handle h, int32_t cap, int32_t* kinds, int64_t* doubles, double* ms,
                                  int32_t* n_out);

/* ---------------- camera model (batched, device-resident computation) ---------------- */
PTZBA_EXPORT int ptz_ray_to_image(int device, int64_t n, double u, double v, const double* f,
                                  const double* cam_pan, const double* cam_tilt, const double* theta,
                                  const double* phi, double* x_out, double* y_out);
PTZBA_EXPORT int ptz_image_to_ray(int device, int64_t n, double u, double v, const double* f,
                                  const double* cam_pan, const double* cam_tilt, const double* x,
                                  const double* y, double* theta_out, double* phi_out);
/* PTZCamera matrix model with optional 6-parameter displacement (NULL = zeros); one camera, n rays */
PTZBA_EXPORT int ptz_project_rays(int device, int64_t n, double u, double v, double f, double pan,
                                  double tilt, const double* displacement6, const double* rays /*[n][2]*/,
                                  double* xy_out /*[n][2]*/);
PTZBA_EXPORT int ptz_back_project_rays(int device, int64_t n, double u, double v, double f, double pan,
                                       double tilt, const double* displacement6, const double* xy,
                                       double* rays_out);
/* PtzSlam.compute_h_jacobian: H [2n][3+2n] row-major, dense, as the reference */
PTZBA_EXPORT int ptz_h_jacobian(int device, int64_t n, double u, double v, double f, double pan,
                                double tilt, const double* displacement6, const double* rays, double* H_out);

/* ---------------- pose-only refinement (relocalization.py:22-40, 186) ----------------
 * Levenberg-Marquardt over (pan, tilt, f) with the rays fixed, residual = from_ray_to_image(ray) -
 * point (transformation.py:99-135), one workgroup per hypothesis on the device.  Hypotheses share the
 * n_corr correspondences, or hypothesis h uses subset_index[subset_offsets[h] .. subset_offsets[h+1])
 * (both NULL: all).  ptz_inout [n_hyp][3] holds the initial poses and receives the refined ones;
 * cost_out = 0.5 sum rho(r^2), iters_out = accepted iterations, status_out as ptzba.LMSolver
 * (2 ftol, 3 xtol, 0 max_iter, -1 no decrease).  Any output pointer may be NULL. */
typedef struct {
    int32_t max_iter;  /* default 100 */
    int32_t loss;      /* PTZBA_LOSS_LINEAR | PTZBA_LOSS_HUBER */
    double ftol;       /* the reference's 1e-4 */
    double xtol;       /* scipy default 1e-8 */
    double f_scale;
} ptz_refine_opts;
PTZBA_EXPORT int ptz_refine_poses(int device, int32_t n_hyp, double* ptz_inout, int64_t n_corr,
                                  const double* rays, const double* points, double u, double v,
                                  const int64_t* subset_offsets, const int32_t* subset_index,
                                  const ptz_refine_opts* opts, double* cost_out, int32_t* iters_out,
                                  int32_t* status_out);

/* ---------------- host bookkeeping (native) ---------------- */
/* ---------------- feature front-end (image_process.py:178-234, 418-441) ----------------
 * Stateless, synchronous entry points (no handle).  They keep per-device work buffers across calls and hold
 * a per-device lock while using them: safe to call from several host threads (calls on one device run one
 * at a time).  The ptzba_* / ptzekf_* handles are NOT thread-safe: one call at a time per handle. */
/* Brute-force 2-nearest-neighbour matching in L2 (cv.BFMatcher().knnMatch(des1, des2, k=2)): for each of the
 * n1 query descriptors the two nearest of the n2 train descriptors, idx_out[2*i+0/1] (ties: lower index
 * first; -1 when n2 < 2) and their L2 distances dist_out[2*i+0/1].  Descriptors are fp32 rows of `dim`.
 * The ratio test of match_sift_features (m < 0.7 n) runs on the host. */
PTZBA_EXPORT int ptz_match_knn2(int device, int64_t n1, int64_t n2, int32_t dim, const float* des1, const float* des2,
                                int32_t* idx_out, float* dist_out);
/* Device-resident descriptor sets for repeated matching (a sliding keyframe window: image_process.py:509-667 run per
 * keyframe over the window).  ptz_desc_put uploads n fp32 rows of `dim` under a caller-chosen key (replacing what the
 * key held); ptz_desc_drop frees the listed keys (unknown keys are ignored).  ptz_match_knn2_sets = ptz_match_knn2
 * of the concatenation of the query sets (in the order given) against the train set, bit for bit; n_rows must equal
 * the query sets' total row count, idx_out / dist_out hold 2 entries per row. */
PTZBA_EXPORT int ptz_desc_put(int device, uint64_t key, int64_t n, int32_t dim, const float* des);
PTZBA_EXPORT int ptz_desc_drop(int device, int32_t n_keys, const uint64_t* keys);
PTZBA_EXPORT int ptz_match_knn2_sets(int device, int32_t n_sets, const uint64_t* query_keys, uint64_t train_key,
                                     int64_t n_rows, int32_t* idx_out, float* dist_out);
/* The batched SIFT matcher of a new keyframe against resident sets sharing one train set (image_process
 * match_sift_features_batch): ptz_match_knn2_sets, Lowe's ratio test d1 < 0.7 d2 (float32) per query set, the
 * survivors' points from query_xy (the query sets' keypoints concatenated, [rows, 2]) and train_xy ([train_rows, 2]),
 * one ptz_homography_ransac_batch (threshold, n_hyp, seed) over the sets with more than 8 survivors, and the inliers
 * as (query row, train row) pairs: out_off[n_sets + 1] into out_i1 / out_i2 (capacity: the query rows in total);
 * status_out[s] = 1 when set s had 8 or fewer survivors (no pairs), else 0. */
PTZBA_EXPORT int ptz_match_sets_ransac(int device, int32_t n_sets, const uint64_t* query_keys, const int64_t* query_rows,
                                       uint64_t train_key, int64_t train_rows, const double* query_xy,
                                       const double* train_xy, double threshold, int32_t n_hyp, uint64_t seed,
                                       int32_t* status_out, int64_t* out_off, int32_t* out_i1, int32_t* out_i2);
/* Homography RANSAC (cv.findHomography(..., RANSAC, threshold) as called by homography_ransac): n_hyp
 * hypotheses from 4-point samples keyed by (seed, hypothesis, draw), DLT in Hartley-normalised coordinates,
 * the hypothesis with most inliers (reprojection error < threshold px; ties: lowest index), a linear
 * least-squares refit on its inliers, and the final inlier mask (mask_out[n], 1 = inlier), H_out[9]
 * (row-major, H[8] = 1) and the inlier count.  n >= 4. */
PTZBA_EXPORT int ptz_homography_ransac(int device, int64_t n, const double* pts1, const double* pts2, double threshold,
                                       int32_t n_hyp, uint64_t seed, uint8_t* mask_out, double* H_out,
                                       int32_t* n_inliers_out);
/* n_sets independent RANSACs in one call (a new keyframe's pairwise matches, bundle_adjustment.py:145 ->
 * image_process.py:178-234 once per pair): set s = correspondences [off[s], off[s + 1]) of pts1 / pts2 (off[0] =
 * 0, each set >= 4); mask_out[off[n_sets]], H_out[9 n_sets], n_inliers_out[n_sets].  Per set the result of
 * ptz_homography_ransac with the same seed, bit for bit. */
PTZBA_EXPORT int ptz_homography_ransac_batch(int device, int32_t n_sets, const int64_t* off, const double* pts1,
                                             const double* pts2, double threshold, int32_t n_hyp, uint64_t seed,
                                             uint8_t* mask_out, double* H_out, int32_t* n_inliers_out);
/* Pyramidal Lucas-Kanade point tracking (cv.calcOpticalFlowPyrLK(img, next_img, points, None, winSize=(31, 31))
 * as called by optical_flow_matching, image_process.py:393-415).  img0/img1: 8-bit grey, width x height,
 * row-major.  Pyramid of `levels` (cv.pyrDown: 5x5 binomial, reflect-101), Scharr gradients, window `win`
 * (odd, <= 31), at most max_iter Newton steps per level, stop when the step is below eps px; bilinear
 * samples clamp to the image.  Per point: pts1_out [n][2]; status_out 1 = tracked (the window's smaller
 * structure-tensor eigenvalue / win^2 >= min_eig at every level and the result inside the image);
 * err_out = mean |I - J| over the window at the final position (the reference keeps err < 20). */
PTZBA_EXPORT int ptz_lk_track(int device, int32_t width, int32_t height, const uint8_t* img0, const uint8_t* img1,
                              int64_t n, const float* pts0, int32_t levels, int32_t win, int32_t max_iter, double eps,
                              double min_eig, float* pts1_out, uint8_t* status_out, float* err_out);

/* Hamming nearest neighbours both ways (cv.BFMatcher(cv.NORM_HAMMING, crossCheck=True).match of match_orb_features /
 * match_latch_features, image_process.py:237-310): binary descriptors of nbytes (multiple of 4, <= 64);
 * idx12[i] / dist12[i] = the nearest des2 row of des1 row i and its bit distance, idx21[j] the nearest des1 row of
 * des2 row j (ties: lower index; -1 when the other set is empty).  Cross-checked matches: i with idx21[idx12[i]] == i. */
PTZBA_EXPORT int ptz_match_hamming(int device, int64_t n1, int64_t n2, int32_t nbytes, const uint8_t* des1,
                                   const uint8_t* des2, int32_t* idx12, int32_t* dist12, int32_t* idx21);
/* SIFT keypoints and descriptors (cv.xfeatures2d.SIFT_create(nfeatures).detectAndCompute as detect_compute_sift calls
 * it, image_process.py:56-79): img 8-bit grey width x height; OpenCV's defaults (image doubled, 3 layers per octave,
 * sigma 1.6, contrast 0.04, edge 10).  Keypoints ordered by (-response, y, x, angle) and cut to nfeatures (> 0;
 * 0 keeps all); *n_out = their number, of which the first min(n, max_kp) are written: kp_out [.][4] = (x, y, size,
 * angle in degrees), response_out [.] (may be NULL), des_out [.][128] (integer values 0..255 as float).
 * A call on the same image content as the previous call on this device (a frame detected with 500 features, then
 * with 1500 as a keyframe) reuses that call's pyramid and oriented keypoints: the same result, selection and
 * descriptors only (PTZ_SIFT_REUSE=0 disables it). */
PTZBA_EXPORT int ptz_sift(int device, int32_t width, int32_t height, const uint8_t* img, int32_t nfeatures, int32_t max_kp,
                          float* kp_out, float* response_out, float* des_out, int32_t* n_out);

/* Shi-Tomasi corner response (cv.cornerMinEigenVal(img, blockSize=3, ksize=3): the measure of cv.goodFeaturesToTrack
 * in detect_harris_corner_grid, image_process.py:352-390): eig_out [height][width] float32; locmax_out (may be NULL)
 * [height][width] = 1 where eig > 0 is the maximum of its 3x3 neighbourhood and the pixel is not on the image's
 * one-pixel border (goodFeaturesToTrack's candidates after its dilation).  The per-cell threshold, the ordering
 * and the minimum-distance selection run on the host (image_process.detect_harris_corner_grid). */
PTZBA_EXPORT int ptz_corner_min_eig(int device, int32_t width, int32_t height, const uint8_t* img, float* eig_out,
                                    uint8_t* locmax_out);

/* ORB / LATCH detection + description (image_process.py:105-155: cv.ORB_create(nfeatures).detect + compute, and
 * LATCH_create(64).compute on those keypoints): 8-level pyramid (scale 1.2), FAST-9 (threshold 20) with 3x3
 * non-maximum suppression and the 31-px edge, per-level retain-best by FAST score (2 n_l) then Harris response
 * (n_l, OpenCV's geometric split), intensity-centroid angle; descriptor 0 = ORB rBRIEF (32 bytes, 7x7 sigma-2
 * blurred level image), 1 = LATCH (64 bytes, SSD triplets on the 13x13 sigma-2 blurred image, 27-px border).
 * The sampling tables are generated (OpenCV's learned ones are not available: descriptors are not OpenCV's bits,
 * see csrc/orb.hip).  kp_out [max_kp][6] = x, y (level-0 pixels), size, angle (deg), response (Harris), octave;
 * des_out [max_kp][32 or 64].  *n_out = keypoints found (all ties at the per-level cuts kept, as OpenCV): when it
 * exceeds max_kp only max_kp are written; call again with a larger buffer.  Order: level, response desc, y, x. */
PTZBA_EXPORT int ptz_orb(int device, int32_t width, int32_t height, const uint8_t* img, int32_t nfeatures,
                         int32_t descriptor, int32_t max_kp, float* kp_out, uint8_t* des_out, int32_t* n_out);

/* Coupling window of a record set (host only, O(n_obs)): win_out[f] = the highest frame that shares a
 * landmark with frame f (>= f).  Computed over ALL records it is the frame_win_hi every rank of a
 * landmark-sharded solve passes in ptzba_problem_opts. */
PTZBA_EXPORT int ptzba_coupling_window(int32_t n_pose, int32_t n_landmark, int64_t n_obs, const int32_t* obs_frame,
                                       const int32_t* obs_landmark, int32_t* win_out);
/* First-seen landmark ids over ordered pair match lists (image_process.py:611-639).
 * pair_i/pair_j/pair_count: n_pairs; idx_a/idx_b: concatenated match keypoint indices.
 * kp_count[n_frames]: keypoints per frame.  Output landmark id per match (of the src keypoint) and
 * the landmark count; *n_inconsistent counts the reference's "in-consistent matching" warnings. */
PTZBA_EXPORT int ptzba_build_landmarks(int32_t n_frames, const int64_t* kp_count, int64_t n_pairs,
                                       const int32_t* pair_i, const int32_t* pair_j,
                                       const int64_t* pair_count, const int64_t* idx_a,
                                       const int64_t* idx_b, int64_t* landmark_out, int64_t* n_landmark,
                                       int64_t* n_inconsistent);

/* ---------------- correspondence -> packed-observation builder (builder.cpp) ----------------
 * Interpreter-defined orderings the reference's BA results depend on, reproduced bit for bit.
 *
 * ptz_py_shuffle_prefix <- random.shuffle(rand_list)[0:200] (image_process.py:592-597) on the GLOBAL
 *   Mersenne Twister: mt_state[625] = random.getstate()[1] (624 words + index), updated in place for
 *   random.setstate().  Shuffles range(lens[l]) for each list in order and writes the first
 *   min(lens[l], keep) entries of each to out (concatenated). */
PTZBA_EXPORT int ptz_py_shuffle_prefix(uint32_t* mt_state, int64_t n_lists, const int64_t* lens, int64_t keep,
                                       int64_t* out);
/* Iteration order of CPython set() built from the tuple sequence (a[k], b[k]) (non-negative ints). */
PTZBA_EXPORT int ptz_set_order_pairs(int64_t n, const int64_t* a, const int64_t* b, int64_t* out_a,
                                     int64_t* out_b, int64_t* n_out);
/* Keyframe (local keypoint, landmark) lists <- bundle_adjustment.py:218-239: for frame f the tuples
 * (src_pt_index[f][j], landmark_index[f][j]) for j ascending, then (dst_pt_index[j][f],
 * landmark_index[j][f]) for j ascending, de-duplicated in set() iteration order.  Matches are given
 * flat in pair order ((i, j) lexicographic, i < j): frames m_i/m_j, keypoints k1/k2, landmark lm.
 * Output: out_off[n_frames+1] CSR over out_local/out_global (each sized >= 2 n_matches). */
PTZBA_EXPORT int ptz_keyframe_features(int32_t n_frames, int64_t n_matches, const int32_t* m_i,
                                       const int32_t* m_j, const int64_t* k1, const int64_t* k2,
                                       const int64_t* lm, int64_t* out_off, int64_t* out_local,
                                       int64_t* out_global);
/* len() of each keyframe's ptz_keyframe_features list (distinct (local keypoint, landmark) pairs), without the
 * set() order: counts_out[n_frames]. */
PTZBA_EXPORT int ptz_keyframe_feature_counts(int32_t n_frames, int64_t n_matches, const int32_t* m_i, const int32_t* m_j,
                                             const int64_t* k1, const int64_t* k2, const int64_t* lm, int64_t* counts_out);
/* Pair-form records in _compute_residual order (bundle_adjustment.py:67-99): record 2k = (m_i, k1),
 * 2k+1 = (m_j, k2), both on landmark lm[k]; xy from the keypoint table kp_xy[kp_off[f] + k][2].
 * landmark_src_rec[l] = record of the src observation of the LAST match of landmark l, the one the
 * reference initialises the ray from (bundle_adjustment.py:186-195), -1 if none. */
PTZBA_EXPORT int ptz_pack_records(int32_t n_frames, int64_t n_matches, const int32_t* m_i, const int32_t* m_j,
                                  const int64_t* k1, const int64_t* k2, const int64_t* lm,
                                  const int64_t* kp_off, const double* kp_xy, int64_t n_landmark,
                                  int32_t* rec_frame, int32_t* rec_landmark, double* rec_xy,
                                  int64_t* landmark_src_rec);

/* ---------------- EKF tracking state (ptz_slam.py:21-71, 210-315, 376-384, 424-426) ----------------
 * A handle owns the ray landmarks [R][2] and the dense state covariance [(3+2R)][(3+2R)] (row-major,
 * order pan, tilt, f, theta_0, phi_0, ...) in device memory; the reference keeps them as the numpy
 * attributes PtzSlam.rays / PtzSlam.state_cov.  Same ownership rules as ptzba_*: caller-owned host
 * buffers are copied, device buffers belong to the handle, one HIP stream per handle. */
typedef struct ptzekf_ctx* ptzekf_handle;
PTZBA_EXPORT ptzekf_handle ptzekf_new(int device);
PTZBA_EXPORT void ptzekf_delete(ptzekf_handle h);
PTZBA_EXPORT int ptzekf_num_rays(ptzekf_handle h);
/* replaces assignments to PtzSlam.rays / .state_cov (init_system, ptz_slam.py:190-200) */
PTZBA_EXPORT int ptzekf_set_state(ptzekf_handle h, int32_t n_ray, const double* rays, const double* cov);
/* reads PtzSlam.rays / .state_cov back; either pointer may be NULL */
PTZBA_EXPORT int ptzekf_get_state(ptzekf_handle h, double* rays_out, double* cov_out);
/* predict step of tracking(): state_cov[0:3,0:3] += q (ptz_slam.py:425-426); q row-major 3x3 */
PTZBA_EXPORT int ptzekf_add_pose_cov(ptzekf_handle h, const double* q9);
/* PtzSlam.remove_rays (ptz_slam.py:291-315): np.delete semantics (negative indices wrap, duplicates ok) */
PTZBA_EXPORT int ptzekf_remove_rays(ptzekf_handle h, int64_t n, const int64_t* index);
/* PtzSlam.add_rays state growth (ptz_slam.py:376-384): append rays, zero rows/cols, var on the diagonal */
PTZBA_EXPORT int ptzekf_add_rays(ptzekf_handle h, int64_t n, const double* rays, double var);
/* PTZCamera.project_rays(self.rays, height, width) over the handle's rays (ptz_camera.py:212-234):
 * points strictly inside the image, in ray order; index_out as float like the reference.
 * ptz = (pan, tilt, f); xy_out [R][2] and index_out [R] sized for all rays; *count_out = visible. */
PTZBA_EXPORT int ptzekf_project_visible(ptzekf_handle h, double u, double v, const double* displacement6,
                                        const double* ptz, int32_t height, int32_t width, double* xy_out,
                                        double* index_out, int32_t* count_out);
/* PtzSlam.ekf_update (ptz_slam.py:210-289): predicted camera ptz_inout (pan, tilt, f) is replaced by
 * the updated one; observed keypoints obs_xy [n_obs][2] with global ray indices obs_index [n_obs]
 * (matched against the visible predicted rays with the reference's get_overlap_index walk,
 * util.py:75-97); observe_var = the reference's R = observe_var * I (0.1).  Rays and covariance are
 * updated in place on the device with the reference's write-back (:281-289).  velocity_out (3) =
 * K y [0:3] (:273); *n_matched_out = matched rays.  H P H^T + R is factored as L S L^T with a signed
 * diagonal S (it can be indefinite: the reference inverts it regardless); fails (state untouched) only
 * when it is singular. */
PTZBA_EXPORT int ptzekf_update(ptzekf_handle h, double u, double v, const double* displacement6,
                               double* ptz_inout, int64_t n_obs, const double* obs_xy, const int64_t* obs_index,
                               int32_t height, int32_t width, double observe_var, double* velocity_out,
                               int32_t* n_matched_out);

#ifdef __cplusplus
}
#endif
#endif /* PTZBA_H */
