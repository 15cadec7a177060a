// Kernel argument blocks and host-side launchers of libptzba (internal header).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptzba {

constexpr int K1_SEGW = 128;  // K1 segments per LDS window per wave
#ifndef K1_FT_LDS_N
#define K1_FT_LDS_N 384
#endif
// K1 stages its workgroup's frame range of the frame tables in LDS (5 x 8 B per frame) when the range holds at most this
// many frames, else the workgroup reads them from global memory.  Round 6: 640 -> 384 frames (15 KB instead of 25 KB),
// so five workgroups of four waves fit a CU's LDS (38 -> 27 KB per workgroup): 5 waves / SIMD instead of 4
constexpr int K1_FT_LDS = K1_FT_LDS_N;
// dense landmark x frame slot rows, packed (no padding: K1 writes and K2 reads 60 B per fp32 slot, not 80):
// W (3x2) in W_STRIDE reals, U (3x3 sym, 6) | g_pose (3) in UG_STRIDE reals; rows are only 4-B (fp32) / 8-B (fp64)
// aligned, so the vector accesses go through the element-aligned vector types below (dwordx4 / x2 on gfx950)
constexpr int W_STRIDE = 6, UG_STRIDE = 9;
typedef float f4e __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2e __attribute__((ext_vector_type(2), aligned(4)));
typedef double d2e __attribute__((ext_vector_type(2), aligned(8)));
template <typename real>
__device__ __forceinline__ void slot_load6(real (&x)[6], const real* __restrict__ p) {
  if constexpr (sizeof(real) == 4) {
    const f4e lo = *reinterpret_cast<const f4e*>(p);
    const f2e hi = *reinterpret_cast<const f2e*>(p + 4);
    x[0] = lo.x; x[1] = lo.y; x[2] = lo.z; x[3] = lo.w; x[4] = hi.x; x[5] = hi.y;
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const d2e d = *reinterpret_cast<const d2e*>(p + 2 * k);
      x[2 * k] = d.x; x[2 * k + 1] = d.y;
    }
  }
}
template <typename real>
__device__ __forceinline__ void slot_load9(real (&x)[9], const real* __restrict__ p) {
  if constexpr (sizeof(real) == 4) {
    const f4e a = *reinterpret_cast<const f4e*>(p), b = *reinterpret_cast<const f4e*>(p + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const d2e d = *reinterpret_cast<const d2e*>(p + 2 * k);
      x[2 * k] = d.x; x[2 * k + 1] = d.y;
    }
  }
  x[8] = p[8];
}
template <typename real>
__device__ __forceinline__ void slot_store6(real* p, const real (&x)[6]) {
  if constexpr (sizeof(real) == 4) {
    *reinterpret_cast<f4e*>(p) = f4e{x[0], x[1], x[2], x[3]};
    *reinterpret_cast<f2e*>(p + 4) = f2e{x[4], x[5]};
  } else {
#pragma unroll
    for (int k = 0; k < 3; ++k) *reinterpret_cast<d2e*>(p + 2 * k) = d2e{x[2 * k], x[2 * k + 1]};
  }
}
template <typename real>
__device__ __forceinline__ void slot_store9(real* p, const real (&x)[9]) {
  if constexpr (sizeof(real) == 4) {
    *reinterpret_cast<f4e*>(p) = f4e{x[0], x[1], x[2], x[3]};
    *reinterpret_cast<f4e*>(p + 4) = f4e{x[4], x[5], x[6], x[7]};
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<d2e*>(p + 2 * k) = d2e{x[2 * k], x[2 * k + 1]};
  }
  p[8] = x[8];
}
struct LinArgs {
  const int4* lm_work;           // [2 n_work] {landmark, s0, s1, first record}, {lm_meta}, heaviest first
  int n_work;
  const int32_t* lm_seg_begin;   // [n_lm+1]
  const int32_t* seg_frame;      // [n_seg]
  const int64_t* seg_rec_begin;  // [n_seg+1]
  const int32_t* rec_seg;        // [n_rec]
  const uint8_t* rec_key;        // [n_rec] segment - first segment of the landmark, mod K1_SEGW
  const void* rec_xy;            // [2 n_rec] real
  const void* rec_w;             // [n_rec] real or nullptr
  const void* ft;                // FrameTab<real>[n_pose]
  const void* rt;                // RayTab<real>[n_lm]
  const void* ft64;              // FrameTab<double>[n_pose]
  const void* rt64;              // RayTab<double>[n_lm]
  const double2* seg_base;       // [n_seg] base observation; records hold obs - base (real)
  double u, v, fs2, inv_fs2;
  double hcurv;                  // huber: curvature weight beyond the unit = hcurv * rho' (1: IRLS)
  const double* hcurv_dev;       // device-driven LM: the curvature weight from LMDev::hc instead (nullptr: hcurv)
  const int* run_if;             // nullptr, or: the launch exits at once unless *run_if != 0 (re-linearisation)
  void* ug_slot;                 // [n_slot][UG_STRIDE] real: U (6) | g_pose (3) (dense slots)
  void* w_slot;                  // [n_slot][W_STRIDE] real: W (6) at slot toff_l + frame - first_l
  const int4* lm_meta;           // [n_lm] {first frame, last frame, slot offset, 0}
  double* lm_out;                // [n_lm][8]
  // device-driven LM: the linearisation slot is chosen on the device -- with sel != nullptr the kernel writes
  // slot ((*sel) ^ sel_xor): 0 = ug_slot / w_slot / lm_out above, 1 = the *1 buffers
  void* ug_slot1;
  void* w_slot1;
  double* lm_out1;
  const int* sel;
  int sel_xor;
  // frames of the problem: with n_pose <= K1_FT_LDS every workgroup stages the fp64 frame tables in LDS before it
  // reads its work descriptors (off the descriptor's latency), so a segment's frame table is an LDS read instead
  // of a global load that depends on the segment's frame id
  int n_pose;
};

// K2 tiles: block of SCHUR_F1 consecutive free frames x chunk of 64 partner frames; work items are
// splits of a tile's landmark list.  Static structure built once by ptzba_set_problem.
constexpr int SCHUR_F1 = 32;
constexpr int SCHUR_LMAX = 512;  // landmarks per work item (split size cap)
// Single-GPU builds fold k_chol_prepare into the build: the prologue writes the constant diagonal entries
// (padding identity, augmented diagonal, identity below it) and resets info; k_schur_reduce writes the
// augmented row b^T and the pose damping (D_pose = max(D_pose, diag U); S_ff += lambda D_pose), the same
// values in the same order as the prepare launch.  pad == nullptr: not fused (multi-rank exchanges need the
// prepare after the sum).
struct FusedPrep {
  const uint8_t* pad;  // [n_aug] padding rows
  int64_t n_aug;
  int* info;
  double* D_pose;      // [3 n_pose]
  double lambda;
  const double* lam_dev;
};

struct SchurArgs {
  const int4* items;              // [n_items] {f1b, chunk, list begin, list end}
  const int4* groups;             // [n_groups] per tile {f1b, chunk, first item, end item}
  const int4* item_lm;            // item landmark lists: {landmark, first frame, last frame, slot offset}
  const int32_t* frame_win_hi;    // [n_pose]
  const void* ug_slot;            // [n_slot][UG_STRIDE] real: U (6) | g_pose (3) (dense slots)
  const void* w_slot;             // [n_slot][W_STRIDE] real: W (dense landmark x frame slots)
  const double* lm_aux;           // [n_lm][8]
  const int32_t* frame_pos;       // [n_pose] system row of the frame's pan (-1: fixed)
  void* part;                     // [n_items][SCHUR_F1][9][64] split partials (record precision)
  double* part_diag;              // [n_items][SCHUR_F1][12] chunk-0 splits: U | g_pose | sum W V~^-1 g
  double* S;                      // [ld][ld] lower, row-major
  double* b;                      // [n_sys]
  double* g_pose;                 // [n_sys]
  double* dU;                     // [n_sys] diag of U (for Marquardt scaling)
  int64_t ld;
  int n_pose;
  const int* skip_if;             // nullptr, or: exit at once when *skip_if != 0 (device-driven LM)
  const void* ug_slot1;           // sel != nullptr: read slot *sel (1 = these buffers), see LinArgs
  const void* w_slot1;
  const int* sel;
  FusedPrep prep;                 // single-GPU: the prepare's augmented row and damping (pad != nullptr)
};

struct BacksubArgs {
  const int32_t* lm_seg_begin;
  const int32_t* seg_frame;
  const void* w_slot;    // [n_slot][W_STRIDE] real: W
  const int4* lm_meta;   // [n_lm] {first frame, last frame, slot offset, 0}
  const double* lm_out;
  const double* lm_aux;
  const double* D_ray;
  const double* dpose;   // [n_aug] system order
  const int32_t* frame_pos;
  const double* rays;    // [2 n_lm]
  double* rays_trial;    // [2 n_lm]
  double* lm_red;        // [n_lm][4]: pred, |d|^2, |x|^2, |g|max
  int n_lm;
  int n_fixed;
  double lambda;
  const double* lam_dev;  // nullptr, or lambda read from device memory (device-driven LM)
  const void* w_slot1;    // sel != nullptr: read slot *sel (1 = these buffers), see LinArgs
  const double* lm_out1;
  const int* sel;
  // device-driven LM: the state is double-buffered like the linearisation slots -- with sel != nullptr the
  // current state is (rays, ptz) when ((*sel) ^ state_xor) is even, else (rays_trial, ptz_trial), and the trial
  // goes to the other pair, so an accepted trial needs no copy (the decision's slot flip commits it)
  int state_xor;
};

// device-driven Levenberg-Marquardt state (ptzba_lm_*): parameters, running state, last decision
struct LMParams {
  double ftol, xtol, gtol, lambda0, min_lambda, max_lambda;
  double huber_curvature, curvature_switch;  // see ptzba_lm_opts
  int max_iter, max_retries, gauss_newton;
  // how the curvature switch reaches the linearisations: 0 (single GPU) the trial's K1 linearises with hc_trial,
  // chosen before it from the trial's predicted reduction (k_reduce_cols curvature mode); 1 (ranks: the predicted
  // reduction is a sum over ranks only after K1) the decision switches and the next build re-linearises (relin)
  int relin_mode;
};
struct LMDev {
  LMParams p;
  double cost, initial_cost, lam, nu, last_actual, last_rho;
  double hc;        // huber curvature weight of the current linearisation (1 until the switch)
  double hc_trial;  // relin_mode 0: the weight the trial's linearisation used (the current one's if accepted)
  int it, nfev, trials, retries, status, done, accepted;
  int relin;  // the decision switched the curvature: the next build re-linearises the current point first
  int seq;  // host ring record: written last (after a system-scope fence) = trial index + 1
  int cur;  // current linearisation slot (flips on an accepted trial: the trial linearised into the other)
};
void launch_lm_init(LMDev* st, const double* scal, const LMParams& p, int cur0, hipStream_t s);
void launch_lm_decide(LMDev* st, const double* scal, const double* loc, const int* info, LMDev* rec, int seq,
                      hipStream_t s, int info_in_loc = 0);
void launch_lm_commit(const LMDev* st, double* ptz, const double* ptz_trial, int n3, double* rays,
                      const double* rays_trial, int64_t n2, hipStream_t s);
// the decision fused into the trial-cost reduction (single GPU: no exchange between them): the reduction's last
// workgroup applies k_lm_decide's rules to the sums it has just formed
struct DecideArgs {
  LMDev* st;
  const double* loc;
  const int* info;
  LMDev* rec;
  int seq;
  int curv;  // 1: not a decision -- the last workgroup sets st->hc_trial from the reduced predicted reduction
};

template <typename real>
void launch_tables(const double* ptz, const double* rays, int n_pose, int n_lm, void* ft64, void* rt64, void* ft, void* rt,
                   const int* run_if, hipStream_t st, double* zero = nullptr, int n_zero = 0);  // zero[0, n_zero) = 0
template <typename real>
// ev0 / ev1 != nullptr: the launch carries the event pair itself (hipExtLaunchKernelGGL: the kernel packet's own
// start / end timestamps, no marker packets around it)
void launch_linearize(const LinArgs& a, int loss, hipStream_t st, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
template <typename real>
void launch_schur(const SchurArgs& a, int n_items, int n_groups, int n_fixed, hipStream_t st);
// scratch: RED_SCRATCH doubles (partials + counter), zero-initialised once, reused across calls
constexpr int RED_SCRATCH = 64 * 8 + 2;
// scal[8] | loc[8] | info -> one packed device block (read back with a single copy)
void launch_pack_scalars(const double* scal, const double* loc, const int* info, double* host_dev, hipStream_t st);
// src1 / sel / sel_xor: with sel != nullptr the first source is src when ((*sel) ^ sel_xor) == 0, else src1
void launch_reduce_cols(const double* src, int64_t n, int stride, int nk, int maxmask, double* out, double* scratch,
                        hipStream_t st, const double* src2 = nullptr, int stride2 = 0, int nk2 = 0,
                        double* out2 = nullptr, const double* src1 = nullptr, const int* sel = nullptr,
                        int sel_xor = 0, const DecideArgs* decide = nullptr);
// build prologue (zero pattern tiles + b|g|dU, landmark damping) in one launch
void launch_build_prologue(double* S, int64_t ld, const int2* zt, int n_tiles, double* vec, int64_t n_vec,
                           const double* lm_out, const int32_t* lm_seg_begin, double* D_ray, double* lm_aux, int n_lm,
                           double lambda, const double* lam_dev, const int* skip_if, hipStream_t st,
                           const double* lm_out1 = nullptr, const int* sel = nullptr, const FusedPrep& fp = FusedPrep{});
// trial state (ray back-substitution + pose trial + the trial's frame / ray tables) in one launch
// fmask (part-owned solve, else nullptr): per frame bit 0 = this rank's solve updates the pose, bit 1 = the
// frame's terms count in this rank's pose partials (each frame is counted by exactly one rank)
template <typename real>
void launch_trial(const BacksubArgs& a, const double* ptz, const double* g_pose, const double* D_pose, double* ptz_trial,
                  double* out4, int n_pose, void* ft64, void* rt64, void* ft, void* rt, hipStream_t st,
                  const uint8_t* fmask = nullptr, const int* info = nullptr);
template <typename real>
void launch_residual(const int32_t* rec_seg, const int32_t* seg_frame, const int32_t* seg_lm, const double2* seg_base,
                     const void* rec_xy, const int64_t* perm, const void* ft64, const void* rt64, double u, double v,
                     int64_t n_rec, double* r_out, hipStream_t st);

// dense-tile SPD solve of the reduced camera system (chol_kernels.hip)
// A: [ld][ld] row-major fp64, lower triangle of S in system order (n = n_aug rows incl. padding),
// ld = roundup(n + 1, CHOL_NB).  prepare: row n <- b^T (augmented), A[n][n] huge, identity on padding
// rows.  cholesky: one launch per elimination level over host-built int4 tasks
// {type, i, j, packed update panels}.  backsolve: x = S^-1 b into xout, one workgroup per chain.
constexpr int CHOL_NB = 32;
void launch_chol_prepare(double* A, int64_t ld, int n, double* b, const uint8_t* pad, int* info, hipStream_t st);
// the same plus the Marquardt damping of the pose rows (k_pose_damp's work) in one launch
void launch_chol_prepare_damped(double* A, int64_t ld, int n, double* b, const uint8_t* pad, int* info,
                                const double* dU, double* D_pose, const int32_t* frame_pos, int n_pose, int n_fixed,
                                double lambda, const double* lam_dev, hipStream_t st, const uint8_t* row_phase = nullptr,
                                int phase = 0);  // part-owned solve: rows of one phase only (chol_kernels.hip)
// sgn != nullptr: signed factor L Sigma L^T of an indefinite matrix (sigma per row into sgn[ld])
// tasks_host (optional, the host copy of `tasks`): levels of <= CHOL_KT tasks pass them by value
constexpr int CHOL_KT = 240;  // 3.75 KB of kernel arguments
void launch_cholesky(double* A, int64_t ld, const int4* tasks, const int* task_off_host, int n_launch, double* Ldiag,
                     int* info, hipStream_t st, double* sgn = nullptr, const int4* tasks_host = nullptr,
                     double* Minv = nullptr,  // Minv: target of type-2 tasks (diagonal tile inverses)
                     int first_level = 0,     // levels [first_level, n_launch)
                     bool delayed = false);   // tasks carry a second pair of update panels (api.hip make_plan)

// la_tasks: lookahead back substitution's [lookahead tile per position | task offsets per (chain, helper) |
// tasks q << 16 | tile], built by the host plan (api.hip make_plan)
constexpr int BS_HELPERS = 7;
void launch_chol_backsolve(const double* L, int64_t ld, int n, int n_chain, int n_pos, const int* chain_off,
                           const int* chain_cols, const int* upd_off, const int* upd_tiles, int n_upd,
                           const int* la_tasks, int n_tasks, const double* Ldiag, double* Minv, double* xout,
                           const int* lo_off, const int* lo_tiles, hipStream_t st,
                           const int* tinv_list = nullptr, int n_tinv = 0);  // tinv_list: see k_tile_inv_list
// blocked right-looking back substitution (large systems): one launch per step of api.hip make_bs_steps'
// schedule (step_off_host: task offsets), r: scratch [ld]; BSB_P chain columns per block
constexpr int BSB_P = 4;
void launch_chol_backsolve_blk(const double* L, int64_t ld, int n, const int4* tasks, const int* step_off_host,
                               int n_steps, const double* Ldiag, double* Minv, double* r, double* xout,
                               hipStream_t st, const int* tinv_list, int n_tinv);
// persistent form: every step's tasks in ONE launch (task order = step order), hand-offs through per-column update
// counters (write-through r stores, relaxed counter adds; expect: per task the counts to wait for, tot: per column
// the updates one solve applies, epoch: the number of earlier launches on these counters); err: set to 1 when a
// wait gives up (a bounded spin: a plan error must not hang the GPU)
void launch_chol_backsolve_pst(const double* L, int64_t ld, int n, const int4* tasks, const int4* expect, int n_tasks,
                               const double* Ldiag, double* Minv, double* r, double* xout, unsigned* cnt,
                               const int* tot, uint32_t epoch, int* err, hipStream_t st, const int* tinv_list,
                               int n_tinv);
// largest ld the back substitution keeps in LDS (left-looking form: x [ld] doubles + 4.4 KiB)
constexpr int64_t CHOL_MAX_LD = 18944;
// zero the factor pattern's tiles and the b | g_pose | dU vectors before a build (replaces a memset of
// the whole ld x ld region: entries outside the pattern are never written)
void launch_zero_tiles(double* S, int64_t ld, const int2* zt, int n_tiles, double* vec, int64_t n_vec, hipStream_t st);
// packed exchange of the Schur-written tiles + b | g_pose | dU (vec = b, contiguous 3 ld doubles)
void launch_pack_exchange(double* S, int64_t ld, const int2* xt, int n_tiles, double* vec, double* buf, int unpack,
                          hipStream_t st);
// part-owned exchanges: tile list + up to three ranges of the b | g_pose | dU vectors; mode 0 pack, 1 unpack,
// 2 pack zeros
struct VecRanges {
  int64_t off[3], count[3];
  int n;
};
void launch_pack_region(double* S, int64_t ld, const int2* xt, int n_tiles, double* vec, const VecRanges& vr,
                        double* buf, int mode, hipStream_t st);
// task word w: bits 0-13 update panel p1 + 1, bits 14-27 p2 + 1 (0 = none), bits 28/29: p1/p2 also update T
inline int chol_pack_updates(int p1, int p2, int tmask) { return (p1 + 1) | ((p2 + 1) << 14) | (tmask << 28); }
// task word x: type (2 bits) + the second pair of update panels of a delayed-trailing plan (api.hip make_plan)
inline int chol_pack_type(int type, int p3, int p4, int tmask34) {
  return (int)((unsigned)type | ((unsigned)(p3 + 1) << 2) | ((unsigned)(p4 + 1) << 16) | ((unsigned)tmask34 << 30));
}

// camera batch kernels (camera_kernels.hip)
void launch_ray_to_image(int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                         const double* th, const double* ph, double* x, double* y, hipStream_t st);
void launch_image_to_ray(int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                         const double* x, const double* y, double* th, double* ph, hipStream_t st);
void launch_project_rays(int64_t n, double u, double v, double f, double pan, double tilt, const double* disp6,
                         const double* rays, double* xy, hipStream_t st);
void launch_back_project(int64_t n, double u, double v, double f, double pan, double tilt, const double* disp6,
                         const double* xy, double* rays, hipStream_t st);
void launch_h_jacobian(int64_t n, double u, double v, double f, double pan, double tilt, const double* disp6,
                       const double* rays, double* H, hipStream_t st);

// setup_kernels.hip: the GPU front of set_problem (large problems; n < 2^31, n_lm * n_pose < 2^32).  Each returns 0 or
// -1 with fail() set.  setup_sort_runs: order / key_sorted = records in (landmark, frame, index) order, rec_seg = the
// inclusive scan of the run starts, *n_seg = the number of segments (synchronises the stream).
int setup_sort_runs(hipStream_t st, int64_t n, int n_pose, int n_lm, const int32_t* frame, const int32_t* lm,
                    uint32_t* order, uint32_t* key_sorted, int32_t* rec_seg, int64_t* n_seg);
// rec_seg -> segment ids; seg_frame / seg_lm [n_seg], seg_rec_begin [n_seg + 1], lm_first [n_lm] (landmarks with
// segments only)
int setup_fill_segments(hipStream_t st, int64_t n, int n_pose, int64_t n_seg, const uint32_t* key_sorted, int32_t* rec_seg,
                        int32_t* seg_frame, int32_t* seg_lm, int64_t* seg_rec_begin, int32_t* lm_first);
// seg_base [2 n_seg] fp64, rec_xy [2 n] / rec_w [n] (w == nullptr: none) in the record precision, rec_key [n], perm [n]
template <typename real>
int setup_records(hipStream_t st, int64_t n, int64_t n_seg, const uint32_t* order, const int32_t* rec_seg,
                  const int32_t* seg_lm, const int64_t* seg_rec_begin, const int32_t* lm_first, const double* xy,
                  const double* w, double* seg_base, real* rec_xy, real* rec_w, uint8_t* rec_key, int64_t* perm);

}  // namespace ptzba
